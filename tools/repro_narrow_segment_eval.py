"""Regression check (GPU box) for DESIGN.md §4.4e: with the persistent narrow segment kernel on,
a second learning_process call whose evaluation graph is re-captured used to read a wrong
evaluation count (~7e13) from its 5th evaluation on — a count output zeroed by a captured
hipMemsetAsync node whose zeroing did not take effect.  Every entry point now zeroes with a
kernel (tw_common.h tw_zero_async); every line below must print the same values."""
import sys, logging, pathlib, gc
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np, torch
import tuplewise.learning as lr
from tuplewise import _engine as E
g = dict(np.load(pathlib.Path(__file__).resolve().parents[1] / "tests/golden/golden.npz"))
logging.disable(logging.CRITICAL)
def P(n_it=200):
    return {"n_it": n_it, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
            "learning_rate": 0.01, "eval_mod": 25, "w_init": g["learn/w0"],
            "test_X": g["learn/test_X"], "test_Z": g["learn/test_Z"],
            "train_mon_pairs": [tuple(p) for p in g["learn/mon"]],
            "train_X": g["learn/X"], "train_Z": g["learn/Z"]}
print("test shapes", g["learn/test_X"].shape, g["learn/test_Z"].shape, E.pick_algo("auto", g["learn/test_X"].shape[0], g["learn/test_Z"].shape[0], "gt"))
lr.NARROW_SEGMENT = True
lr.DEFER_EVALS = False
def run(tag):
    p = P(); np.random.seed(77)
    lr.learning_process(g["learn/X"], g["learn/Z"], p, rng_mode="replay")
    for k in ("bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        print(tag, k, ["%.4g" % v for v in p[k]][3:6], flush=True)
run("first")
run("second")
orig = E.pick_algo
E.pick_algo = lambda algo, a, b, m: "pairs"
run("second-pairs-count")
E.pick_algo = orig
lr.NARROW_SEGMENT = False
run("nseg-off")
