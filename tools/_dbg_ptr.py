import sys, logging, pathlib
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
lr.NARROW_SEGMENT = True
lr.DEFER_EVALS = False
outs = []
orig = E.count_launch
def spy(*a, **k):
    o = orig(*a, **k)
    outs.append(o.data_ptr())
    return o
E.count_launch = spy
engines = []
origE = lr.SGDEngine.__init__
def einit(self, *a, **k):
    origE(self, *a, **k)
    engines.append(self)
lr.SGDEngine.__init__ = einit
for call in range(2):
    outs.clear()
    p = P(); np.random.seed(77)
    lr.learning_process(g["learn/X"], g["learn/Z"], p, rng_mode="replay")
    eng = engines[-1]
    bufs = {"w": eng.w, "dw": eng.dw, "grads": eng.grads, "ctl": eng._ctl, "rows_x": eng.rows_x,
            "rows_z": eng.rows_z}
    if eng._slot1 is not None:
        for i, b in enumerate(eng._slot1): bufs[f"slot1_{i}"] = b
    print("call", call, "tr", ["%.4g" % v for v in p["tr_AUC"]][3:6])
    print("  count outs", [hex(x) for x in outs][:6])
    for k, b in bufs.items():
        if b is not None:
            print("  ", k, hex(b.data_ptr()), b.numel() * b.element_size())
    ent = lr._CACHE.dev.get("eval_graph")
    print("  eval res", hex(ent[3][0].data_ptr()))
