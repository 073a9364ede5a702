"""Where the replay-mode learning loop's host time goes at the C4 shape (bench
sgd_replay_steps_per_s: N = 100, B = 100, reshuffle every 25 steps, no evaluation): steps/s,
then cProfile of one run, top entries by internal time (GPU box)."""
import cProfile
import logging
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tuplewise.learning as lr  # noqa: E402

rng = np.random.RandomState(3)
X = np.hstack([rng.normal(size=(9117, 9)), np.ones((9117, 1))])
Z = np.hstack([rng.normal(0.5, 1, size=(702, 9)), np.ones((702, 1))])
p = {"n_it": 2000, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": 25, "reg": 0.05,
     "learning_rate": 0.01, "eval_mod": 10 ** 9, "w_init": rng.normal(size=(10, 1)),
     "test_X": X[:10], "test_Z": Z[:10], "train_mon_pairs": [(0, 0)], "train_X": X,
     "train_Z": Z}
logging.disable(logging.CRITICAL)
np.random.seed(0)
lr.learning_process(X, Z, dict(p, n_it=50))
torch.cuda.synchronize()
t0 = time.perf_counter()
lr.learning_process(X, Z, p)
torch.cuda.synchronize()
print(f"{2000 / (time.perf_counter() - t0):.0f} steps/s", flush=True)
pr = cProfile.Profile()
pr.enable()
lr.learning_process(X, Z, p)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).strip_dirs().sort_stats("tottime").print_stats(25)
