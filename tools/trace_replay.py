"""Replay-mode learning_process at the C4 shape (as bench sgd_replay_steps_per_s), 5 calls, for
a rocprofv3 --kernel-trace run: the device timeline of the segments (kernels, gaps).
Argument "eager": graphs=False."""
import logging
import pathlib
import sys

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
eager = "eager" in sys.argv[1:]  # graphs=False: the segment kernels launched eagerly
for _ in range(6):
    lr.learning_process(X, Z, p, graphs=not eager)
    torch.cuda.synchronize()
print("done", flush=True)
