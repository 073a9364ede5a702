"""Where the drop-in's time goes at BASELINE configs[0] (est.UnNT(X, Z, 10, 4, "prop-SWOR"),
n = 1000 per class, host arrays): cProfile over 300 calls, top entries by cumulative time
(GPU box)."""
import cProfile
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tuplewise.estimation as est  # noqa: E402

rng = np.random.RandomState(0)
X, Z = rng.normal(0.5, 1, 1000), rng.normal(0, 1, 1000)
np.random.seed(1)
for _ in range(50):
    est.UnNT(X, Z, 10, 4, "prop-SWOR")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(300):
    est.UnNT(X, Z, 10, 4, "prop-SWOR")
print(f"{(time.perf_counter() - t0) / 300 * 1e3:.3f} ms per call", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(300):
    est.UnNT(X, Z, 10, 4, "prop-SWOR")
pr.disable()
pstats.Stats(pr).strip_dirs().sort_stats("cumulative").print_stats(30)
