"""Per-call times of the drop-in est.UnNT(X, Z, 64, 4, "prop-SWOR") on host arrays of 1e6 per
class over many consecutive calls (bench drop_in_C3's shape): the warm-up curve of the
pipelined device-shuffle path.  Run on the GPU box:  python tools/dropin_warmup.py [calls]"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise.estimation as est

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
rng = np.random.RandomState(0)
X, Z = rng.normal(0.5, 1, 1_000_000), rng.normal(0, 1, 1_000_000)
np.random.seed(1)
torch.cuda.init()
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    est.UnNT(X, Z, 64, 4, "prop-SWOR")
    ts.append((time.perf_counter() - t0) * 1e3)
print("per-call ms:", " ".join(f"{t:.2f}" for t in ts), flush=True)
for a in range(0, calls, 10):
    print(f"calls {a}-{min(calls, a + 10) - 1}: median {np.median(ts[a:a + 10]):.2f} ms", flush=True)
