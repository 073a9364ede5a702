"""Host-side cost of one UnN_many call on the step chains (BASELINE configs[2]'s T = 4 and the
driver's K = 20, n = 1e6/class, N = 64): wall time per call, the time until the counts are read
back (the enqueue), and a cProfile of the calls.  Run on the GPU box:
    python tools/host_profile_unn.py [K]"""
import cProfile
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
gen = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X, Z, 64, algo="pairs")
enq = []
orig = S.values


def values(counts, *a, **kw):
    enq.append(time.perf_counter())
    return orig(counts, *a, **kw)


S.values = values
base = [1000]


def call():
    base[0] += K
    t0 = time.perf_counter()
    S.UnN_many(range(base[0], base[0] + K))
    return t0, time.perf_counter()


for _ in range(5):
    call()
torch.cuda.synchronize()
ts = []
for _ in range(30):
    t0, t1 = call()
    ts.append((t1 - t0, enq[-1] - t0))
w = np.array(ts) * 1e3
print(f"K={K}: wall {np.median(w[:, 0]):.3f} ms/call, enqueue (until the counts are read) "
      f"{np.median(w[:, 1]):.3f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(30):
    call()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
