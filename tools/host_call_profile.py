"""Host time of ShardedSample.UnN_many calls at the bench shape (n = 1e6/class, N = 64, carried
images): the wall clock per call of back-to-back calls (each ends in the counts' read-back)
against the device time between HIP events around the call, and a cProfile of the calls'
host side (top functions by own time).  Run on the GPU box:
    python tools/host_call_profile.py [K]"""
import cProfile
import pathlib
import pstats
import statistics
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X, Z, N, algo="pairs")
for i in range(5):
    S.UnN_many(range(1000 * i, 1000 * i + K))
torch.cuda.synchronize()
walls, devs = [], []
for i in range(50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    S.UnN_many(range(100 * i, 100 * i + K))
    e1.record()
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t0) * 1e3)
    devs.append(e0.elapsed_time(e1))
print(f"K={K}: wall {statistics.median(walls):.3f} ms/call, events {statistics.median(devs):.3f} "
      f"ms/call", flush=True)
pr = cProfile.Profile()
pr.enable()
for i in range(50):
    S.UnN_many(range(100 * i, 100 * i + K))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(20)
