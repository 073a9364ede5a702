"""Sweep the sorted-count chunk cap on the bench workload (n=1e6/class, N=64)."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np, torch
import tuplewise
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

n, N = 1_000_000, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
S.repartition(1)
ref = S.local_counts().cpu().numpy()
S.algo = "sorted"
pairs = N * (n // N) ** 2
for cap in (1024, 2048, 4096, 8192, 16384):
    L.call("tw_count_sorted_set_chunk", cap)
    for _ in range(3): c = S.local_counts()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): c = S.local_counts()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    assert np.array_equal(c.cpu().numpy(), ref)
    print(f"cap={cap:6d}  {ms*1e3:8.1f} us  {pairs/ms/1e-3:.3e} logical pairs/s", flush=True)
