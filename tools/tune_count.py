"""Sweep tw_count_pairs launch plans on the bench workload (n=1e6/class, N=64)."""
import sys, pathlib, time
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np, torch
import tuplewise
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

n, N = 1_000_000, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N)
S.repartition(1)
ref = None
pairs = N * (n // N) ** 2
for R in (0, 4, 2):
    for zc in (0, 512, 768, 1024, 1536):
        L.call("tw_count_set_plan", R, zc)
        for _ in range(2): c = S.local_counts()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): c = S.local_counts()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        cc = c.cpu().numpy()
        if ref is None: ref = cc
        assert np.array_equal(cc, ref)
        print(f"R={R} zchunk={zc:6d}  {ms:.4f} ms  {pairs/ms/1e-3:.3e} pairs/s  frac={pairs/ms/1e-3/3.93216e13:.3f}", flush=True)
L.call("tw_count_set_plan", 0, 0)
