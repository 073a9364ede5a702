"""Sweep tw_count_pairs launch plans on the bench workload (n=1e6/class, N=64 shards of
15625 x 15625): x-values per lane R, z-chunk length, scalar-unit mix on/off.  GPU box."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch
import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

n, N = 1_000_000, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
S.repartition(1)
ref = None
pairs = N * (n // N) ** 2
MIXES = (1, 0) if len(sys.argv) < 2 else tuple(int(v) for v in sys.argv[1].split(","))
RS = (0, 2, 4, 8) if len(sys.argv) < 3 else tuple(int(v) for v in sys.argv[2].split(","))
ZCS = (0, 256, 512, 1024, 2048, 4096) if len(sys.argv) < 4 else tuple(
    int(v) for v in sys.argv[3].split(","))
for mix in MIXES:
    L.call("tw_count_set_scalar_mix", mix)
    for R in RS:
        for zc in ZCS:
            if mix == 0 and R not in (0, 2):
                continue
            L.call("tw_count_set_plan", R, zc)
            for _ in range(3):
                c = S.local_counts()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                c = S.local_counts()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            cc = c.cpu().numpy()
            if ref is None:
                ref = cc
            assert np.array_equal(cc, ref)
            print(f"mix={mix} R={R} zchunk={zc:5d}  {ms:.4f} ms  {pairs / ms / 1e-3:.3e} pairs/s"
                  f"  frac={pairs / ms / 1e-3 / 3.93216e13:.3f}", flush=True)
L.call("tw_count_set_plan", 0, 0)
L.call("tw_count_set_scalar_mix", 1)
