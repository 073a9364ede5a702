"""Plan sweep for the single-shard complete count (BASELINE configs[1], n = 1e5/class, 1e10
pairs): x-values per lane R and z-chunk length.  GPU box."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

n = 100_000
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, 1, algo="pairs")
ref = None
for R in (0, 4, 8):
    for zc in (0, 256, 384, 512, 768, 1024, 2048):
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
        v = int(c.sum())
        ref = v if ref is None else ref
        assert v == ref
        print(f"R={R} zchunk={zc:5d}  {ms:.4f} ms  frac={n * n / ms / 1e-3 / 3.93216e13:.3f}",
              flush=True)
L.call("tw_count_set_plan", 0, 0)
