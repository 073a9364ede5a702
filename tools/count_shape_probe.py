"""Production count kernel at shard sizes with and without tile padding (GPU box):
n/class = N * 15625 (bench: 4.9% padded lanes at R=4/8) vs N * 16384 (no padding)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

N = 64
for per in (15625, 16384, 16000, 14336):
    n = N * per
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    S = ShardedSample(X, Z, N, algo="pairs")
    S.repartition(1)
    pairs = N * per * per
    for R in (4, 8):
        for zc in (0, 512):
            L.call("tw_count_set_plan", R, zc)
            for _ in range(3):
                S.local_counts()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                S.local_counts()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f"shard {per}x{per} R={R} zc={zc:4d}  {ms:.4f} ms  "
                  f"frac={pairs / ms / 1e-3 / 3.93216e13:.3f}", flush=True)
L.call("tw_count_set_plan", 0, 0)
