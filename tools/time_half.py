"""Complete count with half-ties (TW_PRED_HALF) vs strict at the bench shape, scalar mix on
and off (GPU box)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import ShardedSample  # noqa: E402

n, N = 1_000_000, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
pairs = N * (n // N) ** 2
for tie in ("strict", "half"):
    S = ShardedSample(X, Z, N, algo="pairs", tie_mode=tie)
    S.repartition(1)
    for mix in (1, 0):
        L.call("tw_count_set_scalar_mix", mix)
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
        ops = pairs * (2 if tie == "half" else 1)
        print(f"{tie:6s} mix={mix} {ms:.4f} ms  {pairs / ms / 1e-3:.3e} pairs/s  "
              f"frac={ops / ms / 1e-3 / 3.93216e13:.3f}  sum={int(c.sum())}", flush=True)
L.call("tw_count_set_scalar_mix", 1)
