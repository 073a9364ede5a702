"""Time k_count_rng (device-RNG incomplete count) on the bench workload: 1e6 scores per class,
64 prop-SWOR shards, B pairs per shard.  Run on the GPU box."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
for B in (15625, 1_000_000):
    for _ in range(3):
        S._count_rng(B, 1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        S._count_rng(B, i)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"B={B}: {ms:.4f} ms/launch, {N * B / ms / 1e-3:.3e} pairs/s", flush=True)
