"""Bisect the bench's K=100 UnN_many slowdown (GPU box): same data and settle as bench.py,
then timed K-step runs, repeated."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise.device import ShardedSample  # noqa: E402

torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(1000)
n = 1_000_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X, Z, 64, algo="pairs")
mode = sys.argv[1] if len(sys.argv) > 1 else "settle"
if mode == "settle":
    t_s = time.perf_counter()
    while time.perf_counter() - t_s < 0.2:
        S.UnN_many(range(20_000, 20_005))
S.UnN_many(range(3))
torch.cuda.synchronize()
for K, k0 in ((100, 3), (100, 3), (20, 3), (100, 3), (300, 3)):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    S.UnN_many(range(k0, k0 + K))
    torch.cuda.synchronize()
    print(f"{mode} K={K} {(time.perf_counter() - t0) / K * 1e3:.4f} ms/step", flush=True)
