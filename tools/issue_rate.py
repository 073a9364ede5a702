"""UnN_many at the bench shape for several K: host time to issue the K steps vs total time
(GPU box).  Shows whether the timed loop is GPU-bound."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise.device import ShardedSample  # noqa: E402

n, N = 1_000_000, 64
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
S.UnN_many(range(300))
torch.cuda.synchronize()
import tuplewise.device as D  # noqa: E402
orig = S._run_steps
marks = {}


def run_steps(keys, count_local, fusable):
    t0 = time.perf_counter()
    out = orig(keys, count_local, fusable)
    marks["issued"] = time.perf_counter() - t0
    return out


S._run_steps = run_steps
for K, k0 in ((20, 1000), (50, 1000), (100, 1000), (200, 1000), (100, 3), (100, 103),
              (100, 20000), (20, 3)):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    S.UnN_many(range(k0, k0 + K))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"K={K:4d} keys from {k0:5d}  total {dt / K * 1e3:.4f} ms/step  run_steps(incl. counts copy) "
          f"{marks['issued'] / K * 1e3:.4f} ms/step", flush=True)
