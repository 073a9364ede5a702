"""UnNB_many (device-RNG incomplete statistic, B = 1e6 pairs per shard, the bench shape) wall
time per call at K = 1, 5, 20, 100 keys: the per-call fixed cost is the intercept of time
against K (GPU box)."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise.device import ShardedSample  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, 64, algo="pairs")
B = 1_000_000
S.UnNB_many(B, 5, range(3))
res = {}
for K in (1, 5, 20, 100, 1, 5, 20, 100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    S.UnNB_many(B, 7, range(1000, 1000 + K))
    torch.cuda.synchronize()
    res.setdefault(K, []).append((time.perf_counter() - t0) * 1e3)
Ks = sorted(res)
ms = [min(res[k]) for k in Ks]
slope, icpt = np.polyfit(Ks, ms, 1)
for k, m in zip(Ks, ms):
    print(f"K {k:4d}: {m:8.3f} ms per call, {m / k:.4f} ms per step")
print(f"fit: {slope:.4f} ms per step + {icpt:.3f} ms per call")
