"""The ranking of X u Z (tw_rank_images_query, compact images) at BASELINE configs[1]'s size
(1e5 + 1e5 doubles), 20 calls, for a rocprofv3 --kernel-trace run (per-kernel durations):
    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/prof_rank_small.py
    python3 tools/kernel_grid_stats.py DIR/.../kernel_trace.csv"""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import HipOps  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
ops = HipOps()
for _ in range(20):
    ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)
torch.cuda.synchronize()
print("done", flush=True)
