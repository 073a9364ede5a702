"""Time the replay-mode incomplete count (bench.py incomplete_replay) standalone, optionally
with a tuning hook: python tools/time_replay.py [parts]."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import bench  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402

parts = int(sys.argv[1]) if len(sys.argv) > 1 else 0
L.call("tw_count_idx_set_parts", parts)
g = torch.Generator(device="cuda").manual_seed(1000)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g)
r = bench.incomplete_replay(X, Z, 64, 1_000_000)
print(json.dumps({"parts": parts, **r}), flush=True)
