"""Host-side timeline of one UnN_many call (bench shape, K steps): wall-clock offsets at which
each device operation is enqueued and returns, against HIP events around the call, to see how
much of the call's wall time is host work the device waits for.
    python tools/time_unn_host.py [K]"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, 64, algo="pairs")
log = []
t_call = [0.0]


def wrap(name, fn):
    def w(*a, **kw):
        t0 = time.perf_counter()
        out = fn(*a, **kw)
        log.append((name, (t0 - t_call[0]) * 1e6, (time.perf_counter() - t0) * 1e6))
        return out
    return w


for name in ("rank_images_query", "chain_emit", "count_chain", "chain_scatter"):
    setattr(S.ops, name, wrap(name, getattr(S.ops, name)))
S.values = wrap("values (D2H + host mean)", S.values)
for c in range(8):
    S.UnN_many(range(100 * c, 100 * c + K))
torch.cuda.synchronize()
for c in range(3):
    log.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t_call[0] = time.perf_counter()
    e0.record()
    S.UnN_many(range(1000 + 100 * c, 1000 + 100 * c + K))
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_call[0]) * 1e6
    print(f"call {c}: wall {wall:.0f} us, events {e0.elapsed_time(e1) * 1e3:.0f} us")
    for name, at, dur in log:
        print(f"   +{at:8.0f} us  {name:28s} {dur:8.0f} us")
