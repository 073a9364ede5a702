"""The bench headline's timed K = 20 UnN_many call in its own sequence (a 5-step call, a sync,
the clones of X and Z, then the timed call) against the same call back to back: host wall time
per call and the GPU span (an event recorded at t0 and after the call).  Run on the GPU box:
    python tools/headline_call_probe.py"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

gen = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X.clone(), Z.clone(), 64, algo="pairs")
S.UnN_many(range(40_000, 40_020))
for _ in range(20):
    S.UnN_many(range(20_000, 20_005))
torch.cuda.synchronize()


def timed(pre):
    res = []
    for rep in range(8):
        pre()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        S.UnN_many(range(5 + 20 * rep, 25 + 20 * rep))
        e1.record()
        torch.cuda.synchronize()
        res.append(((time.perf_counter() - t0) * 1e3, e0.elapsed_time(e1)))
    a = np.array(res)
    return f"wall {np.median(a[:, 0]):.3f} ms, GPU span {np.median(a[:, 1]):.3f} ms"


def five():
    S.UnN_many(range(5))


def five_clone():
    S.UnN_many(range(5))
    S.X.clone(), S.Z.clone()


print("back to back:", timed(lambda: None), flush=True)
# bench.py's live timing: its EventPool wrappers around the chain launches
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
ops = S.ops
plain = (ops.count_chain, ops.chain_emit, ops.rank_images_query)
chain_ms, emit_ms, rank_ms = (bench.EventPool(torch, 64), bench.EventPool(torch, 64),
                              bench.EventPool(torch, 8))
ops.count_chain = chain_ms.wrap(ops.count_chain, weight=lambda *a, **kw: a[5])
ops.chain_emit = emit_ms.wrap(ops.chain_emit, weight=lambda *a, **kw: len(a[8]))
ops.rank_images_query = rank_ms.wrap(ops.rank_images_query)


def clear():
    for p in (chain_ms, emit_ms, rank_ms):
        p.clear()


print("with bench's event wrappers:", timed(clear), flush=True)
ops.count_chain, ops.chain_emit, ops.rank_images_query = plain
print("after a 5-step call:", timed(five), flush=True)
# a large Python heap (bench.py's process holds many objects): the cyclic collector's passes
import gc  # noqa: E402
heap = [[i] for i in range(2_000_000)]
print("large heap:", timed(lambda: None), flush=True)
gc.disable()
print("large heap, gc disabled:", timed(lambda: None), flush=True)
gc.enable()
gc.collect()
print("large heap, gc.collect() first:", timed(gc.collect), flush=True)
print("after a 5-step call and the clones:", timed(five_clone), flush=True)
print("back to back:", timed(lambda: None), flush=True)
