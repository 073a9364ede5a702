"""The end of an UnN_many call on one GPU: the counts' read-back (counts.cpu(): a blocking
copy) against a copy into pinned memory + a spin on an event, per-call wall time at K = 4 and
20 (n = 1e6/class, N = 64, carried images).  Run on the GPU box:  python tools/sync_probe.py"""
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


def run(K, spin, calls=40):
    S = ShardedSample(X.clone(), Z.clone(), 64, algo="pairs")
    orig = S.values
    pinned = {}

    def values(counts, *a, **kw):
        if spin:
            buf = pinned.get(counts.shape)
            if buf is None:
                buf = pinned[counts.shape] = torch.empty(counts.shape, dtype=counts.dtype,
                                                         pin_memory=True)
            buf.copy_(counts, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            while not ev.query():
                pass
            counts = buf
        return orig(counts, *a, **kw)
    S.values = values
    base = [1000]
    ts = []
    for i in range(calls + 5):
        base[0] += K
        t0 = time.perf_counter()
        S.UnN_many(range(base[0], base[0] + K))
        if i >= 5:
            ts.append(time.perf_counter() - t0)
    return np.median(ts) * 1e3


for K in (4, 20):
    for rep in range(2):
        a, b = run(K, False), run(K, True)
        print(f"K={K}: counts.cpu() {a:.3f} ms/call, pinned + event spin {b:.3f} ms/call",
              flush=True)
