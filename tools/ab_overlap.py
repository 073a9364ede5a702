"""A/B of device.CHAIN_OVERLAP at the bench's headline shape (n = 1e6/class, N = 64, one GPU):
K-step UnN_many calls with carried images, the emission of chunk j + 1 on a side stream beside
chunk j's count (on) against one chunk of K steps (off), interleaved 10 times; median ms per
call and the estimates (must be equal).  Run on the GPU box:  python tools/ab_overlap.py [K ...]"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise import device as D
from tuplewise.device import ShardedSample

torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
for K in [int(a) for a in sys.argv[1:]] or [20, 100]:
    S = {v: ShardedSample(X.clone(), Z.clone(), N, algo="pairs") for v in (False, True)}
    t = {False: [], True: []}
    est = {False: [], True: []}
    base = 1000
    for rep in range(13):
        for v in (False, True):
            D.CHAIN_OVERLAP = v
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e = S[v].UnN_many(range(base, base + K))
            torch.cuda.synchronize()
            if rep >= 3:
                t[v].append((time.perf_counter() - t0) * 1e3)
                est[v].append(e)
        base += K
    D.CHAIN_OVERLAP = True
    same = est[False] == est[True]
    print(f"K={K}: overlap off {np.median(t[False]):.3f} ms/call, on {np.median(t[True]):.3f} "
          f"ms/call ({np.median(t[False]) / np.median(t[True]):.4f}x); estimates equal: {same}",
          flush=True)
