"""A/B of device.FINAL_BESIDE_COUNT on one GPU: a UnN_many call of K steps at the bench shape
(n = 1e6/class, N = 64, carried images) with the call's final scatters (scores and carried
records) on a side stream beside the last count, against after it; interleaved over 7 rounds,
median ms per call.  Run on the GPU box:  python tools/ab_final_scatter.py [K ...]"""
import pathlib
import statistics
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import tuplewise  # noqa: F401
from tuplewise import device as D
from tuplewise.device import ShardedSample

gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X, Z, N, algo="pairs")
Ks = [int(a) for a in sys.argv[1:]] or [4, 20]
key = [1000]


def call_ms(K, reps=5):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        S.UnN_many(range(key[0], key[0] + K))
        e1.record()
        torch.cuda.synchronize()
        key[0] += K
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


for K in Ks:
    for _ in range(3):
        call_ms(K)  # warm (allocations, clock)
    res = {True: [], False: []}
    vals = {}
    for rnd in range(7):
        for on in ((True, False) if rnd % 2 == 0 else (False, True)):
            D.FINAL_BESIDE_COUNT = on
            res[on].append(call_ms(K))
    D.FINAL_BESIDE_COUNT = True
    a, b = statistics.median(res[True]), statistics.median(res[False])
    print(f"K={K}: final scatters beside the last count {a:.3f} ms/call, after it {b:.3f} "
          f"ms/call ({(b - a) * 1e3:.1f} us saved, {b / a - 1:+.2%})", flush=True)
