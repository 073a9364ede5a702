"""The one-process chain emission (tw_chain_emit into step bags) at the bench shape
(n = 1e6/class, N = 64 shards, K steps) over the emission plans (tw_chain_set_emit: elements
per thread, steps per round): median launch time of 30.  Run on the GPU box:
    python tools/emit_sweep_one.py [plans as epr/spr ...]"""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import HipOps

ops = HipOps()
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
xr, zr = ops.rank_images_query(Z, X, Z, L.TW_F64)
k = n // N
M64 = 2 ** 64 - 1
plans = [tuple(int(v) for v in a.split("/")) for a in sys.argv[1:]] or [(0, 0), (4, 1), (8, 1),
                                                                       (8, 2)]
for K in (4, 20):
    x_bag = torch.empty((K, n), dtype=torch.float32, device="cuda")
    z_bag = torch.empty((K, n), dtype=torch.float32, device="cuda")
    cur = torch.empty(K * 2 * (N + 1), dtype=torch.int32, device="cuda")
    xpos = torch.empty(n, dtype=torch.int32, device="cuda")
    zpos = torch.empty(n, dtype=torch.int32, device="cuda")
    kxs = [(2 * i) & M64 for i in range(K)]
    kzs = [(2 * i + 1) & M64 for i in range(K)]
    res = []
    for epr, spr in plans:
        L.call("tw_chain_set_emit", epr, spr)
        ts = []
        for i in range(33):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.chain_emit(xr, zr, False, xpos, zpos, True, 0, 1, kxs, kzs, k, k, N,
                           x_bag=x_bag, z_bag=z_bag, cursors=cur)
            e1.record()
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(e0.elapsed_time(e1))
        res.append(f"{epr}/{spr} {np.median(ts) * 1e3:.1f}")
    L.call("tw_chain_set_emit", 0, 0)
    print(f"one process K={K} ({2 * n} elements): emission us by plan (epr/spr; 0/0 = auto): "
          + ", ".join(res), flush=True)
