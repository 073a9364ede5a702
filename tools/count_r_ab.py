"""The headline count launch (K = 20 steps x 64 bags of 15625 x 15625, and K = 4) under x-images
per lane R = 8 / 16 and a few z-chunk lengths (tw_count_chain_set_plan), interleaved over 7
rounds; median ms.  Run on the GPU box:  python tools/count_r_ab.py"""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import HipOps, prop_swor_layout

ops = HipOps()
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
x_off, z_off, _ = prop_swor_layout(n, n, N)
xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
k = n // N
for K in (20, 4):
    xb = torch.randint(0, 2 * n, (K, n), device="cuda", generator=gen).float()
    zb = -torch.randint(0, 2 * n, (K, n), device="cuda", generator=gen).float()
    out = torch.empty((K, N), dtype=torch.int64, device="cuda")
    plans = [(0, 0), (8, 3912), (16, 3912), (16, 7816), (16, 1960), (8, 7816)]
    ts = {p: [] for p in plans}
    ref = None
    for rnd in range(7):
        for p in plans:
            L.call("tw_count_chain_set_plan", *p)
            ops.count_chain(xb, xo, zb, zo, N, K, n, n, k, k, False, out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.count_chain(xb, xo, zb, zo, N, K, n, n, k, k, False, out)
            e1.record()
            torch.cuda.synchronize()
            ref = out.clone() if ref is None else ref
            assert torch.equal(out, ref)
            ts[p].append(e0.elapsed_time(e1))
    L.call("tw_count_chain_set_plan", 0, 0)
    print(f"K={K}: " + ", ".join(f"R={p[0] or 'auto'} zc={p[1] or 'auto'} {np.median(ts[p]):.4f} ms"
                                 for p in plans), flush=True)
