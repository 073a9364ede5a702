"""The chain emission of ONE rank of G into send buckets (tw_chain_emit with a send buffer) at
the strong problem's per-rank shape (n = 1e6/class in total, 64/G shards per rank), K steps,
over the emission plans (tw_chain_set_emit: elements per thread, steps per round): median
launch time of 30.  Run on the GPU box:  python tools/emit_sweep_ranks.py"""
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
n = 1_000_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
M64 = 2 ** 64 - 1
for G in (8, 4, 2):
    nl, Nl = n // G, 64 // G
    xr, zr = ops.rank_images_query(Z, X[:nl], Z[:nl], L.TW_F64)
    kx = nl // Nl
    kz = 2 * nl // Nl - kx
    for K in (4, 20):
        cap = 2 * nl // G + 2 * nl // (8 * G) + 1024
        send = torch.empty(G * K * (cap + 1), dtype=torch.int64, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        xpos = torch.empty(nl, dtype=torch.int32, device="cuda")
        zpos = torch.empty(nl, dtype=torch.int32, device="cuda")
        kxs = [(2 * k) & M64 for k in range(K)]
        kzs = [(2 * k + 1) & M64 for k in range(K)]
        res = []
        for epr, spr in ((0, 0), (2, 1), (2, 8), (4, 1), (4, 4), (8, 1), (8, 2)):
            L.call("tw_chain_set_emit", epr, spr)
            ts = []
            for i in range(33):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.chain_emit(xr, zr, False, xpos, zpos, True, G - 1, G, kxs, kzs, kx, kz, Nl,
                               send=send, cap=cap, flag=flag)
                e1.record()
                torch.cuda.synchronize()
                if i >= 3:
                    ts.append(e0.elapsed_time(e1))
            res.append(f"{epr}/{spr} {np.median(ts) * 1e3:.1f}")
        L.call("tw_chain_set_emit", 0, 0)
        print(f"G={G} K={K} ({2 * nl} elements): emission us by plan (epr/spr; 0/0 = auto): "
              + ", ".join(res), flush=True)
