"""A/B of k_count_chain's z-chunk rule (plan_chain, csrc/chain.hip) on the shapes it serves:
the headline (64 bags of 15625 x 15625 per step, K = 20 / 32 / 4), the strong problem's
per-rank shapes (64/G bags per step), half ties (K = 20) and C2 (one bag of 1e5 x 1e5).
Rules: "old" (z chunks of 1024, shorter when fewer than 16 items per SIMD) and
"items<T>/min<M>" (as many z chunks as give ~T work items, chunks of >= M images), each forced
through tw_count_chain_set_plan(0, z_chunk), interleaved over 7 rounds; median ms.
Run on the GPU box:  python tools/count_plan_ab.py"""
import math
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


def zchunk(max_nx, max_nz, bags, half, rule):
    R = 8
    if not half:
        s16 = math.ceil(max_nx / 1024) * 1024
        s8 = math.ceil(max_nx / 512) * 512
        R = 8 if s8 < s16 else 16
    tiles = math.ceil(max_nx / (64 * R))
    base = tiles * bags
    if rule == "old":
        zc = 1024
        if base * math.ceil(max_nz / zc) < 16384:
            zc = max(256, math.ceil(max_nz / max(1, 16384 // base)))
    else:
        T, M = rule
        zc = max(M, math.ceil(max_nz / max(1, math.ceil(T / base))))
    zc = min(zc, 1 << 24, max_nz)
    return math.ceil(zc / 8) * 8


RULES = ["old", (153600, 512), (153600, 1024), (76800, 512), (307200, 512)]
shapes = [("headline K=20", 1, 20, False), ("headline K=32", 1, 32, False),
          ("K=4 (T=4)", 1, 4, False), ("half ties K=20", 1, 20, True),
          ("G=2 K=20", 2, 20, False), ("G=4 K=4", 4, 4, False), ("G=4 K=20", 4, 20, False),
          ("G=8 K=4", 8, 4, False), ("G=8 K=20", 8, 20, False), ("C2", 0, 1, False)]
for name, G, K, half in shapes:
    if G == 0:  # C2: one bag of 1e5 x 1e5
        nl, Nl = 100_000, 1
    else:
        nl, Nl = 1_000_000 // G, 64 // G
    x_off, z_off, _ = prop_swor_layout(nl, nl, Nl)
    xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
    k = int(np.diff(x_off).max())
    kz = int(np.diff(z_off).max())
    g = torch.randint(0, 2 * nl, (K, nl), device="cuda", generator=gen).float()
    xb = torch.stack([g, g + 1], dim=-1).contiguous().view(torch.int64) if half else g
    zb = -torch.randint(0, 2 * nl, (K, nl), device="cuda", generator=gen).float()
    out = torch.empty((K, Nl), dtype=torch.int64, device="cuda")
    zcs = [zchunk(k, kz, K * Nl, half, r) for r in RULES]
    ts = {i: [] for i in range(len(RULES))}
    ref = None
    for rnd in range(7):
        for i, zc in enumerate(zcs):
            L.call("tw_count_chain_set_plan", 0, zc)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ops.count_chain(xb, xo, zb, zo, Nl, K, nl, nl, k, kz, half, out)  # warm
            e0.record()
            ops.count_chain(xb, xo, zb, zo, Nl, K, nl, nl, k, kz, half, out)
            e1.record()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref)
            ts[i].append(e0.elapsed_time(e1))
    L.call("tw_count_chain_set_plan", 0, 0)
    print(f"{name} ({K * Nl} bags of {k} x {kz}): " + ", ".join(
        f"{'old' if r == 'old' else f'items{r[0]}/min{r[1]}'} zc={zc} {np.median(ts[i]):.4f}"
        for i, (r, zc) in enumerate(zip(RULES, zcs))), flush=True)
