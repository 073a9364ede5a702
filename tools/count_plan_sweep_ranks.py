"""k_count_chain at the per-rank shapes of the strong problem (64/G bags of 15625 x 15625 per
step, K steps): median launch time over the z-chunk lengths (tw_count_chain_set_plan; 0 =
automatic).  Run on the GPU box:  python tools/count_plan_sweep_ranks.py"""
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
for G in (8, 4, 1):
    for K in (4, 20):
        nl, Nl = 1_000_000 // G, 64 // G
        x_off, z_off, _ = prop_swor_layout(nl, nl, Nl)
        xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
        k = nl // Nl
        # integer-valued f32 images (x positive, z negated) as the bags hold them
        xb = torch.randint(0, 2 * nl, (K, nl), device="cuda", generator=gen).float()
        zb = -torch.randint(0, 2 * nl, (K, nl), device="cuda", generator=gen).float()
        out = torch.empty((K, Nl), dtype=torch.int64, device="cuda")
        res, ref = [], None
        for zc in (0, 512, 1024, 2048, 4096):
            L.call("tw_count_chain_set_plan", 0, zc)
            ts = []
            for i in range(13):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.count_chain(xb, xo, zb, zo, Nl, K, nl, nl, k, k, False, out)
                e1.record()
                torch.cuda.synchronize()
                if i >= 3:
                    ts.append(e0.elapsed_time(e1))
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref)
            res.append(f"{zc or 'auto'} {np.median(ts):.4f}")
        L.call("tw_count_chain_set_plan", 0, 0)
        print(f"G={G} K={K} ({K * Nl} bags): count ms by z-chunk: " + ", ".join(res), flush=True)
