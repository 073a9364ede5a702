"""Sweep the float32-image incomplete counts (csrc/imagecount.hip) against the rank-code path
at the bench shape (64 shards of 15625 x 15625): replay (1e6 int32 index pairs per shard,
tw_count_pairs_idx32_ws) and device RNG (1e6 draws per shard, tw_count_pairs_rng_ws).
Whole-call times from HIP events; every configuration's counts must equal the reference
configuration's (rank codes)."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _engine as E, _lib as L  # noqa: E402
from tuplewise.device import HipOps  # noqa: E402

k, N, B = 15625, 64, 1_000_000
g = torch.Generator(device="cuda").manual_seed(1000)
X = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g)
base = (torch.arange(N, device="cuda", dtype=torch.int64) * k).repeat_interleave(B)
ix = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
iz = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
del base
off = L.to_device(np.arange(N + 1, dtype=np.int64) * k)
po = np.arange(N + 1, dtype=np.int64) * B
pod = L.to_device(po)
work = L.empty((int(L.lib().tw_count_pairs_rng_work_bytes(N, k, k, L.TW_F64, L.TW_PRED_GT)),),
               torch.uint8)
ops = HipOps()


def replay():
    return E.count_indexed_ranked_dev(X, off, Z, off, k, k, L.TW_F64, ix, iz, po, L.TW_PRED_GT,
                                      pod, work)


def rng():
    return ops.count_rng(X, off, Z, off, N, B, 0xABCDEF, 0, L.TW_F64, L.TW_PRED_GT, max_nx=k,
                         max_nz=k)


def timed(fn, reps=30):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        out = fn()
        e1.record()
    torch.cuda.synchronize()
    return out, float(np.median([a.elapsed_time(b) for a, b in ev]))


for name, fn in (("replay", replay), ("rng", rng)):
    L.call("tw_count_rng_set_codes", 2)
    ref, ms = timed(fn)
    print(json.dumps({"path": name, "codes": 2, "ms": ms,
                      "GBps_8B": 8 * N * B / (ms * 1e-3) / 1e9}), flush=True)
    L.call("tw_count_rng_set_codes", 3)
    for parts in (0, 4):
        for u in ((1, 2, 4, 9, 10, 12) if name == "replay" else (1,)):
            L.call("tw_count_img_set_plan", parts, u)
            out, ms = timed(fn)
            print(json.dumps({"path": name, "codes": 3, "parts": parts, "u": u, "ms": ms,
                              "GBps_8B": 8 * N * B / (ms * 1e-3) / 1e9,
                              "same": bool(torch.equal(out, ref))}), flush=True)
    L.call("tw_count_img_set_plan", 0, 9)
