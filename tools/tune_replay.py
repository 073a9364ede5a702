"""Sweep the replay-mode incomplete count (tw_count_pairs_idx32_ws) over its tuning hooks at
the bench shape (64 shards of 15625 x 15625, 1e6 int32 pairs per shard): rank-code mode
(tw_count_rng_set_codes 1 = equal-depth buckets, 2 = value-range buckets), load variant
(tw_count_idx_set_variant) and blocks per shard (tw_count_idx_set_parts).  Whole-call times
from HIP events; every configuration's counts must equal the default's."""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _engine as E, _lib as L  # noqa: E402

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


def run():
    return E.count_indexed_ranked_dev(X, off, Z, off, k, k, L.TW_F64, ix, iz, po, L.TW_PRED_GT,
                                      pod, work)


def timed(reps=30):
    for _ in range(5):
        run()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        out = run()
        e1.record()
    torch.cuda.synchronize()
    return out, float(np.median([a.elapsed_time(b) for a, b in ev]))


ref, _ = timed(3)
res = []
for codes in (1, 2):
    for var in range(6):
        for parts in (0, 4, 16):
            L.call("tw_count_rng_set_codes", codes)
            L.call("tw_count_idx_set_variant", var)
            L.call("tw_count_idx_set_parts", parts)
            out, ms = timed()
            r = {"codes": codes, "variant": var, "parts": parts, "ms": ms,
                 "GBps_8B": 8 * N * B / (ms * 1e-3) / 1e9, "same": bool(torch.equal(out, ref))}
            res.append(r)
            print(json.dumps(r), flush=True)
L.call("tw_count_rng_set_codes", 1)
L.call("tw_count_idx_set_variant", 0)
L.call("tw_count_idx_set_parts", 0)
best = min(res, key=lambda r: r["ms"])
print("best", json.dumps(best))
