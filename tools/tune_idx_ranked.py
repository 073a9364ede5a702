"""Sweep tw_count_idx_set_parts (blocks per shard of k_count_idx_ranked) at the bench's replay
workload: 64 shards x 15625 scores, 1e6 int64 index pairs per shard; prints ms per call."""
import sys
import pathlib

import numpy as np
import torch

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
from tuplewise import _engine as E, _lib as L  # noqa: E402

shards, k, B = 64, 15625, 1_000_000
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(shards * k, dtype=torch.float64, device="cuda", generator=g)
Z = torch.randn(shards * k, dtype=torch.float64, device="cuda", generator=g)
base = (torch.arange(shards, device="cuda", dtype=torch.int64) * k).repeat_interleave(B)
ix = base + torch.randint(0, k, (shards * B,), device="cuda", generator=g)
iz = base + torch.randint(0, k, (shards * B,), device="cuda", generator=g)
po = np.arange(shards + 1, dtype=np.int64) * B
pod = L.to_device(po)
off = L.to_device(np.arange(shards + 1, dtype=np.int64) * k)
work = L.empty((int(L.lib().tw_count_pairs_rng_work_bytes(shards, k, k, 0, 0)),), torch.uint8)
ref = None
for parts in [0, 2, 4, 8, 12, 16, 24, 32, 64]:
    L.call("tw_count_idx_set_parts", parts)
    for _ in range(3):
        out = E.count_indexed_ranked_dev(X, off, Z, off, k, k, 0, ix, iz, po, 0, pod, work)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for a, b in ev:
        a.record()
        out = E.count_indexed_ranked_dev(X, off, Z, off, k, k, 0, ix, iz, po, 0, pod, work)
        b.record()
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    ref = out.clone() if ref is None else ref
    print(f"parts {parts:3d}: {ms:.4f} ms  {16 * shards * B / ms / 1e6:.0f} GB/s "
          f"same={bool(torch.equal(out, ref))}", flush=True)
L.call("tw_count_idx_set_parts", 0)
