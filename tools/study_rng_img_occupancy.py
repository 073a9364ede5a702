"""Occupancy study of the device-RNG incomplete count (k_count_rng_img, csrc/imagecount.hip;
VERDICT r03 item 2): the same kernel, the same B = 1e6 device-drawn pairs per shard and 64
shards, on shards of 15625 (the bench: 125 KB of float32 images per block, ONE block = 16
waves per CU), 7812 and 3906 scores per side (62.5 / 31 KB: two and four blocks per CU) — the
per-pair work is identical (Philox draws, two range maps, two LDS image reads, a compare), so
a faster per-pair rate on smaller shards measures what occupancy the kernel is starved of.
Rates are per launch (HIP events around back-to-back launches) against the measured int32
lane-op rate (53 lane-ops per pair, bench INC_LANE_OPS)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import ShardedSample  # noqa: E402

torch.cuda.set_device(0)
B, N = 1_000_000, 64
for k in (15625, 7812, 3906):
    n = k * N
    g = torch.Generator(device="cuda").manual_seed(5)
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    S = ShardedSample(X, Z, N, algo="pairs")
    for _ in range(5):
        S._count_rng(B, 11)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 30
    a.record()
    for r in range(reps):
        S._count_rng(B, 11 + r)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    pairs = B * N
    print(f"shard {k:6d} x {k:6d}: {ms * 1e3:7.1f} us/launch, {pairs / (ms * 1e-3):.3e} pairs/s, "
          f"{bench.INC_LANE_OPS * pairs / (ms * 1e-3) / bench.INT_LANE_OPS_MEASURED:.3f} of the "
          f"int32 lane-op rate, LDS images {8 * k / 1024:.1f} KB per block", flush=True)
