"""Attribution of the device-RNG incomplete count's issue gap: the bench
`incomplete` shape (64 prop-SWOR shards of 15625 + 15625 scores, B = 1e6 device-drawn pairs
per shard) counted by one build of libtuplewise.so — the product, or an attribution build of
k_count_rng_img's inner loop (csrc/imagecount.hip TW_RNG_IMG_VARIANT, `make ab-rngimg`):
    1 Philox + Lemire only, 2 + LDS image reads and the compare, 3 = 2 at conflict-free LDS
    addresses, 4 the product with four per-draw Lemire branches (the round-4 loop).
Prints ms per launch (HIP events over 20 launches after 5 warm), pairs/s, and a checksum of the
counts (the product and variant 4 must agree bit for bit; 1-3 count something else).
    TW_LIB_PATH=tools/variants/libtuplewise_rngimg2.so python tools/ab_rng_img.py [reps]"""
import os
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from tuplewise import _lib as L
from tuplewise.device import HipOps, prop_swor_layout

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(3)
n, N, B = 1_000_000, 64, 1_000_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
x_off, z_off, _ = prop_swor_layout(n, n, N)
xo, zo = L.to_device(x_off), L.to_device(z_off)
k = n // N
ops = HipOps()


def launch(seed):
    return ops.count_rng(X, xo, Z, zo, N, B, seed, 0, L.TW_F64, L.TW_PRED_GT, max_nx=k, max_nz=k)


for i in range(5):
    launch(100 + i)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
outs = []
e0.record()
for i in range(reps):
    outs.append(launch(1000 + i))
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
chk = int(sum(int(o.sum()) for o in outs))
lib = os.environ.get("TW_LIB_PATH", "product")
print(f"{pathlib.Path(lib).name}: {ms:.4f} ms/launch, {N * B / ms * 1e3:.4e} pairs/s, "
      f"checksum {chk}", flush=True)
