"""BASELINE configs[1] (C2: est.Un, n = 1e5/class, one shard): the one-shot count's launch
(k_count_chain on compact rank images) under several chain plans (tw_count_chain_set_plan: R,
z chunk), HIP events around back-to-back launches (device-bound: ~0.29 ms each), alternated;
counts checked equal across plans."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import HipOps  # noqa: E402

torch.cuda.set_device(0)
n = 100_000
g = torch.Generator(device="cuda").manual_seed(7)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
ops = HipOps()
xr, zr = ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)
xo = torch.tensor([0, n], dtype=torch.int64, device="cuda")
out = torch.zeros((1, 1), dtype=torch.int64, device="cuda")
plans = [(0, 0), (16, 600), (16, 256), (16, 384), (8, 256), (8, 512), (8, 1056), (16, 128)]
res, ref = {p: [] for p in plans}, None
for rep in range(5):
    for p in plans:
        L.call("tw_count_chain_set_plan", *p)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(12):
            if i == 2:
                a.record()
            out.zero_()
            ops.count_chain(xr, xo, zr, xo, 1, 1, n, n, n, n, False, out)
        b.record()
        torch.cuda.synchronize()
        res[p].append(a.elapsed_time(b) / 10 * 1e3)
        c = int(out.item())
        ref = c if ref is None else ref
        assert c == ref, (p, c, ref)
L.call("tw_count_chain_set_plan", 0, 0)
for p in plans:
    v = sorted(res[p])
    print(f"R={p[0]:2d} z_chunk={p[1]:5d}: median {v[2]:7.1f} us/launch (incl. a zero fill) "
          f"= {n * n / (v[2] * 1e-6) / 3.93216e13:.3f} of the lane-op peak", flush=True)
