"""Probe a collective-free strong-scaling step on ONE GPU: what rank r of G does per step if
every rank keeps the WHOLE sample's rank-image records (replicated, 16 MB at 1e6 + 1e6) — the
one-launch step counts only the rank's 64/G shards of the global layout and repartitions the
whole record arrays with the global keys (no all-to-all).  Reports ms/step per G against the
ideal 1/G of the one-GPU step.  Run on the GPU box:
    python tools/replicated_probe.py"""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch

import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import HipOps, prop_swor_layout

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N, K = 1_000_000, 64, 200
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
ops = HipOps()
xr, zr = ops.rank_images(X, Z, L.TW_F64)
x_off, z_off, _ = prop_swor_layout(n, n, N)
max_nx, max_nz = int(max(x_off[1:] - x_off[:-1])), int(max(z_off[1:] - z_off[:-1]))


def run(G, r, steps, mode="step"):
    s = N // G
    xo = torch.tensor(x_off[r * s:(r + 1) * s + 1], device="cuda")
    zo = torch.tensor(z_off[r * s:(r + 1) * s + 1], device="cuda")
    a, b = xr.clone(), zr.clone()
    outs = torch.zeros((steps + 1, s), dtype=torch.int64, device="cuda")
    bufs = [(torch.empty_like(a), torch.empty_like(b)) for _ in range(2)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        an, bn = bufs[i & 1]
        if mode == "count":  # the rank's counts alone
            ops.count_rank_step(a, xo, b, zo, s, max_nx, max_nz, outs[i], None, 0, None, 0,
                                None)
            continue
        if mode == "perm":  # the whole-array repartition alone
            ops.count_rank_step(a, xo, b, zo, 0, max_nx, max_nz, outs[i], an, 2 * i + 2, bn,
                                2 * i + 3, None)
        else:
            ops.count_rank_step(a, xo, b, zo, s, max_nx, max_nz, outs[i], an, 2 * i + 2, bn,
                                2 * i + 3, outs[i + 1])
        bufs[i & 1] = (a, b)
        a, b = an, bn
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, outs[:steps]


base = None
for G in (1, 2, 4, 8):
    run(G, 0, 20)
    ms, _ = run(G, 0, K)
    ms_last, _ = run(G, G - 1, K)
    if base is None:
        base = ms
    print(f"  G={G} parts: counts alone {run(G, 0, K, 'count')[0]:.4f} ms, whole-array "
          f"repartition alone {run(G, 0, K, 'perm')[0]:.4f} ms", flush=True)
    print(f"G={G}: rank 0 {ms:.4f} ms/step, rank {G - 1} {ms_last:.4f} ms/step; ideal "
          f"{base / G:.4f}; efficiency {base / G / max(ms, ms_last):.3f}", flush=True)
# the counts of the G slices are the one-GPU counts (same global permutation chain)
_, full = run(1, 0, 8)
parts = torch.cat([run(4, r, 8)[1] for r in range(4)], dim=1)
print("slices == one GPU:", bool(torch.equal(full, parts)), flush=True)

# weak form (1e6/class and 64 shards PER rank): the replicated chain permutes G x the records
for G in (2, 4, 8):
    Xw = torch.randn(G * n, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Zw = torch.randn(G * n, dtype=torch.float64, device="cuda", generator=g)
    xr, zr = ops.rank_images(Xw, Zw, L.TW_F64)
    x_off, z_off, _ = prop_swor_layout(G * n, G * n, G * N)
    N_saved, N = N, G * N
    run(G, 0, 20)
    ms, _ = run(G, 0, K)
    N = N_saved
    print(f"weak G={G}: rank 0 {ms:.4f} ms/step (one GPU, 64 shards, own records: "
          f"{base:.4f})", flush=True)

# plan sweep at the strong-scaling shapes: spare-block placement x z-chunk length
x_off, z_off, _ = prop_swor_layout(n, n, N)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
xr, zr = ops.rank_images(X, Z, L.TW_F64)
for G in (8, 4, 2, 1):
    for front in (0, 1):
        for R, zc in ((0, 0), (8, 512), (8, 1024), (16, 512), (16, 1024)):
            L.call("tw_count_rank_set_next", front)
            L.call("tw_count_rank_set_plan", R, zc)
            run(G, 0, 20)
            ms = run(G, 0, K)[0]
            mc = run(G, 0, K, "count")[0]
            print(f"sweep G={G} front={front} R={R} zc={zc}: step {ms:.4f} ms (counts alone "
                  f"{mc:.4f})", flush=True)
L.call("tw_count_rank_set_next", 0)
L.call("tw_count_rank_set_plan", 0, 0)
