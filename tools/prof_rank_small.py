"""The ranking of X u Z (tw_rank_images_query, compact images) at BASELINE configs[1]'s size
(1e5 + 1e5 doubles).  Default: 20 calls, for a rocprofv3 --kernel-trace run (per-kernel
durations):
    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/prof_rank_small.py
    python3 tools/kernel_grid_stats.py DIR/.../kernel_trace.csv
`--sweep`: HIP-event time per call for each small-Z plan (tw_rank_set_small: sample size,
z per interval bucket, z per thread), interleaved, images checked equal to the default plan's
(back-to-back rankings: host enqueue bound, so the trace mode is the device-time measure)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import HipOps  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 100_000
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
ops = HipOps()
plan_arg = [a for a in sys.argv if a.startswith("--plan=")]
if plan_arg:  # one small-Z plan for the trace: --plan=SAMPLE,Z_PER_INTERVAL,PER
    L.call("tw_rank_set_small", *[int(v) for v in plan_arg[0][7:].split(",")])
if "--sweep" not in sys.argv:
    for _ in range(20):
        ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)
    torch.cuda.synchronize()
    print("done", flush=True)
    sys.exit(0)
plans = [(s, z, p) for s in (256, 512) for z in (1024, 2048) for p in (4, 8, 16)]
L.call("tw_rank_set_small", 256, 2048, 8)
ref = [r.clone() for r in ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)]
times = {p: [] for p in plans}
for rep in range(5):
    for p in plans:
        L.call("tw_rank_set_small", *p)
        for _ in range(3):
            ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            out = ops.rank_images_query(Z, X, Z, L.TW_F64, compact=True)
        b.record()
        torch.cuda.synchronize()
        times[p].append(a.elapsed_time(b) / 20 * 1e3)
        assert all(torch.equal(u, v) for u, v in zip(out, ref)), p
for p in plans:
    v = sorted(times[p])
    print(f"n={n} sample={p[0]:5d} z/interval={p[1]:5d} per={p[2]:2d}: "
          f"median {v[len(v) // 2]:7.1f} us "
          f"per ranking (min {v[0]:.1f})", flush=True)
