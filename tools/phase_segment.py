"""Per-step phase breakdown of the persistent SGD segment kernel (csrc/sgdseg.hip) at the C5
shape (5e6 x 512 per class, N = 256 shards, B = 100, device RNG): builds
tools/_dbg/libtw_seg.so from csrc/{capi,sgdseg}.hip with -DTW_SEG_TIMING (thread 0 of every
block stamps the 100 MHz wall clock at four points of every step), runs one 25-step segment and
prints, per step, the median / max over blocks of: gradient (w read -> gradients published),
barrier 1 wait, update, and the step period.  (The instrumented build is for this study only.)

    python tools/phase_segment.py build [-DFLAG ...]     (here, CPU)
    python tools/phase_segment.py [n_per_class]          (GPU box)
"""
import ctypes
import pathlib
import subprocess
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "trade-offs-in-distributed-tuplewise-estimation-and-learning_amd" / "csrc"
OUT = ROOT / "tools" / "_dbg" / "libtw_seg.so"

if len(sys.argv) > 1 and sys.argv[1] == "build":
    flags = [a for a in sys.argv[2:] if a.startswith("-D")]
    OUT.parent.mkdir(exist_ok=True)
    objs = []
    for src in ("capi.hip", "sgdseg.hip"):
        o = OUT.parent / ("seg_" + src + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-std=c++17", "-ffp-contract=off", "-DTW_SEG_TIMING"] + flags +
                       ["-c", str(CSRC / src), "-o", str(o)], check=True)
        objs.append(str(o))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    str(OUT)] + objs, check=True)
    sys.exit(0)

import torch  # noqa: E402  (before the dlopen: one HIP runtime)

lib = ctypes.CDLL(str(OUT))
vp, i64, i32, f64, u64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                          ctypes.c_uint64)
lib.tw_sgd_segment.argtypes = [vp, vp, i64, vp, i64, vp, i64, vp, vp, i64, i32, i64, f64, i32,
                               u64, vp, i32, i32, vp, vp, vp, f64, f64, f64, vp, vp]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
if len(sys.argv) > 2:  # prefetch mode: 1 rows (default), 0 indices only
    lib.tw_sgd_segment_set_prefetch(int(sys.argv[2]))
d, N, B, steps = 512, 256, 100, 25
kx = kz = n // N
g = torch.Generator(device="cuda").manual_seed(5)
X = torch.randn((n, d), dtype=torch.float64, device="cuda", generator=g) + 0.1
Z = torch.randn((n, d), dtype=torch.float64, device="cuda", generator=g)
rows_x = torch.randint(0, n, (N, kx), device="cuda", generator=g)
rows_z = torch.randint(0, n, (N, kz), device="cuda", generator=g)
w = torch.full((d,), 0.01, dtype=torch.float64, device="cuda")
dw = torch.zeros_like(w)
grads = torch.empty((N, d), dtype=torch.float64, device="cuda")
ctr = torch.zeros((1,), dtype=torch.int64, device="cuda")
ctl = torch.zeros((2,), dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream


def run():
    rc = lib.tw_sgd_segment(X.data_ptr(), Z.data_ptr(), d, rows_x.data_ptr(), kx,
                            rows_z.data_ptr(), kz, None, None, 0, N, B, 1.0, 0, 12345,
                            ctr.data_ptr(), 0, steps, w.data_ptr(), dw.data_ptr(),
                            grads.data_ptr(), 0.05, 0.01, 0.9, ctl.data_ptr(), s)
    assert rc == 0, rc


for _ in range(3):
    run()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
run()
ev[1].record()
torch.cuda.synchronize()
assert int(ctl[1]) == 0
t = np.zeros(256 * 32 * 8, dtype=np.uint64)
assert lib.tw_debug_seg_times(t.ctypes.data_as(vp), t.size) == 0
t = t.reshape(256, 32, 8)[:N, :steps].astype(np.int64) * 10  # ns
print(f"segment {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us for {steps} steps")
cols = [("grad", 0, 1), ("st.land", 1, 4), ("b1", 4, 2), ("upd.ld", 2, 5), ("upd.sum", 5, 3),
        ("upd.land", 3, 6)]
print("step | " + " | ".join(f"{c} med/max" for c, _, _ in cols) +
      " | b2+w (next 0 - 6) med/max | period | last stored -> max b1 pass")
for k in range(steps):
    row = []
    for _, a_, b_ in cols:
        v = t[:, k, b_] - t[:, k, a_]
        row.append(f"{np.median(v)/1e3:5.1f} {v.max()/1e3:5.1f}")
    if k + 1 < steps:
        v = t[:, k + 1, 0] - t[:, k, 6]
        row.append(f"{np.median(v)/1e3:5.1f} {v.max()/1e3:5.1f}")
        row.append(f"{(t[:, k + 1, 0].max() - t[:, k, 0].max())/1e3:5.1f}")
    else:
        row += ["", ""]
    row.append(f"{(t[:, k, 2].max() - t[:, k, 1].max())/1e3:5.1f}")
    print(f"{k:3d} | " + " | ".join(row))
