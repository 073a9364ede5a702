"""Per-block timeline of the streaming wide gradient kernel (k_hinge_grad_stream) at the C5
shape (5e6 x 512 per class, N = 256, B = 100, device RNG), in a step sequence (gradient +
update launches): builds tools/_dbg/libtw_hinge.so from csrc/{capi,hinge}.hip with
-DTW_HINGE_TIMING (thread 0 stamps the 100 MHz wall clock at entry, rows resolved, first
chunk reduced, exit) and prints the distributions over blocks for the last launch.  (Study
build only.)

    python tools/phase_hinge.py build      (here, CPU)
    python tools/phase_hinge.py            (GPU box)
"""
import ctypes
import pathlib
import subprocess
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "trade-offs-in-distributed-tuplewise-estimation-and-learning_amd" / "csrc"
OUT = ROOT / "tools" / "_dbg" / "libtw_hinge.so"

if len(sys.argv) > 1 and sys.argv[1] == "build":
    OUT.parent.mkdir(exist_ok=True)
    objs = []
    for src in ("capi.hip", "hinge.hip"):
        o = OUT.parent / ("hg_" + src + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                        "-std=c++17", "-ffp-contract=off", "-DTW_HINGE_TIMING", "-c",
                        str(CSRC / src), "-o", str(o)], check=True)
        objs.append(str(o))
    # the rest of the library as built (make), for the symbols hinge.hip uses from elsewhere
    rest = [str(p) for p in sorted(CSRC.glob("*.o"))
            if p.name not in ("capi.o", "hinge.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    str(OUT)] + objs + rest + ["-ldl", "-pthread"], check=True)
    sys.exit(0)

import torch  # noqa: E402

lib = ctypes.CDLL(str(OUT))
vp, i64, i32, f64, u64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                          ctypes.c_uint64)
lib.tw_pair_grad_rng.argtypes = [vp, vp, i64, vp, i64, vp, i64, i32, i64, vp, f64, i32, u64, vp,
                                 i32, vp, vp]
lib.tw_sgd_update.argtypes = [vp, vp, vp, i32, i64, f64, f64, f64, vp, vp]
n, d, N, B = 5_000_000, 512, 256, 100
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
st = torch.cuda.current_stream().cuda_stream


def step():
    assert lib.tw_pair_grad_rng(X.data_ptr(), Z.data_ptr(), d, rows_x.data_ptr(), kx,
                                rows_z.data_ptr(), kz, N, B, w.data_ptr(), 1.0, 0, 12345,
                                ctr.data_ptr(), 0, grads.data_ptr(), st) == 0
    assert lib.tw_sgd_update(w.data_ptr(), dw.data_ptr(), grads.data_ptr(), N, d, 0.05, 0.01,
                             0.9, ctr.data_ptr(), st) == 0


for _ in range(20):
    step()
torch.cuda.synchronize()
t = np.zeros(N * 4, dtype=np.uint64)
assert lib.tw_debug_hinge_times(t.ctypes.data_as(vp), t.size) == 0
t = t.reshape(N, 4).astype(np.int64) * 10  # ns
t0 = t[:, 0].min()
q = lambda v: f"min {v.min()/1e3:6.2f} med {np.median(v)/1e3:6.2f} max {v.max()/1e3:6.2f} us"
print("block start (after first) ", q(t[:, 0] - t0))
print("rows resolved             ", q(t[:, 1] - t[:, 0]))
print("first chunk reduced       ", q(t[:, 2] - t[:, 1]))
print("rest of the block         ", q(t[:, 3] - t[:, 2]))
print("block total               ", q(t[:, 3] - t[:, 0]))
print("kernel span (first start -> last exit) %.2f us" % ((t[:, 3].max() - t0) / 1e3))
order = np.argsort(t[:, 3])
print("exit times of the last 16 blocks (us after first start):",
      np.round((t[order[-16:], 3] - t0) / 1e3, 1).tolist())
print("exit time quantiles 10/50/90%:", np.round(np.percentile(t[:, 3] - t0, [10, 50, 90]) / 1e3, 1).tolist())
