"""tw_gemv_f64 (evaluation_step's score products, make_exps.py:163, :170-171) at C5 widths
(GPU box): a thread per row vs one wave per row (tw_gemv_set_variant), GB/s of rows, and the
largest relative difference between the two and against torch's matmul."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(3)
for n, d in ((2_000_000, 512), (4_000_000, 100), (9117, 10)):
    A = torch.randn((n, d), dtype=torch.float64, device="cuda", generator=g)
    w = torch.randn((d,), dtype=torch.float64, device="cuda", generator=g)
    res = {}
    for v in (0, 1):
        L.call("tw_gemv_set_variant", v)
        out = torch.empty((n,), dtype=torch.float64, device="cuda")
        for _ in range(3):
            L.call("tw_gemv_f64", L.ptr(A), n, d, L.ptr(w), L.ptr(out), L.stream_handle())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            L.call("tw_gemv_f64", L.ptr(A), n, d, L.ptr(w), L.ptr(out), L.stream_handle())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[v] = out.clone()
        print(f"n={n} d={d} variant {v}: {ms:.3f} ms, {n * d * 8 / ms / 1e6:.0f} GB/s", flush=True)
    ref = A @ w
    rel = lambda a, b: float(((a - b).abs() / b.abs().clamp_min(1e-300)).max())
    print(f"   max rel diff variants {rel(res[1], res[0]):.2e}, vs torch {rel(res[1], ref):.2e}")
    L.call("tw_gemv_set_variant", 1)
