"""Cost of the once-per-call ranking of the rank-image path (tw_rank_images, csrc/rankimage.hip)
at the bench shape (1e6 + 1e6 doubles), GPU box: host enqueue time, device time (HIP events
with the GPU already busy, so the enqueue is hidden), and the parts: the workspace query, the
records kernels, the final gathers."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    ops = HipOps()
    g = torch.Generator(device="cuda").manual_seed(1)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    for _ in range(3):
        ops.rank_images(X, Z, L.TW_F64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        L.lib().tw_rank_images_work_bytes(n, n)
    print(f"work_bytes query: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us host", flush=True)
    host, dev = [], []
    busy = torch.empty((1 << 27,), dtype=torch.float64, device="cuda")
    for _ in range(10):
        torch.cuda.synchronize()
        busy.mul_(1.0)  # keep the GPU busy while the ranking is enqueued
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        xr, zr = ops.rank_images(X, Z, L.TW_F64)
        host.append(time.perf_counter() - t0)
        e1.record()
        torch.cuda.synchronize()
        dev.append(e0.elapsed_time(e1))
    print(f"rank_images: host enqueue {np.median(host) * 1e6:.1f} us, device {np.median(dev) * 1e3:.1f} us "
          f"(events around the call, GPU busy before)", flush=True)
    ev = []
    for _ in range(10):
        busy.mul_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gather_records(X, xr)
        ops.gather_records(Z, zr)
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1))
    print(f"two gather_records: {np.median(ev) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
