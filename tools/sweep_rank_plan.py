"""The once-per-call ranking (tw_rank_images) at the bench shape (1e6 + 1e6 doubles) under each
large-Z plan of tw_rank_set_plan (sample keys x z per thread), device time by HIP events with
the GPU busy before the call (GPU box).  Gaussian scores and a tie-heavy variant."""
import itertools
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    ops = HipOps()
    g = torch.Generator(device="cuda").manual_seed(1)
    n = 1_000_000
    data = {"gauss": (torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5,
                      torch.randn(n, dtype=torch.float64, device="cuda", generator=g)),
            "ties": (torch.randint(0, 5000, (n,), device="cuda", generator=g).double(),
                     torch.randint(0, 5000, (n,), device="cuda", generator=g).double()),
            "ties1k": (torch.randint(0, 1000, (n,), device="cuda", generator=g).double(),
                       torch.randint(0, 1000, (n,), device="cuda", generator=g).double())}
    # the images against the oracle's definition g(v) = #{z < v} (searchsorted on sorted Z)
    for k, (X, Z) in data.items():
        xr, zr = ops.rank_images(X, Z, L.TW_F64)
        zs = torch.sort(Z).values
        gx = torch.searchsorted(zs, X, right=False).to(torch.float32)
        gz = torch.searchsorted(zs, Z, right=False).to(torch.float32)
        img = lambda r: (r & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
        print(f"{k}: x images exact {bool(torch.equal(img(xr), gx))}, "
              f"z images exact {bool(torch.equal(img(zr), -gz))}", flush=True)
    busy = torch.empty((1 << 26,), dtype=torch.float64, device="cuda")
    ref = {k: ops.rank_images(X, Z, L.TW_F64) for k, (X, Z) in data.items()}
    for sample, per in itertools.product(*((list(map(int, sys.argv[1].split(","))), list(map(int, sys.argv[2].split(",")))) if len(sys.argv) > 2 else ((512, 1024, 2048), (4, 8, 16)))):
        L.call("tw_rank_set_plan", sample, per)
        row = []
        for k, (X, Z) in data.items():
            xr, zr = ops.rank_images(X, Z, L.TW_F64)
            same = bool(torch.equal(xr, ref[k][0]) and torch.equal(zr, ref[k][1]))
            dev = []
            for _ in range(15):
                busy.mul_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.rank_images(X, Z, L.TW_F64)
                e1.record()
                torch.cuda.synchronize()
                dev.append(e0.elapsed_time(e1))
            row.append(f"{k} {np.median(dev) * 1e3:6.1f} us (same images: {same})")
        print(f"sample {sample:4d} per {per:2d}: " + "; ".join(row), flush=True)
    L.call("tw_rank_set_plan", 1024, 8)


if __name__ == "__main__":
    main()
