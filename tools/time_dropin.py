"""Parts of the drop-in est.UnNT(X, Z, 64, 4, "prop-SWOR") device-shuffle path at C3 size (GPU
box): host draws, uploads, device swap rounds, write-back, count; each step synchronised."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tuplewise  # noqa: E402,F401
import tuplewise.estimation as est  # noqa: E402
from tuplewise import _engine as E, _lib as L  # noqa: E402
from tuplewise.numpy_rng import shuffle_draws32  # noqa: E402

n, T, N = 1_000_000, 4, 64
rng = np.random.RandomState(0)
X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
np.random.seed(1)
for _ in range(3):
    est.UnNT(X, Z, N, T, "prop-SWOR")
torch.cuda.synchronize()


def tick(label, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    print(f"  {label}: {(t - t0) * 1e3:.2f} ms", flush=True)
    return t


for rep in range(2):
    t0 = time.perf_counter()
    v = est.UnNT(X, Z, N, T, "prop-SWOR")
    t0 = tick("est.UnNT call", t0)
    jx, jz = [], []
    for _ in range(T):
        jx.append(shuffle_draws32(n))
        jz.append(shuffle_draws32(n))
    t0 = tick("host draws (2T)", t0)
    jxd = [L.to_device(a.view(np.int32)) for a in jx]
    jzd = [L.to_device(a.view(np.int32)) for a in jz]
    t0 = tick("upload draws", t0)
    xd, zd = L.to_device(X), L.to_device(Z)
    t0 = tick("upload X, Z", t0)
    xs, zs = E.shuffle_snapshots_device(xd, zd, jx, jz)
    t0 = tick("shuffle_snapshots_device (incl. draw uploads)", t0)
    a = xs[T - 1].cpu().numpy()
    b = zs[T - 1].cpu().numpy()
    t0 = tick("write-back D2H", t0)

# A/B of the one-workgroup tail of the swap rounds (tw_shuffle_swaps_set_tail)
for tail in (0, 1, 0, 1):
    L.call("tw_shuffle_swaps_set_tail", tail)
    est.UnNT(X, Z, N, T, "prop-SWOR")
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est.UnNT(X, Z, N, T, "prop-SWOR")
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    xs, zs = E.shuffle_snapshots_device(xd, zd, jx, jz)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    xs, zs = E.shuffle_snapshots_device(xd, zd, jx, jz)
    torch.cuda.synchronize()
    print(f"tail {tail}: est.UnNT {np.median(ts) * 1e3:.2f} ms/call (median of 5), "
          f"shuffle_snapshots_device {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
L.call("tw_shuffle_swaps_set_tail", 1)
