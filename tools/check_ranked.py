"""Ranked vs plain device-RNG incomplete counts at the bench shape (GPU box); on a mismatch,
check the rank codes against NumPy searchsorted."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch
import tuplewise  # noqa: F401
from tuplewise import _lib as L
from tuplewise.device import ShardedSample

n, N, B = 1_000_000, 64, 1_000_000
g = torch.Generator(device="cuda").manual_seed(1)
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, algo="pairs")
S.repartition(3)
ops = S.ops
args = (S.X, S.x_off_dev, S.Z, S.z_off_dev, N, B, 99, 0, S.dtype, S.pred)
plain = ops.count_rng(*args).cpu().numpy()
ranked = ops.count_rng(*args, max_nx=S.max_nx, max_nz=S.max_nz).cpu().numpy()
print("equal:", np.array_equal(plain, ranked), "diff shards:", np.nonzero(plain != ranked)[0][:10])
wb = int(L.lib().tw_count_pairs_rng_work_bytes(N, S.max_nx, S.max_nz, S.dtype, S.pred))
work = torch.empty(wb, dtype=torch.uint8, device="cuda")
out = torch.empty(N, dtype=torch.int64, device="cuda")
L.call("tw_count_pairs_rng_ws", L.ptr(S.X), L.ptr(S.x_off_dev), L.ptr(S.Z), L.ptr(S.z_off_dev),
       N, S.max_nx, S.max_nz, B, 99, 0, S.dtype, S.pred, L.ptr(work), wb, L.ptr(out),
       L.stream_handle())
torch.cuda.synchronize()
k = n // N
C, chunks = 4096, 4
keys_bytes = ((N * chunks * C * 8 + 255) // 256) * 256
cx = work[keys_bytes:keys_bytes + N * k * 2].view(torch.int16).cpu().numpy().astype(np.int64) & 0xFFFF
pz_off = keys_bytes + ((N * k * 2 + 255) // 256) * 256
pz = work[pz_off:pz_off + N * k * 2].view(torch.int16).cpu().numpy().astype(np.int64) & 0xFFFF
Xh, Zh = S.X.cpu().numpy(), S.Z.cpu().numpy()
bad = 0
for s in range(N):
    zs = np.sort(Zh[s * k:(s + 1) * k])
    ex = np.searchsorted(zs, Xh[s * k:(s + 1) * k], side="left")
    ez = np.searchsorted(zs, Zh[s * k:(s + 1) * k], side="left")
    bx = np.nonzero(cx[s * k:(s + 1) * k] != ex)[0]
    bz = np.nonzero(pz[s * k:(s + 1) * k] != ez)[0]
    if len(bx) or len(bz):
        bad += 1
        if bad <= 3:
            print("shard", s, "bad x", len(bx), bx[:8], "bad z", len(bz), bz[:8])
print("shards with bad codes:", bad)
