"""A/B in one process, interleaved: UnN_many at the bench shape (1e6/class, 64 shards, K steps)
through the step chains and through one launch per step; then the counts alone — K launches of
the per-step rank count against one chain count launch of K steps (and of K/4 steps x 4) — to
separate launch structure from box-to-box clock differences.
    python tools/ab_chain.py [K] [rounds]"""
import pathlib
import subprocess
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np
import torch

import tuplewise  # noqa: F401
from tuplewise import device as D
from tuplewise.device import HipOps, ShardedSample, prop_swor_layout

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
torch.cuda.set_device(0)
gen = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
S = ShardedSample(X.clone(), Z.clone(), N, algo="pairs")
key = [1000]


def call(chain):
    D.CHAIN_STEPS = chain
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    S.UnN_many(range(key[0], key[0] + K))
    torch.cuda.synchronize()
    key[0] += K
    D.CHAIN_STEPS = True
    return (time.perf_counter() - t0) * 1e3


for _ in range(2):
    call(True), call(False)
res = {True: [], False: []}
for r in range(rounds):
    for chain in (True, False):
        res[chain].append(call(chain))
for chain in (True, False):
    v = res[chain]
    print(f"UnN_many K={K} {'step chains' if chain else 'per-step   '}: median {np.median(v):.3f} "
          f"ms/call ({np.median(v) / K:.4f} ms/step), runs " + " ".join(f"{x:.2f}" for x in v),
          flush=True)

# the counts alone on fixed bags / records (no repartition)
ops = HipOps()
xr, zr = ops.rank_images_query(Z, X, Z, 0)
x_off, z_off, _ = prop_swor_layout(n, n, N)
xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
k = n // N
xbag = (xr & 0xFFFFFFFF).to(torch.int32).view(torch.float32).repeat(K, 1).contiguous()
zbag = (zr & 0xFFFFFFFF).to(torch.int32).view(torch.float32).repeat(K, 1).contiguous()
out = torch.zeros((K, N), dtype=torch.int64, device="cuda")


def ev(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def per_step():
    for i in range(K):
        ops.count_rank_step(xr, xo, zr, zo, N, k, k, out[i], None, 0, None, 0, None)


def one_chain():
    ops.count_chain(xbag, xo, zbag, zo, N, K, n, n, k, k, False, out)


def quarter_chain():
    q = max(1, K // 4)
    for i0 in range(0, K, q):
        c = min(q, K - i0)
        ops.count_chain(xbag[i0:], xo, zbag[i0:], zo, N, c, n, n, k, k, False, out[i0:i0 + c])


for f in (per_step, one_chain, quarter_chain):
    f()
res = {f.__name__: [] for f in (per_step, one_chain, quarter_chain)}
for r in range(rounds):
    for f in (per_step, one_chain, quarter_chain):
        res[f.__name__].append(ev(f))
for name, v in res.items():
    print(f"counts alone, {name:13s}: median {np.median(v) / K * 1e3:.1f} us/step, runs "
          + " ".join(f"{x / K * 1e3:.1f}" for x in v), flush=True)
try:
    print(subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True,
                         timeout=30).stdout[-800:])
except Exception as e:  # noqa: BLE001
    print("rocm-smi:", e)
