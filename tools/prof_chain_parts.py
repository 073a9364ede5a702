"""The once-per-call parts of UnN_many's step chains at the bench shape, device time per call
(HIP events, the GPU busy while the calls are enqueued; also usable under rocprofv3
--kernel-trace): the ranking of X u Z (one process,
and rank 0's share at G = 8 against the whole Z), the chain emission of 20 steps with 2, 4 and
8 elements per thread and 1 or 16 / that many steps per round (tw_chain_set_emit), one process
and a G = 8 rank's send buckets.
    python3 tools/prof_chain_parts.py"""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tuplewise  # noqa: E402,F401
from tuplewise import _lib as L  # noqa: E402
from tuplewise.device import HipOps  # noqa: E402

torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(1)
n, N, K = 1_000_000, 64, 20
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
ops = HipOps()
M64 = 2 ** 64 - 1
kxs = [(2 * k) & M64 for k in range(7, 7 + K)]
kzs = [(2 * k + 1) & M64 for k in range(7, 7 + K)]
G = 8
nl = n // G
busy = torch.empty((1 << 26,), dtype=torch.float64, device="cuda")


def dev_ms(fn, reps=5):
    """Device time per call, the GPU kept busy while the calls are enqueued."""
    fn()
    torch.cuda.synchronize()
    busy.mul_(1.0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for cs, per in ((2048, 16), (1024, 16), (512, 16), (2048, 8), (2048, 4), (1024, 8), (1024, 4)):
    L.call("tw_rank_set_plan", cs, per)
    a = dev_ms(lambda: ops.rank_images_query(Z, X, Z, L.TW_F64))
    b = dev_ms(lambda: ops.rank_images_query(Z, X[:nl], Z[:nl], L.TW_F64))
    print(f"ranking sample={cs} per={per}: one process {a * 1e3:.1f} us, a G = 8 rank's share "
          f"{b * 1e3:.1f} us", flush=True)
L.call("tw_rank_set_plan", 1024, 8)
xr, zr = ops.rank_images_query(Z, X, Z, L.TW_F64)
xq, zq = ops.rank_images_query(Z, X[:nl], Z[:nl], L.TW_F64)
xb = torch.empty((K, n), dtype=torch.float32, device="cuda")
zb = torch.empty((K, n), dtype=torch.float32, device="cuda")
xp = torch.empty(n, dtype=torch.int32, device="cuda")
zp = torch.empty(n, dtype=torch.int32, device="cuda")
cur = torch.empty(K * 2 * (N + 1), dtype=torch.int32, device="cuda")
cap = 2 * nl // G + 2 * nl // (8 * G) + 1024
send = torch.empty(G * K * (cap + 1), dtype=torch.int64, device="cuda")
flag = torch.zeros(1, dtype=torch.int32, device="cuda")
for epr, spr in ((2, 1), (2, 8), (4, 1), (4, 4), (8, 1), (8, 2)):
    L.call("tw_chain_set_emit", epr, spr)
    a = dev_ms(lambda: ops.chain_emit(xr, zr, False, xp, zp, True, 0, 1, kxs, kzs, n // N,
                                      n // N, N, x_bag=xb, z_bag=zb, cursors=cur))
    b = dev_ms(lambda: ops.chain_emit(xq, zq, False, xp[:nl], zp[:nl], True, 0, G, kxs, kzs,
                                      nl // 8, nl // 8, 8, send=send, cap=cap, flag=flag))
    print(f"emit {K} steps epr={epr} s={spr}: one process {a * 1e3:.1f} us, a G = 8 rank "
          f"{b * 1e3:.1f} us", flush=True)
L.call("tw_chain_set_emit", 0, 0)
print("done", flush=True)
