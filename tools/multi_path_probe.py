"""Probe the multi-rank UnN_many path on ONE GPU (world size 1, RCCL): the exchange kernels
run on a side stream beside the count kernel.  Reports ms/step against the bare count, for a
normal- and a high-priority side stream.  Run on the GPU box:
    python tools/multi_path_probe.py"""
import os
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
opts = dist.ProcessGroupNCCL.Options()
opts.is_high_priority_stream = True
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                        pg_options=opts)
import tuplewise  # noqa: F401
from tuplewise.device import ShardedSample

g = torch.Generator(device="cuda").manual_seed(1)
n, N = 1_000_000, 64
X = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) + 0.5
Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
S = ShardedSample(X, Z, N, group=dist.group.WORLD, algo="pairs")
S._force_multi = True  # take the multi-rank code path at world size 1
from tuplewise import _lib as L
for prio, grid in ((0, 2048), (-1, 2048), (-1, 256), (-1, 0), (-1, 64), (-1, 32)):
    L.call("tw_exchange_set_grid", grid)
    S._side = torch.cuda.Stream(priority=prio)
    S.UnN_many(range(30))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = 30
    S.UnN_many(range(100, 100 + K))
    torch.cuda.synchronize()
    print(f"side priority {prio}, exchange grid {grid}: "
          f"{(time.perf_counter() - t0) / K * 1e3:.4f} ms/step", flush=True)
L.call("tw_exchange_set_grid", 0)
S._force_multi = False
S.UnN_many(range(30))
torch.cuda.synchronize()
t0 = time.perf_counter()
S.UnN_many(range(200, 230))
torch.cuda.synchronize()
print(f"one-GPU path: {(time.perf_counter() - t0) / 30 * 1e3:.4f} ms/step", flush=True)
dist.destroy_process_group()
