"""Can two ranks share one GPU over RCCL (backend "nccl")?  Spawns 2 processes on cuda:0 and
runs an all_reduce, an all_gather_into_tensor and an async all_to_all_single (GPU box)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(0)
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0), pg_options=opts)
    x = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    g = torch.empty(world * 4, device="cuda")
    dist.all_gather_into_tensor(g, torch.arange(4, device="cuda", dtype=torch.float32) + 10 * rank)
    a = torch.arange(world * 2, device="cuda", dtype=torch.int64) + 100 * rank
    b = torch.empty_like(a)
    w = dist.all_to_all_single(b, a, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {x.tolist()} all_gather {g.tolist()} all_to_all {b.tolist()}",
          flush=True)
    dist.barrier(device_ids=[0])
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2, 29517), nprocs=2, join=True)
    print("ok")
