"""gloo all_to_all_single with split sizes on CUDA tensors, 3 ranks on one GPU, the receive
buffer a view at an offset of a larger tensor (the partitioned row exchange's pattern)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def w(r, G, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=r, world_size=G)
    torch.cuda.set_device(0)
    sc = [[0, 3, 5], [2, 0, 4], [1, 6, 0]][r]
    rc = [[0, 2, 1], [3, 0, 6], [5, 4, 0]][r]
    send = torch.cat([torch.full((c,), 100 * r + g, dtype=torch.float64) for g, c in
                      enumerate(sc)]).cuda()
    for view in (False, True):
        big = torch.zeros(100, dtype=torch.float64, device="cuda")
        recv = big[10:10 + sum(rc)] if view else torch.zeros(sum(rc), dtype=torch.float64,
                                                             device="cuda")
        dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc)
        print(r, "view" if view else "plain", recv.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(w, args=(3, int(sys.argv[1]) if len(sys.argv) > 1 else 29611), nprocs=3)
