"""Learning over ranks on ONE GPU (gloo for setup, the device-resident peer exchange per step,
csrc/peer.hip): bench.py's sgd_steps_per_s at the C4 shape and at C5 B = 100 with G co-resident
ranks, against one rank — the rehearsal VERDICT r04 item 3 asks for (on one GPU the ranks share
the chip, so the G-rank step does the one-GPU step's work plus the exchange).
    python tools/probe_learn_ranks.py G [c4|c5|both] [trace|allcols]
allcols: the round-5 per-step exchange (every rank updates all d columns, tw_peer_step) instead
of the column owners' (tw_peer_step_cols, learning.PEER_COLUMNS).
trace: a further short run of each line under torch.profiler (kineto, in-process: no re-exec),
rank 0's per-kernel mean device time printed beside the line."""
import json
import os
import pathlib
import socket
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))


def kernel_means(fn):
    """fn() under torch.profiler: {kernel name: [launches, mean us]} of the device kernels."""
    import torch
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    out = {}
    for e in prof.key_averages():
        n, tot = e.count, getattr(e, "device_time_total", getattr(e, "cuda_time_total", 0))
        if tot > 0 and n and not e.key.startswith(("aten::", "cuda", "hip")):
            out[e.key[:60]] = [n, round(tot / n, 2)]
    return out


def worker(rank, G, port, what, q, trace=False, allcols=False):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    torch.cuda.set_device(0)
    import bench
    import tuplewise.learning as lr
    lr.PEER_COLUMNS = not allcols  # forced either way (the default picks by G)
    g = dist.group.WORLD
    out = {}
    if what in ("c4", "both"):
        out["C4"] = bench.sgd_steps_per_s(9117, 702, 10, 100, 100, 25, 4000, 2, group=g,
                                          check_prefix=20)
    if what in ("c5", "both"):
        out["C5_B100"] = bench.sgd_steps_per_s(bench.C5_N, bench.C5_N, 512, 256, 100, 25, 500,
                                               2, group=g, check_prefix=20)
    if trace:
        shapes = {"C4": (9117, 702, 10, 100, 100, 25, 200, 1),
                  "C5_B100": (bench.C5_N, bench.C5_N, 512, 256, 100, 25, 200, 1)}
        for k in list(out):
            out[k]["kernels"] = kernel_means(lambda: bench.sgd_steps_per_s(*shapes[k], group=g))
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    G = int(sys.argv[1])
    what = sys.argv[2] if len(sys.argv) > 2 else "both"
    trace = len(sys.argv) > 3 and sys.argv[3] == "trace"
    allcols = len(sys.argv) > 3 and sys.argv[3] == "allcols"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, G, port, what, q, trace, allcols)) for r in range(G)]
    for p in ps:
        p.start()
    res = q.get(timeout=900)
    for p in ps:
        p.join(timeout=120)
    print(json.dumps({"ranks": G, "exchange": "all columns" if allcols else "column owners",
                      **{k: {kk: v[kk] for kk in ("steps_per_s", "ms_per_step",
                                                               "trajectory_equal_1rank", "kernels")
                                         if kk in v} | {"launches": v["config"]["launches"]}
                                     for k, v in res.items()}}), flush=True)
