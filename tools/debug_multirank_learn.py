"""G gloo ranks on the box's one GPU running learning_process (tests/test_gpu_multirank.py's
problem) with progress printed per rank — for a multi-rank learning failure that the pytest run
only shows as a hang.
    python tools/debug_multirank_learn.py G MODE LAYOUT [trajectory|segments]"""
import faulthandler
import os
import pathlib
import socket
import sys
import traceback

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np


def problem():
    rng = np.random.RandomState(0)
    X = np.hstack([rng.normal(size=(400, 7)), np.ones((400, 1))])
    Z = np.hstack([rng.normal(0.5, 1, size=(90, 7)), np.ones((90, 1))])
    w0 = rng.normal(size=(8, 1))
    tX = np.hstack([rng.normal(size=(50, 7)), np.ones((50, 1))])
    tZ = np.hstack([rng.normal(0.5, 1, size=(20, 7)), np.ones((20, 1))])
    mon = [(int(a), int(b)) for a, b in zip(rng.randint(0, 400, 300), rng.randint(0, 90, 300))]
    p = {"n_it": 40, "margin": 1, "N": 8, "B": 16, "reshuffle_mod": 5, "reg": 0.05,
         "learning_rate": 0.01, "eval_mod": 1000, "w_init": w0, "test_X": tX, "test_Z": tZ,
         "train_mon_pairs": mon, "train_X": X, "train_Z": Z}
    return X, Z, p


def worker(rank, port, G, mode, layout, what):
    faulthandler.dump_traceback_later(100, exit=True)
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=G)
        torch.cuda.set_device(0)
        import tuplewise.learning as lr
        X, Z, p = problem()
        print(f"[{rank}] start {what}", flush=True)
        np.random.seed(99)
        if what == "trajectory":
            traj = []
            lr.learning_process(X, Z, p, rng_mode=mode, trajectory=traj,
                                group=dist.group.WORLD, x_layout=layout)
            print(f"[{rank}] done, w[-1][:3] = {np.stack(traj)[-1].ravel()[:3]}", flush=True)
        else:
            p2 = dict(p, n_it=60, eval_mod=20)
            lr.learning_process(X, Z, p2, rng_mode=mode, group=dist.group.WORLD,
                                x_layout=layout)
            print(f"[{rank}] done, norm_w = {p2['norm_w']}", flush=True)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        print(f"[{rank}] FAILED\n{traceback.format_exc()}", flush=True)
        os._exit(3)


if __name__ == "__main__":
    import torch.multiprocessing as mp
    G, mode, layout = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    what = sys.argv[4] if len(sys.argv) > 4 else "trajectory"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, port, G, mode, layout, what)) for r in range(G)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=120)
        if pr.is_alive():
            pr.kill()
    print("exit codes", [pr.exitcode for pr in procs], flush=True)
