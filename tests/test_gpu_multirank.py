"""Multi-rank paths with the real HIP kernels: 2 processes on the box's one GPU, gloo
(RCCL needs distinct devices; the 8-GPU RCCL run is the driver's scaling bench).  Checks that
sharding over ranks changes nothing: trajectories and estimates equal the 1-process ones."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_HIST = ("norm_w", "tr_AUC", "tc_AUC", "bc_AUC")


def _learn_worker(rank, port, G, mode, q, layout="replicated", cols=None):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    torch.cuda.set_device(0)
    import tuplewise.learning as lr
    lr.PEER_COLUMNS = cols  # True: the column owners' per-step exchange (tw_peer_step_cols)
    X, Z, w0, p = _problem()
    traj = []
    np.random.seed(99)
    lr.learning_process(X, Z, p, rng_mode=mode, trajectory=traj, group=dist.group.WORLD,
                        x_layout=layout)
    # no trajectory: the segments — over ranks the persistent peer segment, whose gradient
    # exchange runs between the two processes' kernels through IPC-mapped peer buffers
    p2 = dict(_problem()[3], n_it=60, eval_mod=20)
    np.random.seed(99)
    lr.learning_process(X, Z, p2, rng_mode=mode, group=dist.group.WORLD, x_layout=layout)
    if rank == 0:
        q.put((np.stack(traj), {k: p2[k] for k in _HIST}))
    dist.barrier()
    dist.destroy_process_group()


def _problem():
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
    return X, Z, w0, p


@pytest.mark.parametrize("G,mode,layout,cols",
                         [(2, m, la, None) for m in ("replay", "device")
                          for la in ("replicated", "partitioned")]
                         + [(3, "replay", "replicated", None), (3, "device", "partitioned", None),
                            (2, "device", "replicated", True), (3, "replay", "partitioned", True),
                            (8, "device", "replicated", None)])
def test_learning_two_ranks_equals_one(gpu, G, mode, layout, cols):
    """G ranks (gloo) on the box's GPU equal one rank bit for bit — with a trajectory (the
    per-step peer exchange) and without (the persistent peer segment, three evaluations).
    G = 3: N = 8 shards split 2/3/3 (uneven splits, the reference's N = 100 over 8 GPUs).
    cols=True: the per-step exchange by column owners (tw_peer_step_cols; d = 8 over 3 ranks
    gives owners of 2, 3 and 3 columns); G = 8 with the default (column owners from 8 ranks:
    one shard and one column per rank) — the driver's 8-GPU learning lines' exchange."""
    import torch.multiprocessing as mp
    import tuplewise.learning as lr
    X, Z, w0, p = _problem()
    ref = []
    np.random.seed(99)
    lr.learning_process(X, Z, p, rng_mode=mode, trajectory=ref)
    p2 = dict(_problem()[3], n_it=60, eval_mod=20)
    np.random.seed(99)
    lr.learning_process(X, Z, p2, rng_mode=mode)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_learn_worker, args=(r, port, G, mode, q, layout, cols))
             for r in range(G)]
    for pr in procs:
        pr.start()
    got, hist = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert np.array_equal(got, np.stack(ref))
    assert len(hist["norm_w"]) == 3 and hist == {k: p2[k] for k in _HIST}


def _est_worker(rank, port, G, q, exchange="fixed", chain=True):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=G)
    torch.cuda.set_device(0)
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    D.CHAIN_STEPS = chain  # False: the per-step all-to-all of rank-image records
    rng = np.random.RandomState(3)
    n_loc, N = 40_000, 8
    X = rng.normal(0.3, 1, G * n_loc)
    Z = rng.normal(0, 1, G * n_loc)
    S = ShardedSample(torch.from_numpy(X[rank * n_loc:(rank + 1) * n_loc].copy()).cuda(),
                      torch.from_numpy(Z[rank * n_loc:(rank + 1) * n_loc].copy()).cuda(), N,
                      group=dist.group.WORLD, exchange=exchange, algo="pairs")
    vals = [float(S.UnN(k)) for k in (1, 2, 3)] + [float(S.UnNB(500, seed=4))]
    vals += [float(v) for v in S.UnN_many([5, 6, 7])]  # rank images: the step chains
    # the incomplete statistic on the chains (exact-position bags, device draws on images)
    vals += [float(v) for v in S.UnNB_many(700, 21, [15, 16, 17])]
    S.algo = "sorted"  # the chains' exact bucket count of every bag (per-step path unchained)
    vals += [float(v) for v in S.UnN_many([8, 9])]
    Xg = [torch.empty(S.X.shape, dtype=S.X.dtype) for _ in range(G)]
    Zg = [torch.empty(S.Z.shape, dtype=S.Z.dtype) for _ in range(G)]
    dist.all_gather(Xg, S.X.cpu())
    dist.all_gather(Zg, S.Z.cpu())
    if rank == 0:
        q.put((vals, torch.cat(Xg).numpy(), torch.cat(Zg).numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G,exchange,chain", [(2, "fixed", True), (2, "fixed", False),
                                               (2, "exact", False), (3, "fixed", True),
                                               (3, "exact", False)])
def test_sharded_sample_two_ranks_equals_one(gpu, G, exchange, chain):
    """G ranks (gloo, real kernels) equal one process: UnN with a key, UnNB, the step chains
    (all-pairs and exact bucket counts) and the final arrays.  G = 3: three send buckets per
    rank (G = 2 has one remote peer only)."""
    import torch
    import torch.multiprocessing as mp
    from tuplewise.device import ShardedSample
    n_loc, N = 40_000, 8
    rng = np.random.RandomState(3)
    X = rng.normal(0.3, 1, G * n_loc)
    Z = rng.normal(0, 1, G * n_loc)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), G * N,
                      algo="pairs")
    want = [float(S.UnN(k)) for k in (1, 2, 3)] + [float(S.UnNB(500, seed=4))]
    want += [float(v) for v in S.UnN_many([5, 6, 7])]
    want += [float(S.UnNB(700, 21 + t, k)) for t, k in enumerate([15, 16, 17])]
    assert S._chain_ok() and S.algo == "pairs"
    S.algo = "sorted"
    want += [float(v) for v in S.UnN_many([8, 9])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_est_worker, args=(r, port, G, q, exchange, chain))
             for r in range(G)]
    for pr in procs:
        pr.start()
    got, Xg, Zg = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert got == want
    assert np.array_equal(Xg, S.X.cpu().numpy()) and np.array_equal(Zg, S.Z.cpu().numpy())
