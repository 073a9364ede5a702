"""Every RCCL call of the multi-rank product path, executed on the box's one GPU (VERDICT r04
item 1): a world-size-1 `nccl` process group initialised as bench.py does (ProcessGroupNCCL
options with the high-priority stream), and the G > 1 branches forced through it with
`collectives=True`:

* ShardedSample._unn_many_chain: all_gather_into_tensor of both samples (`_all_gather`'s nccl
  branch), the chain emission into send buckets, the async all_to_all_single + work.wait()
  per chunk (and per sub-chunk with device.CHAIN_SUB > 0), chain_unpack, chain_gather, the
  counts' all-reduce with the overflow flag;
* ShardedSample._run_steps (UnNB_many, UnN with a key): the fixed-capacity exchange on the
  high-priority side stream (all_to_all_single) and the counts' all-reduce; the counted
  exchange (`exchange="exact"`: all_to_all_single with split sizes);
* SGDEngine over ranks: the device-resident gradient exchange (csrc/peer.hip: per-step publish
  + wait-and-update with a trajectory, the persistent peer segment without), and with
  learning.PEER_EXCHANGE = False the per-step all_gather_into_tensor of the shard gradients;
  the partitioned layout's row exchange (all_to_all_single of counts and rows).

Each must give the estimates, final arrays and trajectories of the plain one-process path bit
for bit (reference: the serial shard loop estimation-experiment/main.py:48-69 and the learning
loop learning-experiment/make_exps.py:122-141 that these collectives distribute)."""
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _learn_problem():
    rng = np.random.RandomState(0)
    X = np.hstack([rng.normal(size=(400, 7)), np.ones((400, 1))])
    Z = np.hstack([rng.normal(0.5, 1, size=(90, 7)), np.ones((90, 1))])
    w0 = rng.normal(size=(8, 1))
    tX = np.hstack([rng.normal(size=(50, 7)), np.ones((50, 1))])
    tZ = np.hstack([rng.normal(0.5, 1, size=(20, 7)), np.ones((20, 1))])
    mon = [(int(a), int(b)) for a, b in zip(rng.randint(0, 400, 300), rng.randint(0, 90, 300))]
    p = {"n_it": 50, "margin": 1, "N": 8, "B": 16, "reshuffle_mod": 5, "reg": 0.05,
         "learning_rate": 0.01, "eval_mod": 25, "w_init": w0, "test_X": tX, "test_Z": tZ,
         "train_mon_pairs": mon, "train_X": X, "train_Z": Z}
    return X, Z, p


def _estimates(S, ties):
    """The estimator calls whose multi-rank branches hold RCCL calls, in a fixed order."""
    vals = [float(v) for v in S.UnN_many(range(5, 45))]  # 40 steps: two chunks, emitted
    vals += [float(v) for v in S.UnN_many(range(50, 54))]  # est.UnNT's own T = 4
    vals.append(float(S.UnN(3)))  # one repartition (exchange) + global counts
    if not ties:
        vals += [float(v) for v in S.UnNB_many(700, 11, [8, 9, 10])]  # side-stream exchange
        S.algo = "sorted"  # the chains' exact bucket count of every bag
        vals += [float(v) for v in S.UnN_many([12, 13, 14])]
        S.algo = "pairs"
    return vals, S.X.cpu().numpy(), S.Z.cpu().numpy()


def _worker(port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        opts = dist.ProcessGroupNCCL.Options()  # bench.py's RCCL options
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0), pg_options=opts)
        g = dist.group.WORLD
        assert dist.get_backend(g) == "nccl"
        import tuplewise.learning as lr
        from tuplewise.device import ShardedSample
        out = {"mismatch": [], "ran": []}
        gen = torch.Generator(device="cuda").manual_seed(7)
        n = 60_000
        data = {"f64": (torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.4,
                        torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)),
                "i64": (torch.randint(0, 500, (n,), device="cuda", generator=gen),
                        torch.randint(0, 480, (n,), device="cuda", generator=gen))}
        cases = [("f64", "strict", "fixed"), ("f64", "half", "fixed"), ("i64", "half", "fixed"),
                 ("f64", "strict", "exact")]
        import tuplewise.device as D
        for dt, tie, exch in cases:
            X, Z = data[dt]
            # UnNB_many over ranks: the step chains with exact-position bags (device.CHAIN_RNG,
            # tw_chain_unpack_exact + tw_count_pairs_chain_rng); the "exact" case keeps the
            # per-step exchange of _run_steps
            D.CHAIN_RNG = exch != "exact"
            plain = ShardedSample(X.clone(), Z.clone(), 8, tie_mode=tie, algo="pairs")
            forced = ShardedSample(X.clone(), Z.clone(), 8, group=g, tie_mode=tie, algo="pairs",
                                   exchange=exch, collectives=True)
            assert forced.coll and forced._chain_ok() and plain._chain_ok()
            a = _estimates(plain, tie == "half")
            b = _estimates(forced, tie == "half")
            tag = f"{dt}/{tie}/{exch}"
            out["ran"].append(tag)
            if a[0] != b[0]:
                out["mismatch"].append((tag, "estimates"))
            if not (np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])):
                out["mismatch"].append((tag, "final arrays"))
        D.CHAIN_RNG = True
        # configs[2]'s incomplete leg at its size on the chains: n = 1e6 per class, N = 64,
        # B = 1e6 pairs per shard, T = 4, two calls (the second carries the images)
        Xc = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen) + 0.5
        Zc = torch.randn(1_000_000, dtype=torch.float64, device="cuda", generator=gen)
        plain = ShardedSample(Xc.clone(), Zc.clone(), 64, algo="pairs")
        forced = ShardedSample(Xc.clone(), Zc.clone(), 64, group=g, algo="pairs",
                               collectives=True)
        assert forced._chain_rng_ok()
        for i, keys in enumerate(([31, 32, 33, 34], [35, 36, 37, 38])):
            a = plain.UnNB_many(1_000_000, 0xC3C3 + 10 * i, keys)
            b = forced.UnNB_many(1_000_000, 0xC3C3 + 10 * i, keys)
            if a != b:
                out["mismatch"].append((f"C3 incomplete chains call {i}", (a, b)))
        if not (torch.equal(plain.X, forced.X) and torch.equal(plain.Z, forced.Z)):
            out["mismatch"].append(("C3 incomplete chains", "final arrays"))
        out["ran"].append("C3/incomplete/chains")
        X, Z = data["f64"]  # the chunks' sub-chunks (CHAIN_SUB > 0: emissions on a side stream)
        a = _estimates(ShardedSample(X.clone(), Z.clone(), 8, algo="pairs"), False)
        D.CHAIN_SUB = 5
        try:
            b = _estimates(ShardedSample(X.clone(), Z.clone(), 8, group=g, algo="pairs",
                                         collectives=True), False)
        finally:
            D.CHAIN_SUB = 0
        out["ran"].append("f64/strict/fixed/sub-chunks")
        if a[0] != b[0] or not (np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])):
            out["mismatch"].append(("f64/strict/fixed/sub-chunks", "estimates or arrays"))
        Xl, Zl, p = _learn_problem()
        for peer, mode, layout in [(pe, m, la) for pe in (True, False)
                                   for m in ("replay", "device")
                                   for la in ("replicated", "partitioned")]:
            lr.PEER_EXCHANGE = peer  # False: the per-step RCCL all-gather of the partials
            if True:
                ref, got = [], []
                np.random.seed(99)
                lr.learning_process(Xl, Zl, dict(p), rng_mode=mode, trajectory=ref,
                                    x_layout=layout)
                np.random.seed(99)
                lr.learning_process(Xl, Zl, dict(p), rng_mode=mode, trajectory=got, group=g,
                                    x_layout=layout, collectives=True)
                tag = f"learning/{'peer' if peer else 'allgather'}/{mode}/{layout}"
                out["ran"].append(tag)
                if len(ref) != 50 or not np.array_equal(np.stack(ref), np.stack(got)):
                    out["mismatch"].append((tag, "trajectory"))
                # no trajectory: the segments (over ranks: the persistent peer segment); the
                # evaluation histories come from w at steps 0, 25
                pa, pb = dict(p), dict(p)
                np.random.seed(99)
                lr.learning_process(Xl, Zl, pa, rng_mode=mode, x_layout=layout)
                np.random.seed(99)
                lr.learning_process(Xl, Zl, pb, rng_mode=mode, group=g, x_layout=layout,
                                    collectives=True)
                if any(pa[k] != pb[k] for k in ("norm_w", "tr_AUC", "tc_AUC", "bc_AUC")):
                    out["mismatch"].append((tag, "segment histories"))
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put(("ok", out))
    except Exception:
        q.put(("error", traceback.format_exc()))


def test_rccl_world_size_one_equals_one_process(gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_worker, args=(_port(), q))
    pr.start()
    status, out = q.get(timeout=300)
    pr.join(timeout=120)
    assert status == "ok", out
    assert pr.exitcode == 0
    assert len(out["ran"]) == 14, out["ran"]
    assert out["mismatch"] == [], out["mismatch"]
