"""learning_process / evaluation_step (make_exps.py:96-190) on the device vs the reference's
golden run: the w trajectory (captured by hooking grad_inc_block in the reference) and the
evaluation lists that learning_process appends to p_learn.

Tolerance: north_star asks for SGD trajectories within 1e-5 relative; the device
reproduces NumPy's operation order except BLAS's dot-product order inside the filter test,
so we hold it to 1e-10 here.  AUC values are count-derived but sit on device-computed scores
(GEMV order differs from BLAS by an ulp): exact unless a score pair ties within an ulp."""
import logging

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _p_learn(golden, n_it=300):
    return {"n_it": n_it, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
            "learning_rate": 0.01, "eval_mod": 25, "w_init": golden["learn/w0"],
            "test_X": golden["learn/test_X"], "test_Z": golden["learn/test_Z"],
            "train_mon_pairs": [tuple(p) for p in golden["learn/mon"]],
            "train_X": golden["learn/X"], "train_Z": golden["learn/Z"]}


def test_trajectory_matches_reference(gpu, golden):
    import tuplewise.learning as lr
    p = _p_learn(golden)
    traj = []
    logging.disable(logging.CRITICAL)
    np.random.seed(2024)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=traj)
    ref = golden["learn/ws"]
    got = np.stack(traj)
    assert got.shape == ref.shape
    rel = np.abs(got - ref).max() / np.abs(ref).max()
    assert rel < 1e-10, rel
    for k in ("iter", "norm_w"):
        np.testing.assert_allclose(p[k], golden[f"learn/{k}"], rtol=1e-10)
    for k in ("bc_AUC", "tc_AUC"):
        np.testing.assert_allclose(p[k], golden[f"learn/{k}"], rtol=1e-9)
    for k in ("br_AUC", "tr_AUC"):
        np.testing.assert_allclose(p[k], golden[f"learn/{k}"], rtol=0, atol=1e-12)


def test_trajectory_sign_audit(gpu, golden):
    """count and report the hinge-filter decisions that could differ from the
    reference's BLAS order.  The 300-step golden run with the audit on: the same trajectory,
    zero filter flips, and the near-zero count reported (it bounds how many could flip)."""
    import tuplewise.learning as lr
    p = _p_learn(golden)
    audit = []
    logging.disable(logging.CRITICAL)
    np.random.seed(2024)
    traj = []
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=traj,
                        sign_audit=audit)
    ref = golden["learn/ws"]
    assert np.abs(np.stack(traj) - ref).max() / np.abs(ref).max() < 1e-10
    assert len(audit) == ref.shape[0]
    pairs = sum(a["pairs"] for a in audit)
    near = sum(a["near_zero"] for a in audit)
    flips = sum(a["flips"] for a in audit)
    print(f"sign audit: {pairs} pairs, {near} with |S| within the rounding bound, {flips} flips")
    assert flips == 0 and flips <= near
    assert pairs == ref.shape[0] * p["N"] * p["B"]


def test_sgd_optimizer_and_assert(gpu, golden):
    import tuplewise.learning as lr
    from oracle import oracle as O
    p = _p_learn(golden, n_it=30)
    traj = []
    np.random.seed(7)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, optim_type="SGD",
                        trajectory=traj)
    # oracle with plain SGD updates
    np.random.seed(7)
    w = golden["learn/w0"]
    X, Z = golden["learn/X"], golden["learn/Z"]
    X_s, Z_s = O.SWR_divide(X, Z, 10)
    dw = 0
    ws = []
    for i in range(30):
        if i % 5 == 0:
            X_s, Z_s = O.SWR_divide(X, Z, 10)
        ws.append(w.copy())
        g = O.UN_split(X_s, Z_s, O.grad_inc_block(w, 20, 1))
        w, dw = O.sgd_step(w, dw, g, 0.05, 0.01, optim_type="SGD")
    np.testing.assert_allclose(np.stack(traj), np.stack(ws), rtol=1e-10, atol=1e-14)
    with pytest.raises(AssertionError):
        lr.learning_process(X, Z, _p_learn(golden, n_it=2), optim_type="adam")


def test_device_rng_mode_matches_restatement(gpu, golden):
    """rng_mode="device": draws on the GPU (Philox), exact vs oracle's restatement."""
    import tuplewise.learning as lr
    from oracle import oracle as O
    p = _p_learn(golden, n_it=60)
    traj = []
    np.random.seed(31)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, rng_mode="device",
                        trajectory=traj)
    np.random.seed(31)
    seed = int(np.random.randint(0, 2 ** 63 - 1, dtype=np.int64))
    ws, _ = O.device_rng_learning_trajectory(golden["learn/X"], golden["learn/Z"], p, seed)
    np.testing.assert_allclose(np.stack(traj), np.stack(ws), rtol=1e-10, atol=1e-14)


def test_device_rng_graphs_equal_eager(gpu, golden):
    """hipGraph-replayed segments give the same w as eager launches."""
    import tuplewise.learning as lr
    out = []
    for graphs in (False, True):
        p = _p_learn(golden, n_it=137)
        p["eval_mod"] = 50
        np.random.seed(8)
        eng_w = []
        lr.learning_process(golden["learn/X"], golden["learn/Z"], p, rng_mode="device",
                            graphs=graphs)
        out.append((p["norm_w"], p["bc_AUC"]))
    assert out[0] == out[1]


def test_make_exps_writes_reference_schema(gpu, golden, tmp_path):
    """make_exps (make_exps.py:192-243): dynamics.json keys/lengths and the log file."""
    import json
    import tuplewise.learning as lr
    p = {"n_it": 60, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
         "learning_rate": 0.01, "eval_mod": 25, "w_init": np.random.normal(0, 1, (10, 1)),
         "test_X": golden["learn/test_X"], "test_Z": golden["learn/test_Z"]}
    out = tmp_path / "run_00"
    logging.disable(logging.NOTSET)
    for h in logging.root.handlers[:]:
        logging.root.removeHandler(h)
    lr.make_exps(5, str(out), p, data={"X": golden["pre/X"], "y": golden["pre/y"]})
    dyn = json.loads((out / "dynamics.json").read_text())
    for k in ("n_it", "margin", "N", "B", "reshuffle_mod", "reg", "learning_rate", "eval_mod",
              "iter", "norm_w", "bc_AUC", "br_AUC", "tr_AUC", "tc_AUC"):
        assert k in dyn, k
    assert dyn["iter"] == [0, 25, 50]
    assert not any(k.startswith(("train_", "test_", "w_")) for k in dyn)
    log = (out / "learning_process.log").read_text()
    assert "it     0: bc_AUC = " in log and "#X: " in log
    for h in logging.root.handlers[:]:
        logging.root.removeHandler(h)


@pytest.mark.parametrize("mode", ["replay", "device"])
def test_partitioned_layout_equals_replicated(gpu, golden, mode):
    """x_layout="partitioned" (rows exchanged at each reshuffle) changes no arithmetic."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for layout in ("replicated", "partitioned"):
        p = _p_learn(golden, n_it=60)
        traj = []
        np.random.seed(31)
        lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=traj,
                            rng_mode=mode, x_layout=layout)
        out[layout] = (np.stack(traj), p["bc_AUC"], p["tc_AUC"])
    assert np.array_equal(out["replicated"][0], out["partitioned"][0])
    assert out["replicated"][1:] == out["partitioned"][1:]


def test_row_exchange_kernels_simulated_ranks(gpu):
    """tw_row_route_counts / tw_row_pack / tw_row_unpack for G=3 owners simulated in one
    process (the all_to_all is a host-side regrouping): every requester's matrix == X[rows]."""
    import torch
    from tuplewise import _lib as L
    rng = np.random.RandomState(5)
    n, d, N, k, G = 1001, 13, 6, 37, 3
    X = rng.normal(size=(n, d))
    rows = rng.randint(0, n, size=N * k).astype(np.int64)
    rows[:5] = [0, n - 1, n // 3, n // 3 - 1, 2 * n // 3]  # owner boundaries
    M, M_q = N * k, (N // G) * k
    rows_d = L.to_device(rows)
    buckets = [[] for _ in range(G)]
    for r in range(G):
        lo, hi = r * n // G, (r + 1) * n // G
        part = L.to_device(X[lo:hi])
        counts = L.empty((G,), torch.int64)
        L.call("tw_row_route_counts", L.ptr(rows_d), M, M_q, lo, hi, G, L.ptr(counts),
               L.stream_handle())
        c = counts.cpu().numpy()
        owned = (rows >= lo) & (rows < hi)
        assert np.array_equal(c, owned.reshape(G, M_q).sum(1))
        start = torch.cumsum(counts, 0) - counts
        send = L.empty((max(int(c.sum()), 1), d + 1), torch.float64)
        cursor = L.empty((G,), torch.int64)
        L.call("tw_row_pack", L.ptr(rows_d), M, M_q, lo, hi, G, L.ptr(part), d, L.ptr(start),
               L.ptr(cursor), L.ptr(send), L.stream_handle())
        s = send.cpu().numpy()
        off = np.concatenate([[0], np.cumsum(c)])
        for q in range(G):
            buckets[q].append(s[off[q]:off[q + 1]])
    for q in range(G):
        recv = L.to_device(np.concatenate(buckets[q]))
        assert recv.shape[0] == M_q
        out = L.empty((M_q, d), torch.float64)
        L.call("tw_row_unpack", L.ptr(recv), M_q, d, L.ptr(out), L.stream_handle())
        assert np.array_equal(out.cpu().numpy(), X[rows[q * M_q:(q + 1) * M_q]])


@pytest.mark.parametrize("mode", ["replay", "device"])
def test_logistic_learning_matches_restatement(gpu, golden, mode):
    """learning_process(..., loss="logistic") — the pairwise-logistic SGD BASELINE.json names
    (no reference implementation, parity pinned against the oracle's
    restatement) — follows the oracle's trajectory within 1e-10."""
    import tuplewise.learning as lr
    from oracle import oracle as O
    logging.disable(logging.CRITICAL)
    p = _p_learn(golden, n_it=80)
    traj = []
    np.random.seed(41)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=traj,
                        rng_mode=mode, loss="logistic")
    np.random.seed(41)
    if mode == "replay":
        ws, _ = O.learning_trajectory(golden["learn/X"], golden["learn/Z"], p, loss="logistic")
    else:
        seed = int(np.random.randint(0, 2 ** 63 - 1, dtype=np.int64))
        ws, _ = O.device_rng_learning_trajectory(golden["learn/X"], golden["learn/Z"], p, seed,
                                                 loss="logistic")
    np.testing.assert_allclose(np.stack(traj), np.stack(ws), rtol=1e-10, atol=1e-14)
    assert len(p["tc_AUC"]) == len(p["iter"]) and np.all(np.isfinite(p["tc_AUC"]))


def test_replay_segments_graphs_match_reference(gpu, golden):
    """Replay mode without trajectory capture: the steps between reshuffles/evaluations are
    drawn in one native call and replayed as hipGraphs.  The evaluation lists (w at every
    evaluation) match the reference's golden run as in the per-step path, graphs and eager
    launches agree bit for bit, and the NumPy RNG ends in the reference's state."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for graphs in (True, False):
        p = _p_learn(golden)
        np.random.seed(2024)
        lr.learning_process(golden["learn/X"], golden["learn/Z"], p, graphs=graphs)
        out[graphs] = (p, np.random.get_state()[1].copy(), np.random.get_state()[2])
        for k in ("iter", "norm_w"):
            np.testing.assert_allclose(p[k], golden[f"learn/{k}"], rtol=1e-10)
        for k in ("bc_AUC", "tc_AUC"):
            np.testing.assert_allclose(p[k], golden[f"learn/{k}"], rtol=1e-9)
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][0][k] == out[False][0][k], k
    assert np.array_equal(out[True][1], out[False][1]) and out[True][2] == out[False][2]
    # the per-step (trajectory) path leaves the same RNG state
    p = _p_learn(golden)
    np.random.seed(2024)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=[])
    assert np.array_equal(np.random.get_state()[1], out[True][1])
    assert p["norm_w"] == out[True][0]["norm_w"]


@pytest.mark.parametrize("mode", ["replay", "device"])
def test_complete_gradient_learning(gpu, golden, mode):
    """learning_process(..., gradient="complete") (extension): every step uses all pairs of
    every shard; the trajectory follows the oracle's complete-block restatement, graphs and
    eager launches agree."""
    import tuplewise.learning as lr
    from oracle import oracle as O
    logging.disable(logging.CRITICAL)
    p = _p_learn(golden, n_it=40)
    traj = []
    np.random.seed(5)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p, trajectory=traj,
                        rng_mode=mode, gradient="complete", loss="logistic")
    X, Z = golden["learn/X"], golden["learn/Z"]
    np.random.seed(5)
    if mode == "replay":
        O.SWR_divide(X, Z, p["N"])  # the reference's redundant first draw
    else:
        seed = int(np.random.randint(0, 2 ** 63 - 1, dtype=np.int64))
    w, dw, ws = p["w_init"], 0, []
    kx, kz = int(X.shape[0] / p["N"]), int(Z.shape[0] / p["N"])
    for i in range(p["n_it"]):
        if i % p["reshuffle_mod"] == 0:
            if mode == "replay":
                X_s, Z_s = O.SWR_divide(X, Z, p["N"])
            else:
                X_s = [X[O._mulhi64(O._sgd_draw(seed, i, np.arange(kx), s, 0x40000000)[0],
                                    X.shape[0])] for s in range(p["N"])]
                Z_s = [Z[O._mulhi64(O._sgd_draw(seed, i, np.arange(kz), s, 0x20000000)[0],
                                    Z.shape[0])] for s in range(p["N"])]
        ws.append(np.array(w, copy=True))
        g = O.UN_split(X_s, Z_s, O.grad_complete_block(w, p["margin"], "logistic"))
        w, dw = O.sgd_step(w, dw, g, p["reg"], p["learning_rate"])
    np.testing.assert_allclose(np.stack(traj), np.stack(ws), rtol=1e-10, atol=1e-14)
    out = []
    for graphs in (True, False):
        q = _p_learn(golden, n_it=40)
        np.random.seed(5)
        lr.learning_process(X, Z, q, rng_mode=mode, gradient="complete", graphs=graphs)
        out.append(q["norm_w"])
    assert out[0] == out[1]


@pytest.mark.parametrize("loss", ["hinge", "logistic"])
@pytest.mark.parametrize("optim", ["momentum", "SGD"])
def test_fused_sgd_step_equals_grad_plus_update(gpu, golden, loss, optim):
    """tw_sgd_step (the previous step's update fused into the gradient launch, ping-pong
    w/dw/grads slots) gives the bits of one gradient + one update launch per step: device
    and replay draws, segments of 1, 2 and 7 steps, eager and hipGraph."""
    import torch
    import tuplewise.learning as lr
    X, Z, w0 = golden["learn/X"], golden["learn/Z"], golden["learn/w0"]
    N, B = 10, 20
    rs = np.random.RandomState(3)
    kx, kz = X.shape[0] // N, Z.shape[0] // N

    def run(fused, mode, graphs):
        eng = lr.SGDEngine(X, Z, w0, N, B, 1, 0.05, 0.01, optim, loss=loss)
        assert eng.fused  # d = 10, N*d = 100: the fusable shape
        eng.fused = fused
        ws = []
        if mode == "device":
            eng.enable_device_rng(12345)
            for n, resh in ((1, True), (2, False), (7, True), (7, False)):
                eng.run_segment(n, resh, graphs)
                ws.append(eng.w_host())
        else:
            rr = np.random.RandomState(9)
            eng.set_shards([rr.randint(0, X.shape[0], kx) for _ in range(N)],
                           [rr.randint(0, Z.shape[0], kz) for _ in range(N)])
            for tag, n in enumerate((1, 2, 7)):
                d = np.stack([np.stack([rr.randint(0, kx, (N, B)), rr.randint(0, kz, (N, B))])
                              for _ in range(n)]).astype(np.int64)
                eng.run_replay_segment(torch.from_numpy(d).cuda(), n, graphs, tag)
                ws.append(eng.w_host())
        torch.cuda.synchronize()
        return np.stack(ws), eng.dw.cpu().numpy()

    for mode in ("device", "replay"):
        ref = run(False, mode, False)
        assert np.all(np.isfinite(ref[0])) and np.abs(ref[0][-1] - w0).max() > 0
        for graphs in (False, True):
            got = run(True, mode, graphs)
            assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), \
                (mode, graphs)


def test_same_as_batch_monitor_matches_reference(gpu, golden, monkeypatch):
    """evaluation_step's SAME_AS_BATCH branch (make_exps.py:154-160) on the device, against the
    reference's own run with TYPE_TRAIN_MONITOR = "SAME_AS_BATCH" (tests/golden/make_golden.py
    section 5b): bc/br on the current shards, tr/tc on the test set."""
    import tuplewise.learning as lr
    monkeypatch.setattr(lr, "TYPE_TRAIN_MONITOR", "SAME_AS_BATCH")
    p = _p_learn(golden)
    p["n_it"] = 120
    logging.disable(logging.CRITICAL)
    np.random.seed(2025)
    lr.learning_process(golden["learn/X"], golden["learn/Z"], p)
    for k in ("iter", "norm_w"):
        np.testing.assert_allclose(p[k], golden[f"learn_sab/{k}"], rtol=1e-10)
    for k in ("bc_AUC", "tc_AUC"):
        np.testing.assert_allclose(p[k], golden[f"learn_sab/{k}"], rtol=1e-9)
    for k in ("br_AUC", "tr_AUC"):
        np.testing.assert_allclose(p[k], golden[f"learn_sab/{k}"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("layout", ["replicated", "partitioned"])
def test_same_as_batch_device_rng_equals_host_formula(gpu, golden, monkeypatch, layout):
    """Device-RNG mode: the device SAME_AS_BATCH statistics equal the reference formula
    (UN_split of conv_AUC / Un over X_s.dot(w)) evaluated on the same shards and w."""
    import torch
    import tuplewise.compute_stats as cs
    import tuplewise.learning as lr
    from oracle import oracle as O
    X, Z = golden["learn/X"], golden["learn/Z"]
    w = golden["learn/w0"]
    eng = lr.SGDEngine(X, Z, w, 10, 20, 1, 0.05, 0.01, "momentum", x_layout=layout)
    eng.enable_device_rng(321)
    eng.reshuffle_device()
    torch.cuda.synchronize()
    bc, br = lr._same_as_batch_device(eng.batch_view(), eng.w, 1, "hinge")
    if layout == "partitioned":
        rx, rz = eng.rows_all_x.cpu().numpy(), eng.rows_all_z.cpu().numpy()
    else:
        rx, rz = eng.rows_x.cpu().numpy(), eng.rows_z.cpu().numpy()
    sc_X = [X[r].dot(w) for r in rx]
    sc_Z = [Z[r].dot(w) for r in rz]
    want_bc = O.UN_split(sc_X, sc_Z, O.conv_AUC(1))
    want_br = O.UN_split(sc_X, sc_Z, lambda x, z: O.cs_Un(x, z, kernel="AUC"))
    assert np.isclose(bc, want_bc, rtol=1e-12) and abs(br - want_br) < 1e-12
    assert 0.0 <= br <= 1.0 and cs.Un is not None


@pytest.mark.parametrize("mode,fused", [("replay", True), ("device", True), ("replay", False),
                                        ("device", False)])
def test_deferred_evaluations_equal_synchronous(gpu, golden, mode, fused, monkeypatch):
    """learning.DEFER_EVALS: the loop enqueues each evaluation's device part and runs its host
    part once the statistics are back — the evaluation lists (and the log) are those of the
    synchronous evaluation, bit for bit; so is the final NumPy RNG state.  fused=False: the
    evaluation takes the separate launches, which run on the loop's stream instead of beside
    the next persistent segment."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    monkeypatch.setattr(lr, "EVAL_FUSED", fused)
    out = {}
    for defer in (True, False):
        monkeypatch.setattr(lr, "DEFER_EVALS", defer)
        p = _p_learn(golden, n_it=200)
        np.random.seed(77)
        lr.learning_process(golden["learn/X"], golden["learn/Z"], p, rng_mode=mode)
        out[defer] = (p, np.random.get_state()[2])
    for k in ("iter", "norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        a, b = np.array(out[True][0][k]), np.array(out[False][0][k])
        assert np.array_equal(a, b), (k, np.nonzero(a != b), a[a != b], b[a != b])
    assert len(out[True][0]["iter"]) == 8 and out[True][1] == out[False][1]


@pytest.mark.parametrize("mode", ["replay", "device"])
def test_narrow_segment_kernel_same_trajectory(gpu, golden, mode, monkeypatch):
    """learning.NARROW_SEGMENT (the persistent narrow segment kernel, on by default, DESIGN.md
    §4.4e): the same w at every evaluation as one launch per step, bit for bit."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for seg in (True, False):
        monkeypatch.setattr(lr, "NARROW_SEGMENT", seg)
        p = _p_learn(golden, n_it=200)
        np.random.seed(78)
        lr.learning_process(golden["learn/X"], golden["learn/Z"], p, rng_mode=mode)
        out[seg] = p["norm_w"]
    assert out[True] == out[False]


def test_deferred_evals_slot_reuse(gpu):
    """_DeferredEvals with fewer pinned slots than evaluations in flight: every host part runs
    once, in push order, with the values the device held at its push (slots are reused only
    after their copy has landed)."""
    import torch
    import tuplewise.learning as lr
    w = torch.zeros(5, dtype=torch.float64, device="cuda")
    res = torch.zeros(4, dtype=torch.float64, device="cuda")
    d = lr._DeferredEvals(w, (5,), slots=3)
    seen = []
    for i in range(20):
        res.fill_(float(i))
        w.fill_(-float(i))
        d.push(i, res, w, lambda j, r, ww: seen.append((j, r.tolist(), ww.tolist())))
    d.drain()
    assert [s[0] for s in seen] == list(range(20))
    for j, r, ww in seen:
        assert r == [float(j)] * 4 and ww == [-float(j)] * 5


@pytest.mark.parametrize("loss", ["hinge", "logistic"])
@pytest.mark.parametrize("mode", ["replay", "device"])
def test_fused_evaluation_equals_separate_launches(gpu, golden, loss, mode, monkeypatch):
    """learning.EVAL_FUSED (evaluation_step's FIXED_PAIRS statistics in two launches,
    tw_eval_small) against the separate GEMV / pair-sum / count launches: the same lists bit
    for bit (the fused kernel runs the same blocks and reduces in the same order); the replay
    hinge run also against the reference's golden lists.  Out-of-range monitor pairs raise
    IndexError instead of reading past the scores."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(lr, "EVAL_FUSED", fused)
        p = _p_learn(golden)
        np.random.seed(2024)
        lr.learning_process(p["train_X"], p["train_Z"], p, rng_mode=mode, loss=loss)
        out[fused] = p
    for k in ("iter", "norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][k] == out[False][k], k
    if mode == "replay" and loss == "hinge":
        q = out[True]
        np.testing.assert_allclose(q["norm_w"], golden["learn/norm_w"], rtol=1e-10)
        for k in ("bc_AUC", "tc_AUC"):
            np.testing.assert_allclose(q[k], golden[f"learn/{k}"], rtol=1e-9)
        for k in ("br_AUC", "tr_AUC"):
            np.testing.assert_allclose(q[k], golden[f"learn/{k}"], rtol=0, atol=1e-12)
    monkeypatch.setattr(lr, "EVAL_FUSED", True)
    p = _p_learn(golden, n_it=3)
    p["train_mon_pairs"] = [(0, 0), (len(p["train_X"]), 0)]
    with pytest.raises(IndexError):
        lr.evaluation_step(0, None, None, p["w_init"], p)
