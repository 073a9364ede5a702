"""learning_process at the reference's own shape (make_exps.py:210-214: N = 100 shards, B = 100
pairs each, eval_mod 25) on the shuttle-shaped rows of tests/golden/shapes.py, at both ends of
the paper's reshuffle sweep (learning-experiment/main.py:20): reshuffle_mod = 1 (a new SWR
draw before every step: one-step segments) and 10000 (one draw for the whole run: segments
bounded by the evaluations).  Against the reference's golden run (tests/golden/make_golden.py
section 5c): the w trajectory, every evaluation list, the NumPy RNG state — through the per-step
path AND the default production path (replay draws in segments, the persistent narrow segment
kernel, deferred evaluations, hipGraphs), with graphs and eager launches bit-identical.

Tolerances: trajectory 1e-10 relative (north_star asks 1e-5; only BLAS's dot order inside the
hinge filter differs); AUCs are counts on device GEMV scores (exact unless two scores tie
within an ulp); surrogate values 1e-9 relative."""
import logging

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODS = [1, 10000]


def _p(mod, n_it=250):
    from golden.shapes import shuttle_problem
    X, Z, tX, tZ, w0, mon = shuttle_problem()
    return X, Z, {"n_it": n_it, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": mod,
                  "reg": 0.05, "learning_rate": 0.01, "eval_mod": 25, "w_init": w0,
                  "test_X": tX, "test_Z": tZ, "train_mon_pairs": mon, "train_X": X,
                  "train_Z": Z}


def _check_lists(p, golden, mod):
    g = f"shuttle_mod{mod}"
    assert list(p["iter"]) == list(golden[f"{g}/iter"])
    np.testing.assert_allclose(p["norm_w"], golden[f"{g}/norm_w"], rtol=1e-10)
    for k in ("bc_AUC", "tc_AUC"):
        np.testing.assert_allclose(p[k], golden[f"{g}/{k}"], rtol=1e-9)
    for k in ("br_AUC", "tr_AUC"):
        np.testing.assert_allclose(p[k], golden[f"{g}/{k}"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("mod", MODS)
def test_reference_shape_trajectory(gpu, golden, mod):
    """Per-step path (trajectory capture): w before every step vs the reference's, and the
    evaluation lists."""
    import tuplewise.learning as lr
    X, Z, p = _p(mod)
    traj = []
    logging.disable(logging.CRITICAL)
    np.random.seed(3000 + mod)
    lr.learning_process(X, Z, p, trajectory=traj)
    ref = golden[f"shuttle_mod{mod}/ws"]
    got = np.stack(traj)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-10
    _check_lists(p, golden, mod)


@pytest.mark.parametrize("mod", MODS)
def test_reference_shape_default_path(gpu, golden, mod, monkeypatch):
    """The default path (no trajectory): replay segments drawn in one native call each, the
    persistent narrow segment kernel for segments of > 1 step (it must run when mod = 10000),
    deferred evaluations, hipGraphs; graphs and eager launches give the same bits, the
    evaluation lists match the reference, and the NumPy RNG ends where the per-step path (and
    the reference) leaves it."""
    import tuplewise.learning as lr
    seen = []
    orig = lr.SGDEngine._fused_steps

    def spy(self, nsteps, draws_dev=None, swr_mod=0, tables=None):
        seen.append((nsteps, self.narrow_seg, tables))
        return orig(self, nsteps, draws_dev, swr_mod, tables)

    monkeypatch.setattr(lr.SGDEngine, "_fused_steps", spy)
    logging.disable(logging.CRITICAL)
    out = {}
    for graphs in (True, False):
        X, Z, p = _p(mod)
        np.random.seed(3000 + mod)
        lr.learning_process(X, Z, p, graphs=graphs)
        _check_lists(p, golden, mod)
        st = np.random.get_state()
        out[graphs] = (p, st[1].copy(), st[2])
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][0][k] == out[False][0][k], k
    assert np.array_equal(out[True][1], out[False][1]) and out[True][2] == out[False][2]
    # segments end at evaluations only (eval_mod 25): at mod 1 they run through a reshuffle
    # before every step, the kernel switching row tables by step
    assert any(n > 1 and nseg for n, nseg, _ in seen), seen[:5]
    if mod == 1:
        assert all(tab is not None and tab[1] == 1 for n, _, tab in seen if n > 1), seen[:5]
        assert max(n for n, _, _ in seen) == 25, seen[:5]
    X, Z, p = _p(mod)
    np.random.seed(3000 + mod)
    lr.learning_process(X, Z, p, trajectory=[])
    assert np.array_equal(np.random.get_state()[1], out[True][1])
    assert p["norm_w"] == out[True][0]["norm_w"]


@pytest.mark.parametrize("mod", MODS)
def test_reference_shape_device_rng_segments(gpu, golden, mod, monkeypatch):
    """rng_mode='device' at the same shape (not bit-comparable with NumPy's stream): the
    persistent narrow segment and the per-step launches give the same bits, and the loop ends
    with finite statistics of the reference's schema."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for seg in (True, False):
        monkeypatch.setattr(lr, "NARROW_SEGMENT", seg)
        X, Z, p = _p(mod)
        np.random.seed(44)
        lr.learning_process(X, Z, p, rng_mode="device")
        out[seg] = p
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][k] == out[False][k], k
        assert len(out[True][k]) == 10 and np.all(np.isfinite(out[True][k]))


@pytest.mark.parametrize("mod", MODS)
def test_reference_shape_draw_ahead_equals_sequential(gpu, golden, mod, monkeypatch):
    """learning.DRAW_AHEAD (the replay draws made two segments ahead by a worker thread): the
    same evaluation lists and final NumPy RNG state as the sequential loop, bit for bit."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for ahead in (True, False):
        monkeypatch.setattr(lr, "DRAW_AHEAD", ahead)
        X, Z, p = _p(mod)
        np.random.seed(3000 + mod)
        lr.learning_process(X, Z, p)
        _check_lists(p, golden, mod)
        out[ahead] = (p, np.random.get_state()[1].copy())
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][0][k] == out[False][0][k], k
    assert np.array_equal(out[True][1], out[False][1])


def test_engine_cache_reuse(gpu, golden, monkeypatch):
    """learning.ENGINE_CACHE: a second replay call of the same shapes reuses the engine (its
    buffers, draw buffers and captured segment graphs) and still gives the reference's lists;
    a call on other rows of the same shapes equals a fresh engine's bit for bit, also after a
    device-RNG run and a call of other shapes in between."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    monkeypatch.setattr(lr, "ENGINE_CACHE", True)
    mod = 10000
    X, Z, p = _p(mod)
    np.random.seed(3000 + mod)
    lr.learning_process(X, Z, p)
    _check_lists(p, golden, mod)
    eng = lr._ENGINE["eng"]
    assert eng is not None and getattr(eng, "_draws", None) is not None
    X, Z, p = _p(mod)
    np.random.seed(3000 + mod)
    lr.learning_process(X, Z, p)
    _check_lists(p, golden, mod)
    assert lr._ENGINE["eng"] is eng

    def other(seed):
        X, Z, p = _p(mod)
        r = np.random.RandomState(seed)
        X2, Z2 = X + 0.1 * r.normal(size=X.shape), Z - 0.1 * r.normal(size=Z.shape)
        p = dict(p, train_X=X2, train_Z=Z2, w_init=p["w_init"] * 0.5)
        np.random.seed(seed)
        lr.learning_process(X2, Z2, p)
        return p, np.random.get_state()[1].copy()

    a = other(7)
    assert lr._ENGINE["eng"] is eng
    X, Z, p = _p(mod)
    np.random.seed(8)
    lr.learning_process(X, Z, p, rng_mode="device")
    Xs, Zs, ps = _p(mod, n_it=30)
    np.random.seed(9)
    lr.learning_process(Xs[:5000], Zs[:500], dict(ps, N=50, B=20))
    b = other(7)
    monkeypatch.setattr(lr, "ENGINE_CACHE", False)
    c = other(7)
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert a[0][k] == b[0][k] == c[0][k], k
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[1], c[1])


@pytest.mark.parametrize("mod", MODS)
def test_native_draw_worker_equals_python_worker(gpu, golden, mod, monkeypatch):
    """learning.NATIVE_DRAWS (the replay draws made ahead by tw_draw_pipe, csrc/drawpipe.hip)
    against the Python worker thread, and learning.FUSED_SHIP (the upload captured in the
    segment graph) against separate launches: the same lists and NumPy RNG state, bit for
    bit, and the reference's lists."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for native, fused in ((True, True), (False, True), (True, False)):
        monkeypatch.setattr(lr, "NATIVE_DRAWS", native)
        monkeypatch.setattr(lr, "FUSED_SHIP", fused)
        X, Z, p = _p(mod)
        np.random.seed(3000 + mod)
        lr.learning_process(X, Z, p)
        _check_lists(p, golden, mod)
        out[native, fused] = (p, np.random.get_state()[1].copy(), np.random.get_state()[2])
    ref = out[True, True]
    for key, (p, st, pos) in out.items():
        for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
            assert p[k] == ref[0][k], (key, k)
        assert np.array_equal(st, ref[1]) and pos == ref[2], key


def test_native_draw_pipe_protocol(gpu):
    """tw_draw_pipe_*: the segments come out in NumPy's order (== Session.pairs_steps_u8 on the
    same state), a reshuffle's rows first; a pipe stopped before its last segment joins
    without hanging (its worker blocked on a buffer the main thread never shipped); a width
    the indices do not fit is refused."""
    import torch
    import tuplewise.learning as lr
    from tuplewise import _lib as L
    from tuplewise.numpy_rng import Session
    N, kx, kz, B = 7, 91, 7, 13
    n_X, n_Z = N * kx, N * kz
    mod = 5  # reshuffles at steps 0, 5, 10
    segs = [(0, 3, 1), (3, 5, 0), (5, 9, 1), (9, 10, 0), (10, 12, 1)]
    np.random.seed(11)
    want = []
    with Session() as s:
        for a, b, r in segs:
            rows = s.randint_flat(np.zeros(2 * N, np.int64),
                                  np.array([n_X] * N + [n_Z] * N, np.int64),
                                  np.array([kx] * N + [kz] * N, np.int64)) if r else None
            o = np.empty((b - a, 2, N, B), np.uint8)
            s.pairs_steps_u8(b - a, N, kx, kz, B, o)
            want.append((rows, o))
    state = np.random.get_state()
    np.random.seed(11)
    d = lr._ReplayDraws(N, kx, kz, B)
    with d.rng:
        pipe = d.native_pipe(segs, n_X, n_Z, mod)
        try:
            for j, (a, b, r) in enumerate(segs):
                rows, k = pipe.wait(j)
                got = d.seg3_np[k][:b - a].copy()
                assert np.array_equal(got, want[j][1]), j
                if r:
                    (rx, rz), _ = rows
                    assert np.array_equal(np.concatenate([rx.ravel(), rz.ravel()]), want[j][0])
                else:
                    assert rows is None
                pipe.shipped(j)
        finally:
            pipe.stop()
    assert np.array_equal(np.random.get_state()[1], state[1])
    assert np.random.get_state()[2] == state[2]
    torch.cuda.synchronize()
    # segments running through reshuffles (replay_through): the same draws, a reshuffle's rows
    # before the pairs of its step, the tables one after another in the row buffer
    tsegs = [(0, 12, 3), (12, 13, 0), (13, 20, 1)]  # reshuffles at 0, 5, 10 | - | 15
    ends = []
    for rw, view in ((8, np.int64), (2, np.uint16)):  # int64 tables, and narrowed to uint16
        np.random.seed(11)
        d3 = lr._ReplayDraws(N, kx, kz, B)
        with d3.rng:
            pipe = d3.native_pipe(tsegs, n_X, n_Z, mod, row_width=rw)
            try:
                tabs = []
                for j, (a, b, r) in enumerate(tsegs):
                    pipe.wait(j, rows=False)
                    k = j % 3
                    per = N * kx + N * kz
                    flat = d3.rows3[k][0].numpy().view(view)
                    tabs += [flat[t * per:(t + 1) * per].astype(np.int64) for t in range(r)]
                    if j == 0:
                        got = d3.seg3_np[k][:12].copy()
                        assert np.array_equal(got, np.concatenate([w[1] for w in want]))
                    pipe.shipped(j)
            finally:
                pipe.stop()
        for t, w in zip(tabs[:3], (want[0][0], want[2][0], want[4][0])):
            assert np.array_equal(t, w), rw
        assert len(tabs) == 4
        ends.append(np.random.get_state())
    assert np.array_equal(ends[0][1], ends[1][1]) and ends[0][2] == ends[1][2]
    torch.cuda.synchronize()
    # stopped early: the worker waits for segment 0's buffer to be shipped, which never happens
    d2 = lr._ReplayDraws(N, kx, kz, B)
    with d2.rng:
        pipe = d2.native_pipe(segs, n_X, n_Z, mod)
        pipe.wait(0)
        pipe.stop()
    P = __import__("ctypes").c_void_p * 3
    with pytest.raises(ValueError):
        L.call("tw_draw_pipe_start", d2.rng._key, d2.rng._pos, 1,
               np.array([1], np.int32).ctypes.data, np.array([0], np.int32).ctypes.data, 1,
               N, 300, kz, B, 300 * N, n_Z, 1, 3, P(*[0, 0, 0]), P(*[0, 0, 0]), 1, 8,
               ctypes_handle())
    with pytest.raises(ValueError):  # a phase outside the reshuffle period
        L.call("tw_draw_pipe_start", d2.rng._key, d2.rng._pos, 1,
               np.array([1], np.int32).ctypes.data, np.array([5], np.int32).ctypes.data, 5,
               N, kx, kz, B, n_X, n_Z, 1, 3, P(*[0, 0, 0]), P(*[0, 0, 0]), 1, 8,
               ctypes_handle())


def ctypes_handle():
    import ctypes
    return ctypes.byref(ctypes.c_void_p())


@pytest.mark.parametrize("mod,eval_mod,n_it", [(1, 25, 101), (7, 25, 101), (10000, 25, 76),
                                               (3, 2, 41)])
def test_swr_in_kernel_equals_row_tables(gpu, golden, mod, eval_mod, n_it, monkeypatch):
    """learning.SWR_IN_KERNEL (device RNG: the persistent narrow segment draws each reshuffle's
    SWR rows itself, segments cut at evaluations only) against the row-table path (a
    tw_swr_rows_rng launch and a new segment per reshuffle): the same statistics bit for bit,
    with reshuffles inside segments, one-step tails whose tables a segment left stale, and
    two-step segments."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    out = {}
    for swr in (True, False):
        monkeypatch.setattr(lr, "SWR_IN_KERNEL", swr)
        X, Z, p = _p(mod, n_it=n_it)
        p["eval_mod"] = eval_mod
        np.random.seed(45)
        lr.learning_process(X, Z, p, rng_mode="device")
        out[swr] = p
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][k] == out[False][k], k
    assert len(out[True]["norm_w"]) == (n_it + eval_mod - 1) // eval_mod


@pytest.mark.parametrize("mod,eval_mod,n_it,monitor", [
    (1, 25, 101, "FIXED_PAIRS"), (3, 25, 101, "FIXED_PAIRS"), (7, 10, 95, "FIXED_PAIRS"),
    (2, 25, 60, "SAME_AS_BATCH"), (5, 7, 50, "SAME_AS_BATCH"), (40, 25, 101, "FIXED_PAIRS")])
def test_replay_through_reshuffles_equals_cut_segments(gpu, golden, mod, eval_mod, n_it,
                                                      monitor, monkeypatch):
    """learning.REPLAY_THROUGH (replay segments running through their reshuffles: the SWR
    tables shipped with the segment's draws, the kernel switching tables at the reshuffle
    steps) against segments cut at every reshuffle: the same evaluation lists and final NumPy
    RNG state, bit for bit — with evaluations that coincide with reshuffles (SAME_AS_BATCH reads
    the new tables), segments that start between reshuffles, and one-step tails."""
    import tuplewise.learning as lr
    logging.disable(logging.CRITICAL)
    monkeypatch.setattr(lr, "TYPE_TRAIN_MONITOR", monitor)
    out = {}
    for through in (True, False):
        monkeypatch.setattr(lr, "REPLAY_THROUGH", through)
        X, Z, p = _p(mod, n_it=n_it)
        p["eval_mod"] = eval_mod
        np.random.seed(46)
        lr.learning_process(X, Z, p)
        out[through] = (p, np.random.get_state()[1].copy(), np.random.get_state()[2])
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert out[True][0][k] == out[False][0][k], k
    assert np.array_equal(out[True][1], out[False][1]) and out[True][2] == out[False][2]
    assert len(out[True][0]["norm_w"]) == (n_it + eval_mod - 1) // eval_mod
