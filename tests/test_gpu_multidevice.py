"""Single-process multi-device path of the drop-in API (tuplewise._multi).

An unchanged reference-style call (est.UnNT, est.replicate, cs.UnNBT, cs.UnNT) spreads its
blocks over device slots; the values must be bit-identical to one device (and to the oracle).
On a one-GPU box the slots are [0, 0, 0]: the same partition, uploads, streams and gathers
run, with host gathers (RCCL needs distinct devices); the RCCL all-gather itself is checked
on a one-device communicator."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def three_slots(gpu):
    from tuplewise import _multi as M
    M.set_devices([0, 0, 0], min_work=0)
    yield
    M.set_devices(None, min_work=1 << 27)


def _reference_data(seed, n=30_000, m=20_000):
    rng = np.random.RandomState(seed)
    return rng.normal(0.3, 1, n), rng.normal(0, 1, m)


@pytest.mark.parametrize("call", ["est_UnNT", "cs_UnNT_prod", "cs_UnNBT_AUC", "cs_UnNBT_gini_SWR",
                                  "est_replicate", "est_UnN_SWOR_int"])
def test_multi_slot_equals_single_device_and_oracle(three_slots, call):
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    from tuplewise import _multi as M
    X, Z = _reference_data(7)
    if call == "est_UnN_SWOR_int":
        X, Z = np.round(X * 3).astype(np.int64), np.round(Z * 3).astype(np.int64)

    def run(mod_est, mod_cs, Xa, Za):
        if call == "est_UnNT":
            return mod_est.UnNT(Xa, Za, 12, 3, "prop-SWOR")
        if call == "cs_UnNT_prod":
            return mod_cs.UnNT(Xa, Za, 12, 2, "SWOR", kernel="prod")
        if call == "cs_UnNBT_AUC":
            return mod_cs.UnNBT(Xa, Za, 12, 5000, 2, "prop-SWOR", kernel="AUC")
        if call == "cs_UnNBT_gini_SWR":
            return mod_cs.UnNBT(Xa, Za, 12, 3000, 2, "prop-SWR", kernel="gini")
        if call == "est_UnN_SWOR_int":
            return mod_est.UnN(Xa, Za, 9, "SWOR")
        return None

    if call == "est_replicate":
        rs = np.random.RandomState(3)
        gx = lambda: rs.normal(0.2, 1, 4000)  # noqa: E731
        gz = lambda: rs.normal(0, 1, 3000)  # noqa: E731
        np.random.seed(5)
        got = est.replicate(est.UnNT, gx, gz, 6, 10, 2, "prop-SWOR")
        M.set_devices([0])
        rs = np.random.RandomState(3)
        np.random.seed(5)
        want = est.replicate(est.UnNT, gx, gz, 6, 10, 2, "prop-SWOR")
        assert got == want
        return
    Xa, Za = X.copy(), Z.copy()
    np.random.seed(11)
    got = run(est, cs, Xa, Za)
    M.set_devices([0])
    Xb, Zb = X.copy(), Z.copy()
    np.random.seed(11)
    single = run(est, cs, Xb, Zb)
    Xo, Zo = X.copy(), Z.copy()
    np.random.seed(11)
    oracle_mods = (type("E", (), {"UnNT": staticmethod(O.est_UnNT), "UnN": staticmethod(O.est_UnN)}),
                   type("C", (), {"UnNT": staticmethod(O.cs_UnNT),
                                  "UnNBT": staticmethod(O.cs_UnNBT)}))
    want = run(*oracle_mods, Xo, Zo)
    assert got == single
    assert np.array_equal(Xa, Xb) and np.array_equal(Za, Zb)
    if call.startswith("cs_UnNT_prod") or "gini" in call:
        assert np.isclose(got, want, rtol=1e-12, atol=0)  # float sums: NumPy's pairwise order
    else:
        assert got == want
    assert np.array_equal(Xa, Xo)


def test_rccl_communicator_one_device(gpu):
    """tw_comm_init / tw_allgather_u64 / _f64 over a one-device communicator (the box has
    one GPU): RCCL is found in the process and the all-gather copies in rank order."""
    import torch
    from tuplewise import _lib as L
    c = ctypes.c_int32(-1)
    dev = (ctypes.c_int32 * 1)(0)
    L.call("tw_comm_init", 1, dev, ctypes.byref(c))
    try:
        for dt, fn in ((torch.int64, "tw_allgather_u64"), (torch.float64, "tw_allgather_f64")):
            send = torch.arange(17, dtype=dt, device="cuda") * 3
            recv = torch.zeros(17, dtype=dt, device="cuda")
            P = ctypes.c_void_p * 1
            s = torch.cuda.current_stream().cuda_stream
            L.call(fn, c.value, P(send.data_ptr()), P(recv.data_ptr()), 17, P(s))
            assert torch.equal(recv, send)
    finally:
        L.call("tw_comm_destroy", c.value)
    with pytest.raises(ValueError):
        two = (ctypes.c_int32 * 2)(0, 0)
        L.call("tw_comm_init", 2, two, ctypes.byref(c))


# ------------------------------------------------------------ learning over device slots
def _learn_p(golden, n_it=60):
    return {"n_it": n_it, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
            "learning_rate": 0.01, "eval_mod": 25, "w_init": golden["learn/w0"],
            "test_X": golden["learn/test_X"], "test_Z": golden["learn/test_Z"],
            "train_mon_pairs": [tuple(p) for p in golden["learn/mon"]],
            "train_X": golden["learn/X"], "train_Z": golden["learn/Z"]}


@pytest.mark.parametrize("mode", ["replay", "device"])
@pytest.mark.parametrize("per_step", [False, True])
def test_learning_process_over_slots_equals_one_device(gpu, golden, mode, per_step):
    """learning_process(devices=[0, 0]): two slots (own streams) own 5 shards each, gather the
    shard gradients in shard order and apply the same update — the evaluation history and the
    w trajectory are identical to one device, in replay and device-RNG mode, per step and in
    segments."""
    import tuplewise.learning as lr
    X, Z = golden["learn/X"], golden["learn/Z"]
    out = []
    for devices in (None, [0, 0]):
        p = _learn_p(golden)
        traj = [] if per_step else None
        np.random.seed(11)
        lr.learning_process(X, Z, p, rng_mode=mode, trajectory=traj, devices=devices)
        out.append((p["norm_w"], p["bc_AUC"], p["tr_AUC"], traj,
                    np.random.randint(0, 2 ** 31)))
    a, b = out
    assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2] and a[4] == b[4]
    if per_step:
        assert len(a[3]) == len(b[3]) and all(np.array_equal(u, v) for u, v in zip(a[3], b[3]))


def test_learning_devices_wide_rows_over_three_slots(gpu):
    """d = 64 wide rows, N = 9 shards over the slots [0, 0, 0], device RNG, against one
    device: the same history."""
    import tuplewise.learning as lr
    rng = np.random.RandomState(4)
    n, d = 3000, 64
    X = rng.normal(0.3, 1.0, size=(n, d))
    Z = rng.normal(0.0, 1.0, size=(n, d))
    hist = []
    for devices in (None, [0, 0, 0]):
        mon = np.random.RandomState(1)
        p = {"N": 9, "B": 64, "margin": 1.0, "reg": 0.01, "learning_rate": 0.05, "n_it": 40,
             "reshuffle_mod": 10, "eval_mod": 20, "w_init": np.full((d, 1), 0.01),
             "test_X": X[:500], "test_Z": Z[:500], "train_X": X, "train_Z": Z,
             "train_mon_pairs": list(zip(mon.randint(0, n, 300), mon.randint(0, n, 300)))}
        np.random.seed(7)
        lr.learning_process(X, Z, p, rng_mode="device", devices=devices)
        hist.append((p["norm_w"], p["tr_AUC"]))
    assert hist[0] == hist[1]


@pytest.mark.parametrize("draw_ahead", [True, False])
def test_same_as_batch_replay_over_slots_reshuffle_every_step(gpu, golden, monkeypatch,
                                                                draw_ahead):
    """SAME_AS_BATCH monitoring in the pipelined replay loop over two slots (no
    batch_view: the host formula reads the SWR rows), a reshuffle and an evaluation every step:
    the pinned ring slots are refilled by the draw worker while later segments run, so the
    evaluation must read its own copy of the rows.  History equals the one-device run and the
    sequential loop (DRAW_AHEAD=False)."""
    import tuplewise.learning as lr
    monkeypatch.setattr(lr, "TYPE_TRAIN_MONITOR", "SAME_AS_BATCH")
    monkeypatch.setattr(lr, "DRAW_AHEAD", draw_ahead)
    X, Z = golden["learn/X"], golden["learn/Z"]
    out = []
    for devices in (None, [0, 0]):
        p = _learn_p(golden)
        p["n_it"], p["reshuffle_mod"], p["eval_mod"] = 40, 1, 1
        np.random.seed(13)
        lr.learning_process(X, Z, p, rng_mode="replay", devices=devices)
        out.append((p["norm_w"], p["bc_AUC"], p["br_AUC"], p["tr_AUC"]))
    for a, b in zip(*out):
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=0)
