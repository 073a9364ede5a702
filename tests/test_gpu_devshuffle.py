"""Device swaps of np.random.shuffle (csrc/devshuffle.hip) and the drop-in's device-shuffle path
(_blocks._run_un_repeated_device) against NumPy's own in-place shuffles and the host path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _numpy_snapshots(X, Z, T, seed):
    np.random.seed(seed)
    np.random.random(2)
    xs, zs = [], []
    X, Z = X.copy(), Z.copy()
    for _ in range(T):
        np.random.shuffle(X)
        np.random.shuffle(Z)
        xs.append(X.copy())
        zs.append(Z.copy())
    return xs, zs, np.random.randint(0, 2 ** 31, 3)


@pytest.mark.parametrize("nx,nz,dtype", [(0, 5, np.float64), (1, 1, np.float64),
                                         (2, 3, np.int64), (1000, 17, np.float64),
                                         (65537, 4099, np.int64),
                                         (1_000_000, 1_000_000, np.float64)])
@pytest.mark.parametrize("rounds,tail", [(0, 1), (0, 0), (17, 1), (40, 1)])
def test_device_shuffle_snapshots_match_numpy(gpu, nx, nz, dtype, rounds, tail):
    """T = 3 chained shuffles of X and Z on the device == NumPy's sequential in-place
    shuffles with the same stream, every state; rounds = 17 (the least allowed) forces
    resumed batches, 40 resumed batches that end in the one-workgroup tail; tail = 0 one
    launch per round throughout."""
    from tuplewise import _engine as E, _lib as L
    from tuplewise.numpy_rng import shuffle_draws32
    rs = np.random.RandomState(nx + nz)
    X = rs.normal(size=nx).astype(dtype) if dtype == np.float64 else rs.randint(-9, 9, nx)
    Z = rs.normal(size=nz).astype(dtype) if dtype == np.float64 else rs.randint(-9, 9, nz)
    X, Z = X.astype(dtype), Z.astype(dtype)
    want_x, want_z, probe = _numpy_snapshots(X, Z, 3, 11)
    np.random.seed(11)
    np.random.random(2)
    jx, jz = [], []
    for _ in range(3):
        jx.append(shuffle_draws32(nx))
        jz.append(shuffle_draws32(nz))
    assert np.array_equal(np.random.randint(0, 2 ** 31, 3), probe)
    L.call("tw_shuffle_swaps_set_rounds", rounds)
    L.call("tw_shuffle_swaps_set_tail", tail)
    try:
        xs, zs = E.shuffle_snapshots_device(L.to_device(X), L.to_device(Z), jx, jz)
    finally:
        L.call("tw_shuffle_swaps_set_rounds", 0)
        L.call("tw_shuffle_swaps_set_tail", 1)
    for k in range(3):
        assert np.array_equal(xs[k].cpu().numpy(), want_x[k])
        assert np.array_equal(zs[k].cpu().numpy(), want_z[k])


@pytest.mark.parametrize("nx,nz", [(0, 1), (3, 2), (1000, 17), (4099, 65537),
                                   (1_000_000, 1_000_000)])
@pytest.mark.parametrize("pieces", [1, 3, 4, 16])
def test_streamed_z_shuffle_matches_numpy(gpu, nx, nz, pieces):
    """DeviceShuffles.draw_push_z_streamed (the drop-in's last shuffle drawn and swapped in
    window groups: tw_np_shuffle_draws32_range + tw_shuffle_swaps_part) == NumPy's in-place
    shuffles, every state, and the RNG state after; T = 2, both Z shuffles streamed."""
    from tuplewise import _engine as E
    from tuplewise.numpy_rng import shuffle_draws32
    rs = np.random.RandomState(nx + 7 * nz)
    X, Z = rs.normal(size=nx), rs.normal(size=nz)
    want_x, want_z, probe = _numpy_snapshots(X, Z, 2, 13)
    np.random.seed(13)
    np.random.random(2)
    ds = E.DeviceShuffles(X, Z, 2)
    for _ in range(2):
        shuffle_draws32(nx, out=ds.draw_x())
        ds.push_x()
        ds.draw_push_z_streamed(pieces)
    assert np.array_equal(np.random.randint(0, 2 ** 31, 3), probe)
    xs, zs = ds.finish()
    for k in range(2):
        assert np.array_equal(xs[k].cpu().numpy(), want_x[k])
        assert np.array_equal(zs[k].cpu().numpy(), want_z[k])


def _call(fn, X, Z, seed):
    X, Z = X.copy(), Z.copy()
    np.random.seed(seed)
    v = fn(X, Z)
    return v, X, Z, np.random.randint(0, 2 ** 31, 4)


CASES = [
    ("est.UnNT prop-SWOR", lambda e, c: lambda X, Z: e.UnNT(X, Z, 8, 3, "prop-SWOR")),
    ("est.UnNT SWOR", lambda e, c: lambda X, Z: e.UnNT(X, Z, 8, 2, "SWOR")),
    ("est.UnNT prop-SWR", lambda e, c: lambda X, Z: e.UnNT(X, Z, 5, 2, "prop-SWR")),
    ("est.UnNT half", lambda e, c: lambda X, Z: e.UnNT(X, Z, 4, 2, "prop-SWOR", tie_mode="half")),
    ("est.UnN SWOR", lambda e, c: lambda X, Z: e.UnN(X, Z, 8, "SWOR")),
    ("cs.UnNT AUC", lambda e, c: lambda X, Z: c.UnNT(X, Z, 8, 3, "SWOR", kernel="AUC")),
    ("cs.UnNT prod", lambda e, c: lambda X, Z: c.UnNT(X, Z, 8, 2, "prop-SWOR", kernel="prod")),
    ("cs.UnNT gini", lambda e, c: lambda X, Z: c.UnNT(X, Z, 4, 2, "prop-SWR", kernel="gini")),
    ("cs.UnNBT AUC", lambda e, c: lambda X, Z: c.UnNBT(X, Z, 8, 5000, 3, "SWOR", kernel="AUC")),
    ("cs.UnNBT prod", lambda e, c: lambda X, Z: c.UnNBT(X, Z, 8, 3000, 2, "prop-SWR",
                                                         kernel="prod")),
    ("cs.UnN AUC", lambda e, c: lambda X, Z: c.UnN(X, Z, 8, "prop-SWOR", kernel="AUC")),
    ("cs.UnNB gini", lambda e, c: lambda X, Z: c.UnNB(X, Z, 8, 2000, "SWOR", kernel="gini")),
]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_drop_in_device_shuffles_equal_host_path(gpu, name, make):
    """The drop-in estimators with their in-place shuffles on the device (DEVICE_SHUFFLE_MIN = 0)
    and on the host: the same value (bit for bit), the same post-call arrays and the same RNG
    state — the host path being the one pinned to the reference's golden vectors."""
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    from tuplewise import _blocks as Bk
    fn = make(est, cs)
    rs = np.random.RandomState(3)
    X = np.round(rs.normal(0.3, 1, 20000), 2)  # ties for the half-ties and AUC paths
    Z = np.round(rs.normal(0, 1, 17000), 2)
    old = Bk.DEVICE_SHUFFLE_MIN
    try:
        Bk.DEVICE_SHUFFLE_MIN = 1 << 40
        host = _call(fn, X, Z, 21)
        Bk.DEVICE_SHUFFLE_MIN = 0
        dev = _call(fn, X, Z, 21)
    finally:
        Bk.DEVICE_SHUFFLE_MIN = old
    assert dev[0] == host[0] and type(dev[0]) is type(host[0])
    for a, b in zip(dev[1:], host[1:]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("early,pieces,threaded", [(False, 0, False), (True, 0, False),
                                                   (False, 4, False), (True, 16, False),
                                                   (False, 0, True), (True, 4, True)])
@pytest.mark.parametrize("name", ["est.UnNT prop-SWOR", "est.UnNT SWOR", "est.UnNT half",
                                  "cs.UnNT AUC", "est.UnNT prop-SWR"])
def test_drop_in_pipelining_equals_host_path(gpu, name, early, pieces, threaded, monkeypatch):
    """The drop-in's round-5 pipelining switched on and off (_blocks.EARLY_COUNTS: step k
    counted while step k + 1 is drawn; STREAM_LAST_SHUFFLE: the last shuffle in parts;
    THREADED_LAUNCHES: uploads and launches on the launcher thread): the value, the post-call
    arrays and the RNG state equal the host path's in every setting."""
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    from tuplewise import _blocks as Bk
    fn = dict(CASES)[name](est, cs)
    rs = np.random.RandomState(4)
    X = np.round(rs.normal(0.3, 1, 30001), 2)
    Z = np.round(rs.normal(0, 1, 25000), 2)
    monkeypatch.setattr(Bk, "DEVICE_SHUFFLE_MIN", 1 << 40)
    host = _call(fn, X, Z, 5)
    monkeypatch.setattr(Bk, "DEVICE_SHUFFLE_MIN", 0)
    monkeypatch.setattr(Bk, "EARLY_COUNTS", early)
    monkeypatch.setattr(Bk, "STREAM_LAST_SHUFFLE", pieces)
    monkeypatch.setattr(Bk, "THREADED_LAUNCHES", threaded)
    dev = _call(fn, X, Z, 5)
    assert dev[0] == host[0] and type(dev[0]) is type(host[0])
    for a, b in zip(dev[1:], host[1:]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("name", ["est.UnNT prop-SWOR", "cs.UnNBT AUC"])
def test_device_shuffles_kept_with_several_devices(gpu, name, monkeypatch):
    """With several device slots visible (slots [0, 0] on the one-GPU box, as TW_DEVICES=0,0
    gives), est.UnNT / cs.UnNBT at >= 2^16 items per sample keep the device-shuffle path (the
    sorted count of their blocks is far below the multi-device threshold): it
    runs, and gives the one-device value, post-call arrays and RNG state bit for bit."""
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    from tuplewise import _blocks as Bk, _multi as M
    fn = dict(CASES)[name](est, cs)
    rs = np.random.RandomState(4)
    X = rs.normal(0.3, 1, 1 << 17)
    Z = rs.normal(0, 1, (1 << 16) + 5)
    one = _call(fn, X, Z, 31)
    taken = []
    orig = Bk._run_un_repeated_device
    monkeypatch.setattr(Bk, "_run_un_repeated_device",
                        lambda *a, **k: taken.append(1) or orig(*a, **k))
    M.set_devices([0, 0])
    try:
        two = _call(fn, X, Z, 31)
    finally:
        M.set_devices(None)
    assert taken, "the device-shuffle path was not taken with two slots"
    assert two[0] == one[0]
    for a, b in zip(two[1:], one[1:]):
        assert np.array_equal(a, b)
