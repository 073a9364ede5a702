"""Host-side logic of the drop-in layer (no GPU): NumPy dtype promotion for the pair
predicates, the prop-SWOR layout, and the block planner's RNG consumption order."""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.mark.parametrize("dx,dz", [(np.float64, np.float64), (np.int64, np.float64),
                                   (np.float32, np.float64), (np.int32, np.int64),
                                   (np.uint64, np.uint64), (np.uint8, np.uint16),
                                   (np.bool_, np.bool_), (np.int64, np.uint64)])
def test_compare_operands_preserve_numpy_order(tw, dx, dz):
    from tuplewise import _engine as E
    rng = np.random.RandomState(0)
    if np.dtype(dx).kind == "b":
        X, Z = rng.rand(50) > 0.5, rng.rand(40) > 0.5
    else:
        hi = 2 ** 62 if np.dtype(dx).itemsize == 8 and np.dtype(dx).kind in "iu" else 100
        X = rng.randint(0, min(hi, np.iinfo(np.int64).max), 50).astype(dx) if \
            np.dtype(dx).kind in "iu" else rng.normal(size=50).astype(dx)
        Z = rng.randint(0, min(hi, np.iinfo(np.int64).max), 40).astype(dz) if \
            np.dtype(dz).kind in "iu" else rng.normal(size=40).astype(dz)
    x, z, code = E.compare_operands(X, Z)
    want = X.reshape(-1, 1) > Z.reshape(1, -1)
    got = x.reshape(-1, 1) > z.reshape(1, -1)
    assert np.array_equal(got, want)


def test_subtract_gt_modes(tw):
    from tuplewise import _engine as E
    x, z, code, mode = E.subtract_gt_operands(np.array([1, 2], np.int64), np.array([3], np.int64))
    assert mode == "gt"  # int64 that cannot wrap: the plain ordered comparison
    _, _, _, mode = E.subtract_gt_operands(np.array([2 ** 62, -2 ** 63], np.int64),
                                           np.array([-2 ** 62 - 1], np.int64))
    assert mode == "subgt"  # 2^62 - (-2^62 - 1) wraps in int64
    _, _, _, mode = E.subtract_gt_operands(np.array([1, 2], np.uint8), np.array([3], np.uint8))
    assert mode == "ne"  # uint8: x - z wraps to >= 0, so "> 0" means "!="
    _, _, _, mode = E.subtract_gt_operands(np.array([1.0]), np.array([3], np.int64))
    assert mode == "gt"
    _, _, _, mode = E.subtract_gt_operands(np.array([1, 2], np.int8), np.array([3], np.int8))
    assert mode == "gt"  # cannot wrap for these values
    with pytest.raises(NotImplementedError):
        E.subtract_gt_operands(np.array([100], np.int8), np.array([-100], np.int8))
    with pytest.raises(TypeError):
        E.subtract_gt_operands(np.array([True]), np.array([False]))


@pytest.mark.parametrize("nx,nz,N", [(1000, 1000, 10), (100, 7, 10), (7, 100, 10),
                                     (1001, 999, 7), (5, 5, 10)])
def test_prop_swor_layout_matches_reference_slicing(tw, nx, nz, N):
    from tuplewise.device import prop_swor_layout
    x_off, z_off, keep = prop_swor_layout(nx, nz, N)
    X, Z = np.arange(nx), np.arange(nz)
    X_rem, Z_rem = X, Z
    tau, k = int((nx + nz) / N), int(nx / N)
    for s in range(N):  # estimation-experiment/main.py:48-64 with prop-SWOR
        assert keep[s] == (k not in (0, tau))
        assert np.array_equal(X[x_off[s]:x_off[s + 1]], X_rem[:k])
        assert np.array_equal(Z[z_off[s]:z_off[s + 1]], Z_rem[:tau - k])
        X_rem, Z_rem = X_rem[k:], Z_rem[tau - k:]


class _Recorder:
    """A block spec whose draws mimic cs.UB; evaluate returns the block sizes."""

    def __init__(self, B):
        self.B = B

    def draw(self, nx, nz):
        return np.random.randint(0, nx, self.B), np.random.randint(0, nz, self.B)

    def evaluate(self, X, Z, blocks):
        return [float(b.nx() * 1000 + b.nz() + b.aux[0].sum() + b.aux[1].sum()) for b in blocks]


@pytest.mark.parametrize("st", ["SWOR", "prop-SWOR", "prop-SWR"])
@pytest.mark.parametrize("variant", ["cs", "est"])
def test_block_planner_rng_order(tw, st, variant):
    """run_un must consume the global RNG exactly like the reference's serial loop."""
    from tuplewise import _blocks as Bk
    rng = np.random.RandomState(1)
    X, Z = rng.normal(size=300), rng.normal(size=120)
    B = 17
    spec = _Recorder(B)

    def f_ref(x, z):  # the reference-protocol twin of the spec
        ix = np.random.randint(0, x.shape[0], B)
        iz = np.random.randint(0, z.shape[0], B)
        return float(x.shape[0] * 1000 + z.shape[0] + ix.sum() + iz.sum())

    def f_tagged(x, z):
        raise AssertionError("tagged block functions are planned, not called")
    f_tagged._tw_block = spec

    X1, Z1, X2, Z2 = X.copy(), Z.copy(), X.copy(), Z.copy()
    np.random.seed(3)
    want = O.UN(X1, Z1, 9, f_ref, st, variant=variant)
    probe_want = np.random.randint(0, 2 ** 31 - 1)
    np.random.seed(3)
    got = Bk.run_un(X2, Z2, 9, f_tagged, st, variant=variant)
    probe_got = np.random.randint(0, 2 ** 31 - 1)
    assert got == want and probe_got == probe_want
    assert np.array_equal(X1, X2) and np.array_equal(Z1, Z2)


def test_load_preprocess_data_matches_reference(tw, golden):
    """make_exps.py:51-93 incl. the `~ind` train-split quirk, vs the reference's own output."""
    import tuplewise.learning as lr
    out = lr.load_preprocess_data({"X": golden["pre/X"], "y": golden["pre/y"]})
    for got, k in zip(out, ("Z_train", "X_train", "Z_test", "X_test")):
        assert np.array_equal(got, golden[f"pre/{k}"]), k


def test_load_preprocess_constant_column_raises(tw):
    import tuplewise.learning as lr
    X = np.ones((100, 3))
    X[:, 1] = np.arange(100)
    y = np.where(np.arange(100) % 10 == 0, 1, -1)
    with pytest.raises(ValueError, match="constant var"):
        lr.load_preprocess_data({"X": X, "y": y})


def test_multi_device_split_and_device_list(monkeypatch):
    """tuplewise._multi (single-process multi-device drop-in path): contiguous, balanced block
    groups; the device list from set_devices / TW_DEVICES."""
    from tuplewise import _multi as M
    w = [5, 1, 1, 1, 5, 1, 1, 1, 5, 1]
    g = M.split(w, 3)
    assert g[0][0] == 0 and g[-1][1] == len(w)
    assert all(a[1] == b[0] for a, b in zip(g, g[1:]))
    loads = [sum(w[a:b]) for a, b in g]
    assert max(loads) - min(loads) <= 5
    assert M.split([], 4) == [(0, 0)] * 4
    assert [b - a for a, b in M.split([1, 1], 4)].count(0) == 2
    monkeypatch.setenv("TW_DEVICES", "0,0,1")
    assert M.devices() == [0, 0, 1]
    M.set_devices([2, 3])
    try:
        assert M.devices() == [2, 3]
        assert M.slots_for(10, 5) is None  # below MIN_WORK: one device
        assert M.slots_for(1 << 40, 1) is None  # one block: nothing to spread
        assert M.slots_for(1 << 40, 5) == [2, 3]
    finally:
        M.set_devices(None)
    # one rank of a torchrun job: only its own GPU, never the other ranks'
    monkeypatch.delenv("TW_DEVICES")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    import torch
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 5)
    assert M.devices() == [5]
    assert M.slots_for(1 << 40, 5) is None


def test_learning_engine_device_selection(monkeypatch):
    """learning_process's device choice (learning._engine_devices): explicit lists are used
    (trimmed so the shards split evenly), the automatic choice spreads only steps that gather
    >= 1 GiB of rows, and partitioned / complete / multi-rank runs stay on one device."""
    import tuplewise.learning as lr
    from tuplewise import _multi as M
    f = lr._engine_devices
    assert f([0, 1], 10, 20, 10, None, "replicated", "incomplete") == [0, 1]
    assert f([0, 1, 2], 10, 20, 10, None, "replicated", "incomplete") == [0, 1]  # 10 % 3
    assert f([0], 10, 20, 10, None, "replicated", "incomplete") is None
    with pytest.raises(ValueError):
        f([0, 1], 10, 20, 10, None, "partitioned", "incomplete")
    assert f(None, 10, 20, 10, None, "replicated", "complete") is None
    monkeypatch.setattr(M, "_DEVICES", [0, 1, 2, 3, 4, 5, 6, 7])
    # C5 at B = 100: 256*100*512*16 B = 0.2 GB per step -> one device; at B = 4096: 8.6 GB
    assert f(None, 256, 100, 512, None, "replicated", "incomplete") is None
    assert f(None, 256, 4096, 512, None, "replicated", "incomplete") == list(range(8))
    assert f(None, 100, 4096, 512, None, "replicated", "incomplete") == [0, 1, 2, 3, 4]
