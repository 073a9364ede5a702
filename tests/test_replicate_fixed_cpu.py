"""estimation.replicate's fixed-layout path (Un / prop-SWOR: snapshot rows, broadcast offsets,
row means, flushes on a worker thread) and the single drop-in call's fixed path
(_blocks.run_un_repeated), on the CPU: the device count is replaced by a NumPy restatement of
the per-block count (the GPU tests run the real kernels, tests/test_gpu_parity.py), so what is
checked here is the host logic — the layouts, the offsets, the row order across flushes and
threads, layout changes, the general-path fallbacks — against the general path and the
oracle's reference loop, with the same RNG consumption."""
import warnings

import numpy as np
import pytest
import torch

from oracle import oracle as O


@pytest.fixture
def host_counts(monkeypatch):
    from tuplewise import _engine as E
    from tuplewise import _lib as L
    from tuplewise import _multi as M

    def count(sh, mode="gt", algo="auto"):
        x, z = np.asarray(sh.x), np.asarray(sh.z)
        out = []
        for s in range(sh.n_shards):
            a = x[sh.x_off[s]:sh.x_off[s + 1]]
            b = z[sh.z_off[s]:sh.z_off[s + 1]]
            c = int((a[:, None] > b[None, :]).sum())
            if mode == "half":
                c = 2 * c + int((a[:, None] == b[None, :]).sum())
            out.append(c)
        return np.array(out, dtype=np.uint64)

    monkeypatch.setattr(E, "count_complete", count)
    monkeypatch.setattr(L, "to_device_many", lambda arrs, pinned=False: [
        torch.from_numpy(np.ascontiguousarray(a)) for a in arrs])
    monkeypatch.setattr(L, "to_device",
                        lambda a, dtype=None: torch.from_numpy(np.ascontiguousarray(a)))
    monkeypatch.setattr(M, "slots_for", lambda *a, **k: False)


@pytest.mark.parametrize("sizes", [[(500, 50)], [(300, 40), (301, 40), (300, 41)], [(95, 3)],
                                   [(300, 40), (95, 3), (300, 40)]])
@pytest.mark.parametrize("tie", ["strict", "half"])
@pytest.mark.parametrize("flush_elems", [1, 3000, 1 << 24])
def test_replicate_fixed_equals_general_and_reference(host_counts, sizes, tie, flush_elems):
    import tuplewise.estimation as est
    it = {"i": 0}

    def gx():
        return 2 * np.random.binomial(1, 0.9, sizes[it["i"] % len(sizes)][0])

    def gz():
        m = sizes[it["i"] % len(sizes)][1]
        it["i"] += 1
        return 2 * np.random.binomial(1, 0.1, m) - 1
    spec = (est._UN_HALF if tie == "half" else est._UN_STRICT)._tw_block
    for which, args, reps, N, st in (("Un", (), 1, None, None),
                                     ("UnN", (10, "prop-SWOR"), 1, 10, "prop-SWOR"),
                                     ("UnNT", (10, 3, "prop-SWOR"), 3, 10, "prop-SWOR")):
        fn = getattr(est, which)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            np.random.seed(4)
            it["i"] = 0
            got = est.replicate(fn, gx, gz, 30, *args, tie_mode=tie, flush_elems=flush_elems)
            probe_got = np.random.randint(2 ** 30)
            np.random.seed(4)
            it["i"] = 0
            want = est._replicate_general(fn, gx, gz, 30, spec, reps, N, st, flush_elems)
            probe_want = np.random.randint(2 ** 30)
            assert len(got) == 30 and probe_got == probe_want, which
            assert np.array_equal(np.array(got), np.array(want), equal_nan=True), which
            if tie == "strict":
                fo = {"Un": O.est_Un, "UnN": O.est_UnN, "UnNT": O.est_UnNT}[which]
                np.random.seed(4)
                it["i"] = 0
                ref = [fo(gx(), gz(), *args) for _ in range(30)]
                assert np.array_equal(np.array(got), np.array(ref), equal_nan=True), which


@pytest.mark.parametrize("seed", range(6))
def test_single_drop_in_call_fixed_path(host_counts, seed):
    """est.UnN / est.UnNT on host arrays (run_un / run_un_repeated's fixed layout) equal the
    oracle's reference loop: values, the arrays shuffled in place, the RNG state after."""
    import tuplewise.estimation as est
    rng = np.random.RandomState(seed)
    n, m = rng.randint(20, 400), rng.randint(5, 300)
    X = np.round(rng.normal(0.4, 1, n), 1)
    Z = np.round(rng.normal(0, 1, m), 1)
    for N in (3, 10):
        for T in (1, 4):
            Xa, Za, Xb, Zb = X.copy(), Z.copy(), X.copy(), Z.copy()
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                np.random.seed(seed)
                got = (est.UnNT(Xa, Za, N, T, "prop-SWOR"), est.UnN(Xa, Za, N, "prop-SWOR"))
                probe_got = np.random.randint(2 ** 30)
                np.random.seed(seed)
                want = (O.est_UnNT(Xb, Zb, N, T, "prop-SWOR"), O.est_UnN(Xb, Zb, N, "prop-SWOR"))
                probe_want = np.random.randint(2 ** 30)
            assert np.array_equal(got, want, equal_nan=True) and probe_got == probe_want
            assert np.array_equal(Xa, Xb) and np.array_equal(Za, Zb)
