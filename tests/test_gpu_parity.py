"""HIP path vs the reference's golden vectors and vs the pinned oracle (MI355X).

Bar: bit-exact for every count-derived value (U-statistics are count / #pairs); float-valued
kernels (prod, gini, hinge) within rtol 1e-12 of NumPy (different summation order); the
hinge gradient within 1e-12 relative (only BLAS's dot-product order can differ).
"""
import warnings

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = ["gauss", "bern_int64", "ties_int", "edge_float", "n1", "m1", "ragged", "int64_wrap",
         "float32", "col_scores"]
FLOAT_RTOL = 1e-12


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f")


@pytest.mark.parametrize("case", CASES)
def test_un_golden(gpu, golden, case):
    import tuplewise.estimation as est
    import tuplewise.compute_stats as cs
    X, Z = golden[f"un/{case}/X"], golden[f"un/{case}/Z"]
    assert same(est.Un(X, Z), golden[f"un/{case}/est_Un"])
    assert same(cs.Un(X, Z, kernel="AUC"), golden[f"un/{case}/cs_AUC"])
    if f"un/{case}/cs_prod" in golden:
        # float32 inputs: NumPy accumulates in float32 (~1e-7 relative per add), we in float64
        rtol = FLOAT_RTOL if X.dtype == np.float64 else 1e-5
        for k in ("prod", "gini"):
            got = cs.Un(X, Z, kernel=k)
            assert np.asarray(got).dtype == golden[f"un/{case}/cs_{k}"].dtype
            np.testing.assert_allclose(got, golden[f"un/{case}/cs_{k}"], rtol=rtol, atol=1e-15)
        np.testing.assert_allclose(cs.conv_AUC(1)(X, Z), golden[f"un/{case}/conv_AUC"],
                                   rtol=rtol)


def _calls():
    import tuplewise.estimation as est
    import tuplewise.compute_stats as cs
    return {
        "est_UnN_propSWOR": lambda X, Z: est.UnN(X, Z, 10, "prop-SWOR"),
        "est_UnN_SWOR": lambda X, Z: est.UnN(X, Z, 10, "SWOR"),
        "est_UnN_propSWR": lambda X, Z: est.UnN(X, Z, 10, "prop-SWR"),
        "est_UnNT_propSWOR": lambda X, Z: est.UnNT(X, Z, 10, 4, "prop-SWOR"),
        "est_UnNT_bern": lambda X, Z: est.UnNT(X, Z, 10, 4, "prop-SWOR"),
        "est_UnN_SWOR_degenerate": lambda X, Z: est.UnN(X, Z, 40, "SWOR"),
        "est_UnN_prop_degenerate": lambda X, Z: est.UnN(X, Z, 40, "prop-SWOR"),
        "cs_UnN_AUC": lambda X, Z: cs.UnN(X, Z, 10, "prop-SWOR", kernel="AUC"),
        "cs_UnN_AUC_SWOR": lambda X, Z: cs.UnN(X, Z, 10, "SWOR", kernel="AUC"),
        "cs_UnN_prod": lambda X, Z: cs.UnN(X, Z, 10, "prop-SWOR"),
        "cs_UnN_gini_SWR": lambda X, Z: cs.UnN(X, Z, 10, "prop-SWR", kernel="gini"),
        "cs_UnNB_AUC": lambda X, Z: cs.UnNB(X, Z, 10, 500, "prop-SWOR", kernel="AUC"),
        "cs_UnNB_AUC_SWR": lambda X, Z: cs.UnNB(X, Z, 10, 300, "prop-SWR", kernel="AUC"),
        "cs_UnNBT_AUC": lambda X, Z: cs.UnNBT(X, Z, 10, 200, 3, "SWOR", kernel="AUC"),
        "cs_UnNT_AUC": lambda X, Z: cs.UnNT(X, Z, 10, 3, "prop-SWOR", kernel="AUC"),
        "cs_UnNB_prod": lambda X, Z: cs.UnNB(X, Z, 10, 400, "prop-SWOR"),
    }


FLOAT_SHARDED = {"cs_UnN_prod", "cs_UnN_gini_SWR", "cs_UnNB_prod"}


@pytest.mark.parametrize("name", [
    "est_UnN_propSWOR", "est_UnN_SWOR", "est_UnN_propSWR", "est_UnNT_propSWOR", "est_UnNT_bern",
    "est_UnN_SWOR_degenerate", "est_UnN_prop_degenerate", "cs_UnN_AUC", "cs_UnN_AUC_SWOR",
    "cs_UnN_prod", "cs_UnN_gini_SWR", "cs_UnNB_AUC", "cs_UnNB_AUC_SWR", "cs_UnNBT_AUC",
    "cs_UnNT_AUC", "cs_UnNB_prod"])
def test_sharded_golden(gpu, golden, name):
    fn = _calls()[name]
    X, Z = golden[f"sh/{name}/X"].copy(), golden[f"sh/{name}/Z"].copy()
    np.random.seed(int(golden[f"sh/{name}/seed"]))
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        val = fn(X, Z)
    if name in FLOAT_SHARDED:
        np.testing.assert_allclose(val, golden[f"sh/{name}/value"], rtol=FLOAT_RTOL)
    else:
        assert same(val, golden[f"sh/{name}/value"]), (val, golden[f"sh/{name}/value"])
    # in-place shuffle side effect and RNG consumption identical to the reference
    assert same(X, golden[f"sh/{name}/X_after"]) and same(Z, golden[f"sh/{name}/Z_after"])
    assert np.random.randint(0, 2 ** 31 - 1) == golden[f"sh/{name}/probe"]


def test_indexed_golden(gpu, golden):
    import tuplewise.compute_stats as cs
    X, Z, ix, iz = golden["idx/X"], golden["idx/Z"], golden["idx/ix"], golden["idx/iz"]
    assert same(cs.UB_indices(X, Z, ix, iz, "AUC"), golden["idx/UB_indices_AUC"])
    for k in ("prod", "gini"):
        np.testing.assert_allclose(cs.UB_indices(X, Z, ix, iz, k), golden[f"idx/UB_indices_{k}"],
                                   rtol=FLOAT_RTOL)
    pairs = list(zip(list(ix), list(iz)))
    assert same(cs.UB_pairs(X, Z, pairs, "AUC"), golden["idx/UB_pairs_AUC"])
    np.testing.assert_allclose(cs.conv_AUC_deter_pairs(1)(X, Z, pairs), golden["idx/conv_deter"],
                               rtol=FLOAT_RTOL)
    np.random.seed(77)
    assert same(cs.UB(X, Z, 1000, kernel="AUC"), golden["idx/UB_AUC_seed77"])


def test_grad_golden(gpu, golden):
    import tuplewise.compute_stats as cs
    X, Z, w = golden["grad/X"], golden["grad/Z"], golden["grad/w"]
    np.random.seed(5)
    g = cs.grad_inc_block(w, 100, 1)(X, Z)
    np.testing.assert_allclose(g, golden["grad/single_seed5"], rtol=1e-12, atol=1e-15)
    np.random.seed(6)
    Xs, Zs = cs.SWR_divide(X, Z, 10)
    gs = cs.UN_split(Xs, Zs, cs.grad_inc_block(w, 50, 1))
    np.testing.assert_allclose(gs, golden["grad/split_seed6"], rtol=1e-12, atol=1e-15)
    assert gs.shape == golden["grad/split_seed6"].shape


# ------------------------------------------------------------------ kernels vs oracle
@pytest.mark.parametrize("algo", ["pairs", "sorted"])
@pytest.mark.parametrize("dtype", ["f64", "i64"])
@pytest.mark.parametrize("mode", ["gt", "half"])
def test_count_kernel_ragged_shards(gpu, dtype, mode, algo):
    from tuplewise import _engine as E, _lib as L
    rng = np.random.RandomState(7)
    nx = [0, 1, 5, 257, 3000, 1, 4096 + 3, 700]
    nz = [3, 0, 9, 1000, 2049, 1, 513, 700]
    if dtype == "f64":
        xs = [rng.normal(size=k).round(1) for k in nx]  # rounding forces ties
        zs = [rng.normal(size=k).round(1) for k in nz]
        code = L.TW_F64
    else:
        xs = [rng.randint(-20, 20, k) for k in nx]
        zs = [rng.randint(-20, 20, k) for k in nz]
        code = L.TW_I64
    if dtype == "f64":  # NumPy comparison edge values in some shards
        xs[3][:6] = [np.nan, -0.0, 0.0, np.inf, -np.inf, 5e-324]
        zs[3][:6] = [0.0, -0.0, np.nan, np.inf, -np.inf, -5e-324]
    sh = E.Shards.from_blocks(xs, zs, code)
    got = E.count_complete(sh, mode, algo=algo)
    for s, (x, z) in enumerate(zip(xs, zs)):
        if mode == "gt":
            want = O.un_count(x, z)
        else:  # 2#{x>z} + #{x==z} straight from the broadcast compare (NaN-safe)
            want = 2 * O.un_count(x, z) + int((x.reshape(-1, 1) == z.reshape(1, -1)).sum())
        assert int(got[s]) == want, (s, int(got[s]), want)


@pytest.mark.parametrize("algo", ["pairs", "sorted"])
def test_count_c2_single_shard_1e5(gpu, algo):
    """BASELINE config C2: n = m = 1e5 in one shard (1e10 pairs), exact vs O(n log n) count."""
    from tuplewise import _engine as E, _lib as L
    rng = np.random.RandomState(2)
    X, Z = rng.normal(0.5, 1, 100_000), rng.normal(0, 1, 100_000)
    sh = E.Shards.from_blocks([X], [Z], L.TW_F64)
    got = int(E.count_complete(sh, "gt", algo=algo)[0])
    assert got == O.count_gt_sorted(X, Z)


@pytest.mark.parametrize("algo", ["pairs", "sorted"])
def test_count_c2_half_ties_1e5(gpu, algo):
    """C2 size with heavy ties (1000 distinct values): half-unit counts 2#{x>z} + #{x==z}
    (the mixed VALU/SALU kernel counts both masks) vs an O(n log n) restatement."""
    from tuplewise import _engine as E, _lib as L
    rng = np.random.RandomState(3)
    X = rng.randint(0, 1000, 100_000).astype(np.float64)
    Z = rng.randint(0, 1000, 100_000).astype(np.float64)
    X[:7] = -0.0
    Z[:5] = 0.0
    sh = E.Shards.from_blocks([X], [Z], L.TW_F64)
    got = int(E.count_complete(sh, "half", algo=algo)[0])
    zs = np.sort(Z)
    gt = int(np.searchsorted(zs, X, side="left").sum())
    ge = int(np.searchsorted(zs, X, side="right").sum())
    assert got == gt + ge


def test_device_sharded_sample_matches_oracle(gpu):
    """Device repartition (Feistel) + one-launch count == oracle restatement, per shard."""
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(4)
    n, m, N = 20_000, 15_000, 16
    X, Z = rng.normal(0.3, 1, n), rng.normal(0, 1, m)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
    key = 99
    v = S.UnN(key)
    Xp = O.permute_scatter(X, 2 * key)
    Zp = O.permute_scatter(Z, 2 * key + 1)
    assert np.array_equal(S.X.cpu().numpy(), Xp) and np.array_equal(S.Z.cpu().numpy(), Zp)
    k, tau = int(n / N), int((n + m) / N)
    vals = [O.un_count(Xp[s * k:(s + 1) * k], Zp[s * (tau - k):(s + 1) * (tau - k)])
            / (k * (tau - k)) for s in range(N)]
    assert v == np.mean(vals)


def test_device_rng_incomplete_matches_oracle(gpu):
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(8)
    n, m, N, B = 4000, 3000, 4, 777
    X, Z = rng.normal(0.2, 1, n), rng.normal(0, 1, m)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
    seed = 0x1234_5678_9ABC
    v = S.UnNB(B, seed)
    k, tau = int(n / N), int((n + m) / N)
    vals = []
    for s in range(N):
        xs, zs = X[s * k:(s + 1) * k], Z[s * (tau - k):(s + 1) * (tau - k)]
        i, j = O.rng_pairs(len(xs), len(zs), B, seed, s)
        vals.append(np.float64(int((xs[i] > zs[j]).sum())) / np.float64(B))
    assert v == np.mean(vals)


def test_north_star_config_exact(gpu):
    """BASELINE config C3 shape: n = 1e6 per class, N = 64 shards (1.5625e10 pairs), one
    repartition on the device; every shard's count equals the oracle's exact count."""
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(5)
    n, N = 1_000_000, 64
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo="pairs")
    S.repartition(7)
    counts = S.local_counts().cpu().numpy()
    S.algo = "sorted"
    assert np.array_equal(S.local_counts().cpu().numpy(), counts)
    Xp, Zp = S.X.cpu().numpy(), S.Z.cpu().numpy()
    assert np.array_equal(np.sort(Xp), np.sort(X))  # a permutation
    k = n // N
    for s in range(N):
        assert counts[s] == O.count_gt_sorted(Xp[s * k:(s + 1) * k], Zp[s * k:(s + 1) * k])


def test_errors_match_reference(gpu):
    import tuplewise.compute_stats as cs
    X, Z = np.random.normal(size=10), np.random.normal(size=5)
    with pytest.raises(AssertionError):
        cs.Un(X, Z, kernel="bogus")
    with pytest.raises(AssertionError):
        cs.UN(X.copy(), Z.copy(), 20, cs.Un, sampling_type="prop-SWOR")  # k == 0 block
    with pytest.raises(TypeError):
        cs.Un(np.array([True, False]), np.array([False]), kernel="AUC")


def test_multicolumn_scores_match_oracle(gpu):
    """2-D score arrays: Un flattens (reshape(-1)), UN slices rows, UB subtracts rows."""
    import tuplewise.estimation as est
    import tuplewise.compute_stats as cs
    rng = np.random.RandomState(12)
    X, Z = rng.normal(size=(300, 3)).round(1), rng.normal(size=(200, 3)).round(1)
    assert est.Un(X, Z) == O.est_Un(X, Z)
    for st in ("prop-SWOR", "SWOR", "prop-SWR"):
        a, b = X.copy(), Z.copy()
        np.random.seed(4)
        got = est.UnN(a, b, 7, st)
        c, d = X.copy(), Z.copy()
        np.random.seed(4)
        want = O.est_UnN(c, d, 7, st)
        assert got == want and np.array_equal(a, c)
    np.random.seed(5)
    got = cs.UnNB(X.copy(), Z.copy(), 5, 64, "prop-SWOR", kernel="AUC")
    np.random.seed(5)
    want = O.cs_UnNB(X.copy(), Z.copy(), 5, 64, "prop-SWOR", "AUC")
    assert got == want
    ix, iz = rng.randint(0, 300, 50), rng.randint(0, 200, 50)
    assert cs.UB_indices(X, Z, ix, iz, "AUC") == O.UB_indices(X, Z, ix, iz, "AUC")


def test_empty_inputs_like_numpy(gpu):
    import tuplewise.estimation as est
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        assert np.isnan(est.Un(np.zeros(0), np.ones(3)))
        assert np.isnan(O.est_Un(np.zeros(0), np.ones(3)))


@pytest.mark.parametrize("which", ["Un", "UnN", "UnNT"])
def test_replicate_equals_reference_loop(gpu, which):
    """estimation.replicate == the Monte-Carlo list comprehension of main.py:106-112."""
    import tuplewise.estimation as est
    n, m, e = 500, 50, 0.1
    gen_X = lambda: 2 * np.random.binomial(1, 1 - e, n)
    gen_Z = lambda: 2 * np.random.binomial(1, e, m) - 1
    args = {"Un": (), "UnN": (10, "prop-SWOR"), "UnNT": (10, 4, "prop-SWOR")}[which]
    fo = {"Un": O.est_Un, "UnN": O.est_UnN, "UnNT": O.est_UnNT}[which]
    np.random.seed(21)
    want = [fo(gen_X(), gen_Z(), *args) for _ in range(60)]
    probe_want = np.random.randint(2 ** 30)
    np.random.seed(21)
    got = est.replicate(getattr(est, which), gen_X, gen_Z, 60, *args, flush_elems=20_000)
    probe_got = np.random.randint(2 ** 30)
    assert got == want and probe_got == probe_want


@pytest.mark.parametrize("case", ["sizes_change", "empty_blocks", "half_ties", "floats"])
def test_replicate_fixed_layout_equals_general(gpu, case):
    """replicate's fixed-layout path (Un / prop-SWOR: snapshot rows, broadcast offsets, row
    means) == the general per-block path and, where the oracle covers it, the reference loop:
    tries whose sizes change (the layout is rebuilt after a flush), plans with empty blocks
    (the general path's nan), tie_mode="half", float scores with ties."""
    import tuplewise.estimation as est
    sizes = {"sizes_change": [(300, 40), (301, 40), (300, 41)], "empty_blocks": [(95, 3)],
             "half_ties": [(400, 60)], "floats": [(350, 45)]}[case]
    it = {"i": 0}

    def gen_X():
        n = sizes[it["i"] % len(sizes)][0]
        if case == "floats":
            return np.round(np.random.normal(0.2, 1, n), 1)
        return 2 * np.random.binomial(1, 0.9, n)

    def gen_Z():
        m = sizes[it["i"] % len(sizes)][1]
        it["i"] += 1
        if case == "floats":
            return np.round(np.random.normal(0, 1, m), 1)
        return 2 * np.random.binomial(1, 0.1, m) - 1
    tie = "half" if case == "half_ties" else "strict"
    spec = (est._UN_HALF if tie == "half" else est._UN_STRICT)._tw_block
    for which, args, reps, N, st in (("Un", (), 1, None, None),
                                     ("UnN", (10, "prop-SWOR"), 1, 10, "prop-SWOR"),
                                     ("UnNT", (10, 3, "prop-SWOR"), 3, 10, "prop-SWOR")):
        fn = getattr(est, which)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            np.random.seed(4)
            it["i"] = 0
            got = est.replicate(fn, gen_X, gen_Z, 25, *args, tie_mode=tie, flush_elems=3000)
            probe_got = np.random.randint(2 ** 30)
            np.random.seed(4)
            it["i"] = 0
            want = est._replicate_general(fn, gen_X, gen_Z, 25, spec, reps, N, st, 3000)
            probe_want = np.random.randint(2 ** 30)
            assert probe_got == probe_want, which
            assert np.array_equal(np.array(got), np.array(want), equal_nan=True), which
            if tie == "strict":
                fo = {"Un": O.est_Un, "UnN": O.est_UnN, "UnNT": O.est_UnNT}[which]
                np.random.seed(4)
                it["i"] = 0
                ref = [fo(gen_X(), gen_Z(), *args) for _ in range(25)]
                assert np.array_equal(np.array(got), np.array(ref), equal_nan=True), which


def test_pipelined_unn_many_equals_sequential(gpu):
    """ShardedSample.UnN_many (repartition i+1 on a side stream during the counts of step i,
    counts combined at the end) == one UnN call per key, value for value, and leaves the
    same permuted arrays."""
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(12)
    n, m, N = 300_000, 250_000, 16
    X, Z = rng.normal(0.3, 1, n), rng.normal(0, 1, m)
    keys = [3, 4, 5, 6, 7]
    for algo in ("pairs", "sorted"):
        S1 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo=algo)
        S2 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo=algo)
        seq = [S1.UnN(k) for k in keys]
        pipe = S2.UnN_many(keys)
        assert seq == pipe
        assert torch.equal(S1.X, S2.X) and torch.equal(S1.Z, S2.Z)
        assert S2.UnNT(3, key0=40) == np.mean([S1.UnN(k) for k in (40, 41, 42)])
    # incomplete statistic with fresh device draws per repartition (cs.UnNBT's loop)
    # (one GPU: each ranked draw-and-count launch also repartitions for the next key on spare
    # blocks, tw_count_pairs_rng_step) — ranked via sort (18750-value shards) and via buckets
    # (<= 16384), strict and half ties, float64 and int64, ragged shards, one key
    ri = np.random.RandomState(13)
    cases = [(X, Z, N, "strict", keys), (X[:200_000], Z[:150_001], 16, "half", keys),
             (ri.randint(0, 50, 160_003), ri.randint(0, 50, 120_000), 12, "half", keys),
             (X[:50_000], Z[:40_000], 4, "strict", [9])]
    for xa, za, nn, tie, ks in cases:
        S1 = ShardedSample(torch.from_numpy(xa).cuda(), torch.from_numpy(za).cuda(), nn,
                           tie_mode=tie)
        S2 = ShardedSample(torch.from_numpy(xa).cuda(), torch.from_numpy(za).cuda(), nn,
                           tie_mode=tie)
        seq = [S1.UnNB(5000, 77 + i, key=k) for i, k in enumerate(ks)]
        assert S2.UnNB_many(5000, 77, ks) == seq, (len(xa), tie)
        assert torch.equal(S1.X, S2.X) and torch.equal(S1.Z, S2.Z)


def test_exchange_kernels_simulated_ranks(gpu):
    """Multi-rank repartition kernels for G=5 ranks simulated in one process (the all-to-all
    is a host-side regrouping): send counts, receive counts from the inverse permutation,
    block-reserved bucket scatter with a position base, scatter into place == the global
    permutation of the oracle."""
    import torch
    from tuplewise.device import HipOps
    ops = HipOps()
    G, n_loc, key = 5, 30_011, 0xDEADBEEF
    n_tot = G * n_loc
    rng = np.random.RandomState(1)
    vals = rng.normal(size=n_tot)
    want = O.permute_scatter(vals, key)
    inbox = [[] for _ in range(G)]
    for r in range(G):
        perm = ops.perm_index(n_loc, r * n_loc, n_tot, key)
        p = O.feistel_perm(np.arange(r * n_loc, (r + 1) * n_loc), n_tot, key)
        assert np.array_equal(perm.cpu().numpy(), p)
        sc = ops.rank_histogram(perm, n_loc, G)
        assert np.array_equal(sc.cpu().numpy(), np.bincount(p // n_loc, minlength=G))
        rc = ops.source_histogram(n_loc, r * n_loc, n_tot, key, n_loc, G).cpu().numpy()
        src = O.feistel_perm_inv(np.arange(r * n_loc, (r + 1) * n_loc), n_tot, key)
        assert np.array_equal(rc, np.bincount(src // n_loc, minlength=G))
        start = torch.cumsum(sc, 0) - sc
        send = torch.full((n_loc, 2), -1, dtype=torch.int64, device="cuda")
        ops.bucket_scatter(perm, torch.from_numpy(vals[r * n_loc:(r + 1) * n_loc]).cuda(),
                           n_loc, G, start, send, 7)
        s = send.cpu().numpy()
        off = np.concatenate([[0], np.cumsum(sc.cpu().numpy())])
        for q in range(G):
            inbox[q].append(s[off[q]:off[q + 1]])
    for q in range(G):
        rec = np.concatenate(inbox[q])
        assert rec.shape[0] == n_loc
        assert np.array_equal(np.sort(rec[:, 1]), np.arange(n_loc) + 7)  # every slot once
        rec[:, 1] -= 7
        out = torch.empty(n_loc, dtype=torch.float64, device="cuda")
        ops.scatter_records(torch.from_numpy(rec).cuda(), out)
        assert np.array_equal(out.cpu().numpy(), want[q * n_loc:(q + 1) * n_loc])


@pytest.mark.parametrize("loss", ["hinge", "logistic"])
@pytest.mark.parametrize("d,B", [(10, 300), (33, 100), (100, 1500), (512, 100), (512, 2100),
                                 (512, 16), (512, 17), (512, 48), (700, 64)])
def test_hinge_grad_wide_rows(gpu, d, B, loss):
    """tw_hinge_grad for wide rows (the streaming kernel for 32 < d <= 512 — chunk counts
    odd/even/partial via B = 16, 17, 48, 100 —, the burst-pipelined and unpipelined ones):
    per-shard gradients vs the restated reference body (compute_stats.py:153-162), and all wide
    kernels bit-identical to each other."""
    import torch
    from tuplewise import _lib as L, _learn
    rng = np.random.RandomState(d + B)
    nX, nZ, N, kx, kz = 3000, 2000, 6, 400, 300
    X, Z = rng.normal(size=(nX, d)), rng.normal(0.2, 1, size=(nZ, d))
    w = rng.normal(size=d) / np.sqrt(d)
    rows_x = rng.randint(0, nX, size=(N, kx))
    rows_z = rng.randint(0, nZ, size=(N, kz))
    code = L.TW_LOSS_HINGE if loss == "hinge" else L.TW_LOSS_LOGISTIC
    ix = rng.randint(0, kx, size=(N, B))
    iz = rng.randint(0, kz, size=(N, B))
    dev = [L.to_device(a) for a in (X, Z, rows_x, rows_z, ix, iz, w)]
    outs = []
    for legacy in (0, 1, 2):
        L.call("tw_hinge_set_variant", legacy)
        try:
            g = _learn.hinge_grads_device(dev[0], dev[1], d, dev[2], kx, dev[3], kz, dev[4],
                                          dev[5], N, B, dev[6], 1.0, code)
        finally:
            L.call("tw_hinge_set_variant", 0)
        outs.append(g.cpu().numpy())
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    for s in range(N):
        diff = Z[rows_z[s][iz[s]]] - X[rows_x[s][ix[s]]]
        want = O.pair_grad(diff, w.reshape(-1, 1), 1.0, B, loss).ravel()
        # hinge: same row-order sums, only BLAS's dot order differs (sign flips at |S| ~ ulp);
        # logistic: sigma(S) also carries the device exp's last-ulp differences
        np.testing.assert_allclose(outs[0][s], want, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("dtype,mode", [("f64", "gt"), ("f64", "half"), ("i64", "subgt")])
def test_count_pairs_step_fused_repartition(gpu, dtype, mode):
    """tw_count_pairs_step: counts == tw_count_pairs on ragged shards, and the same launch
    writes the next repartition (== oracle permutation) and zeroes the next counters."""
    import torch
    from tuplewise import _engine as E, _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(21)
    nx = [0, 1, 5, 257, 3000, 1, 4096 + 3, 700]
    nz = [3, 0, 9, 1000, 2049, 1, 513, 700]
    if dtype == "f64":
        xs = [rng.normal(size=k).round(1) for k in nx]
        zs = [rng.normal(size=k).round(1) for k in nz]
        code = L.TW_F64
    else:
        xs = [rng.randint(-2 ** 62, 2 ** 62, k) * 2 for k in nx]  # wraps in x - z
        zs = [rng.randint(-2 ** 62, 2 ** 62, k) * 2 for k in nz]
        code = L.TW_I64
    sh = E.Shards.from_blocks(xs, zs, code)
    want = E.count_complete(sh, mode, algo="pairs")
    xo, zo = sh.offsets_dev()
    pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF, "subgt": L.TW_PRED_SUBGT}[mode]
    out = torch.zeros(len(nx), dtype=torch.int64, device="cuda")
    out_next = torch.full((5,), 77, dtype=torch.int64, device="cuda")
    xn, zn = torch.empty_like(sh.x), torch.empty_like(sh.z)
    HipOps().count_step(sh.x, xo, sh.z, zo, len(nx), max(nx), max(nz), code, pred, out, xn, 11,
                        zn, 12, out_next)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    assert not out_next.cpu().numpy().any()
    assert np.array_equal(xn.cpu().numpy(), O.permute_scatter(sh.x.cpu().numpy(), 11))
    assert np.array_equal(zn.cpu().numpy(), O.permute_scatter(sh.z.cpu().numpy(), 12))


@pytest.mark.parametrize("dtype,mode,big", [("f64", "gt", False), ("f64", "half", False),
                                            ("i64", "gt", False), ("f64", "gt", True)])
def test_count_pairs_rng_step_fused_repartition(gpu, dtype, mode, big):
    """tw_count_pairs_rng_step: counts == tw_count_pairs_rng_ws (the same draws) on ragged
    shards incl. empty ones, and the same call writes the next repartition (== the oracle
    permutation) and zeroes the next counters — on the float32-image path, where the
    permutation's gathers ride in the count threads (B small and large: the gathers issued in
    the Philox loop or left to the tail), and past it (big: a shard too large for LDS images,
    count + tw_permute_pair + memset)."""
    import torch
    from tuplewise import _engine as E, _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(22)
    nx = [0, 1, 5, 257, 3000, 1, 4096 + 3, 700] + ([41_000] if big else [])
    nz = [3, 0, 9, 1000, 2049, 1, 513, 700] + ([1_000] if big else [])
    if dtype == "f64":
        xs = [rng.normal(size=k).round(1) for k in nx]
        zs = [rng.normal(size=k).round(1) for k in nz]
        code = L.TW_F64
    else:
        xs = [rng.randint(-50, 50, k) for k in nx]
        zs = [rng.randint(-50, 50, k) for k in nz]
        code = L.TW_I64
    sh = E.Shards.from_blocks(xs, zs, code)
    xo, zo = sh.offsets_dev()
    pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF}[mode]
    ops = HipOps()
    for B in (1, 7, 5000, 300_001):
        want = ops.count_rng(sh.x, xo, sh.z, zo, len(nx), B, 99 + B, 3, code, pred,
                             max_nx=max(nx), max_nz=max(nz))
        out = torch.zeros(len(nx), dtype=torch.int64, device="cuda")
        out_next = torch.full((5,), 77, dtype=torch.int64, device="cuda")
        xn, zn = torch.empty_like(sh.x), torch.empty_like(sh.z)
        ops.count_rng_step(sh.x, xo, sh.z, zo, len(nx), B, 99 + B, 3, code, pred, max(nx),
                           max(nz), out, xn, 11 + B, zn, 12 + B, out_next)
        assert torch.equal(out, want), B
        assert not out_next.cpu().numpy().any()
        assert np.array_equal(xn.cpu().numpy(), O.permute_scatter(sh.x.cpu().numpy(), 11 + B))
        assert np.array_equal(zn.cpu().numpy(), O.permute_scatter(sh.z.cpu().numpy(), 12 + B))
    # count only (no next arrays): the counts alone, out_next zeroed by a memset
    out = torch.zeros(len(nx), dtype=torch.int64, device="cuda")
    out_next = torch.full((3,), 5, dtype=torch.int64, device="cuda")
    L.call("tw_count_pairs_rng_step", L.ptr(sh.x), L.ptr(xo), L.ptr(sh.z), L.ptr(zo), len(nx),
           max(nx), max(nz), 4000, 5, 0, code, pred, None, 0, L.ptr(out), 0, None, 0, 0, None,
           0, L.ptr(out_next), 3, L.stream_handle())
    want = ops.count_rng(sh.x, xo, sh.z, zo, len(nx), 4000, 5, 0, code, pred,
                         max_nx=max(nx), max_nz=max(nz))
    assert torch.equal(out, want) and not out_next.cpu().numpy().any()


@pytest.mark.parametrize("dtype,mode,big", [("f64", "gt", False), ("f64", "half", False),
                                            ("i64", "gt", False), ("f64", "gt", True)])
def test_count_pairs_sorted_step_fused_repartition(gpu, dtype, mode, big):
    """tw_count_pairs_sorted_step: counts == the exact all-pairs counts on ragged shards incl.
    empty ones (NaN-free ties: rounded scores / small integers), and the same launch writes the
    next repartition (== the oracle permutation) and zeroes the next counters — on the bucket
    path (gathers in the count threads) and past it (big: a shard with nz > 16384, sort +
    search, then tw_permute_pair and a memset)."""
    import torch
    from tuplewise import _engine as E, _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(23)
    nx = [0, 1, 5, 257, 3000, 1, 4096 + 3, 700, 9000] + ([2_000] if big else [])
    nz = [3, 0, 9, 1000, 2049, 1, 513, 700, 16384] + ([20_000] if big else [])
    if dtype == "f64":
        xs = [rng.normal(size=k).round(1) for k in nx]
        zs = [rng.normal(size=k).round(1) for k in nz]
        code = L.TW_F64
    else:
        xs = [rng.randint(-50, 50, k) for k in nx]
        zs = [rng.randint(-50, 50, k) for k in nz]
        code = L.TW_I64
    sh = E.Shards.from_blocks(xs, zs, code)
    want = E.count_complete(sh, mode, algo="pairs")
    xo, zo = sh.offsets_dev()
    pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF}[mode]
    out = torch.zeros(len(nx), dtype=torch.int64, device="cuda")
    out_next = torch.full((5,), 77, dtype=torch.int64, device="cuda")
    xn, zn = torch.empty_like(sh.x), torch.empty_like(sh.z)
    HipOps().count_sorted_step(sh.x, xo, sh.z, zo, len(nx), max(nx), max(nz), code, pred, out,
                               xn, 31, zn, 32, out_next)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    assert not out_next.cpu().numpy().any()
    assert np.array_equal(xn.cpu().numpy(), O.permute_scatter(sh.x.cpu().numpy(), 31))
    assert np.array_equal(zn.cpu().numpy(), O.permute_scatter(sh.z.cpu().numpy(), 32))


@pytest.mark.parametrize("n,m,N,tie,dt", [(300_000, 250_000, 16, "strict", "f64"),
                                          (100_003, 90_001, 7, "half", "f64"),
                                          (60_000, 70_000, 5, "strict", "i64"),
                                          (5_000, 20, 3, "half", "i64"),
                                          # one block per shard with > 8192 records to append:
                                          # the unstaged emission
                                          (600 * 7_000, 600 * 7_000 + 11, 600, "strict", "f64"),
                                          # 2N + 2 > 2048 buckets: the unstaged emission
                                          (1_100 * 200 + 5, 1_100 * 150, 1_100, "half", "f64")])
def test_sorted_steps_records_path(gpu, n, m, N, tie, dt):
    """UnN_many with the sorted count through tw_count_pairs_sorted_steps (the partition kept
    as destination-bucketed records between steps, csrc/records.h): per-step estimates equal
    the step-at-a-time path (tw_permute_pair + the sorted count), and the arrays after the last
    step equal the oracle's chain of permutations — with tails that belong to no shard
    (n, m not multiples of the shard sizes), ties, int64, T = 1, 2, 5.  The default route
    (the step chains' exact bucket count of every bag, round 4) gives the same again."""
    import torch
    from tuplewise.device import HipOps, ShardedSample

    class OneStep(HipOps):  # without the records entry: one repartition + count per step
        @property
        def count_sorted_steps(self):
            raise AttributeError

        @property
        def count_chain_bucket(self):
            raise AttributeError

    class Records(HipOps):  # the records path, not the step chains' bucket count
        @property
        def count_chain_bucket(self):
            raise AttributeError

    rng = np.random.RandomState(n % 97)
    if dt == "f64":
        X, Z = rng.normal(0.3, 1, n).round(2), rng.normal(0, 1, m).round(2)
    else:
        X, Z = rng.randint(-40, 40, n), rng.randint(-40, 40, m)
    for keys in ([7], [7, 8], [3, 1, 4, 1, 5]) if n < 10 ** 6 else ([7, 8],):
        S1 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                           tie_mode=tie, algo="sorted", ops=OneStep())
        S2 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                           tie_mode=tie, algo="sorted", ops=Records())
        # the default: the step chains with the bags' exact bucket count (round 4)
        S3 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                           tie_mode=tie, algo="sorted")
        want = S1.UnN_many(keys)
        for S in (S2, S3):
            got = S.UnN_many(keys)
            assert got == want, (keys, got, want)
        Xp, Zp = X, Z
        for k in keys:
            Xp = O.permute_scatter(Xp, (2 * k) % 2 ** 64)
            Zp = O.permute_scatter(Zp, (2 * k + 1) % 2 ** 64)
        for S in (S2, S3):
            assert np.array_equal(S.X.cpu().numpy(), Xp) and np.array_equal(S.Z.cpu().numpy(), Zp)


def test_device_sigmoid_accuracy(gpu):
    """The device sigma (tw_common.h pair_weight: 1 / (1 + exp(-S)) with the device exp) within 4 ulp of
    NumPy's 1 / (1 + exp(-S)) over the whole range, incl. saturation, +-inf and NaN: one
    shard per S value, d = 1, x = 0, z = c, w = 1, margin 0, B = 1 -> gradient = sigma(c) c."""
    from tuplewise import _lib as L, _learn
    c = np.concatenate([np.linspace(-50, 50, 2001), [-745.5, -709.9, -40.0, -1e-300, 1e-300,
                        36.0, 40.0, 800.0, 1e10, -1e10], np.random.RandomState(3).normal(0, 5, 2000)])
    c = c[c != 0]
    N = len(c)
    X, Z = np.zeros((N, 1)), c.reshape(-1, 1)
    rows = L.to_device(np.arange(N, dtype=np.int64).reshape(N, 1))
    idx = L.to_device(np.zeros(N, dtype=np.int64))
    g = _learn.hinge_grads_device(L.to_device(X), L.to_device(Z), 1, rows, 1, rows, 1, idx, idx,
                                  N, 1, L.to_device(np.ones(1)), 0.0,
                                  L.TW_LOSS_LOGISTIC).cpu().numpy().ravel()
    with np.errstate(over="ignore"):
        want = (1.0 / (1.0 + np.exp(-c))) * c
    ulp = np.spacing(np.abs(want))
    assert np.all(np.abs(g - want) <= 4 * ulp), np.max(np.abs(g - want) / ulp)
    # inf / NaN scores
    Xs = np.array([[0.0], [0.0], [0.0]])
    Zs = np.array([[np.inf], [-np.inf], [np.nan]])
    r3 = L.to_device(np.arange(3, dtype=np.int64).reshape(3, 1))
    i3 = L.to_device(np.zeros(3, dtype=np.int64))
    g3 = _learn.hinge_grads_device(L.to_device(Xs), L.to_device(Zs), 1, r3, 1, r3, 1, i3, i3, 3,
                                   1, L.to_device(np.ones(1)), 0.0,
                                   L.TW_LOSS_LOGISTIC).cpu().numpy().ravel()
    with np.errstate(over="ignore", invalid="ignore"):
        w3 = (1.0 / (1.0 + np.exp(-Zs.ravel()))) * Zs.ravel()
    assert np.array_equal(g3, w3, equal_nan=True), (g3, w3)


def test_logistic_surrogates_and_block_gradient(gpu):
    """Row L3 extension (parity pinned against the oracle only): conv_AUC / conv_AUC_deter_pairs
    with loss="logistic" and grad_inc_block(..., loss="logistic") inside UN_split."""
    import tuplewise.compute_stats as cs
    rng = np.random.RandomState(17)
    sx, sz = rng.normal(0.3, 1, 700), rng.normal(0, 1, 300)
    for margin in (1.0, 0.0, -0.5):
        got = cs.conv_AUC(margin, loss="logistic")(sx, sz)
        want = O.conv_AUC(margin, loss="logistic")(sx, sz)
        np.testing.assert_allclose(got, want, rtol=1e-12)
    pairs = list(zip(rng.randint(0, 700, 5000), rng.randint(0, 300, 5000)))
    np.testing.assert_allclose(cs.conv_AUC_deter_pairs(1, loss="logistic")(sx, sz, pairs),
                               O.conv_AUC_deter_pairs(1, loss="logistic")(sx, sz, pairs),
                               rtol=1e-12)
    X, Z = rng.normal(size=(400, 12)), rng.normal(0.4, 1, size=(150, 12))
    w = rng.normal(size=(12, 1))
    np.random.seed(9)
    Xs, Zs = cs.SWR_divide(X, Z, 5)
    g = cs.UN_split(Xs, Zs, cs.grad_inc_block(w, 64, 1, loss="logistic"))
    np.random.seed(9)
    Xo, Zo = O.SWR_divide(X, Z, 5)
    want = O.UN_split(Xo, Zo, O.grad_inc_block(w, 64, 1, loss="logistic"))
    np.testing.assert_allclose(g, want, rtol=1e-12, atol=1e-15)
    with pytest.raises(ValueError):
        cs.grad_inc_block(w, 64, 1, loss="exp")


def test_fused_exchange_kernels_simulated_ranks(gpu):
    """tw_exchange_counts / tw_exchange_pack for G=3 ranks simulated in one process: counts vs
    the oracle's forward/inverse permutation histograms, every bucket [X records | Z records],
    and after the (host-side) all-to-all and the scatter both samples equal the oracle's
    global permutations."""
    import torch
    from tuplewise.device import HipOps
    ops = HipOps()
    G, n_loc, m_loc, kx, kz = 3, 20_011, 7_003, 101, 202
    rng = np.random.RandomState(4)
    X, Z = rng.normal(size=G * n_loc), rng.normal(size=G * m_loc)
    want_x, want_z = O.permute_scatter(X, kx), O.permute_scatter(Z, kz)
    inbox = [[] for _ in range(G)]
    for r in range(G):
        cnt, cur = ops.exchange_counts(n_loc, m_loc, r, G, kx, kz)
        c = cnt.cpu().numpy().reshape(4, G)
        for row, (n, key, inv) in enumerate([(n_loc, kx, False), (n_loc, kx, True),
                                             (m_loc, kz, False), (m_loc, kz, True)]):
            g = np.arange(r * n, (r + 1) * n)
            p = O.feistel_perm_inv(g, G * n, key) if inv else O.feistel_perm(g, G * n, key)
            assert np.array_equal(c[row], np.bincount(p // n, minlength=G))
        send = ops.exchange_pack(torch.from_numpy(X[r * n_loc:(r + 1) * n_loc]).cuda(),
                                 torch.from_numpy(Z[r * m_loc:(r + 1) * m_loc]).cuda(), r, G, kx,
                                 kz, cnt, cur).cpu().numpy()
        off = np.concatenate([[0], np.cumsum(c[0] + c[2])])
        for q in range(G):
            b = send[off[q]:off[q + 1]]
            assert (b[:c[0][q], 1] < n_loc).all() and (b[c[0][q]:, 1] >= n_loc).all()
            inbox[q].append(b)
    for q in range(G):
        rec = np.concatenate(inbox[q])
        assert np.array_equal(np.sort(rec[:, 1]), np.arange(n_loc + m_loc))
        out = torch.empty(n_loc + m_loc, dtype=torch.float64, device="cuda")
        ops.scatter_records(torch.from_numpy(rec).cuda(), out)
        o = out.cpu().numpy()
        assert np.array_equal(o[:n_loc], want_x[q * n_loc:(q + 1) * n_loc])
        assert np.array_equal(o[n_loc:], want_z[q * m_loc:(q + 1) * m_loc])


@pytest.mark.parametrize("G,n_loc,m_loc", [(3, 20_011, 7_003), (5, 1_000, 3), (2, 1, 1)])
def test_fixed_exchange_kernels_simulated_ranks(gpu, G, n_loc, m_loc):
    """tw_exchange_pack_fixed / tw_scatter_buckets (the default multi-rank exchange) for G
    ranks simulated in one process: bucket headers equal the oracle's forward-permutation
    histograms, the equal-split all-to-all is done on the host, and after the scatter both
    samples equal the oracle's global permutations; a capacity below a bucket's size raises
    the flag on both sides (never a silent drop)."""
    import torch
    from tuplewise.device import HipOps
    ops = HipOps()
    kx, kz = 101, 202
    rng = np.random.RandomState(5)
    X, Z = rng.normal(size=G * n_loc), rng.normal(size=G * m_loc)
    want_x, want_z = O.permute_scatter(X, kx), O.permute_scatter(Z, kz)
    tot = n_loc + m_loc
    for cap in (max(1, min(tot, tot // G + tot // (8 * G) + 1024)), None):
        hist = np.zeros((G, G), dtype=np.int64)  # [source, destination]
        for r in range(G):
            gx, gz = np.arange(r * n_loc, (r + 1) * n_loc), np.arange(r * m_loc, (r + 1) * m_loc)
            hist[r] = (np.bincount(O.feistel_perm(gx, G * n_loc, kx) // n_loc, minlength=G) +
                       np.bincount(O.feistel_perm(gz, G * m_loc, kz) // m_loc, minlength=G))
        over = cap is None
        if over:
            cap = int(hist.max()) - 1  # one bucket too small
            if cap < 1:
                continue
        sends = []
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        cursor = torch.zeros(G, dtype=torch.int64, device="cuda")
        for r in range(G):
            send = torch.empty((G * (cap + 1), 2), dtype=torch.int64, device="cuda")
            ops.exchange_pack_fixed(torch.from_numpy(X[r * n_loc:(r + 1) * n_loc]).cuda(),
                                    torch.from_numpy(Z[r * m_loc:(r + 1) * m_loc]).cuda(), r, G,
                                    kx, kz, cap, cursor, send, flag)
            s = send.cpu().numpy().reshape(G, cap + 1, 2)
            assert np.array_equal(s[:, 0, 0], hist[r])
            assert not cursor.cpu().numpy().any()  # left zero for the next repartition
            sends.append(s)
        assert bool(flag.item()) == over
        for q in range(G):
            recv = np.concatenate([sends[r][q] for r in range(G)])  # equal-split all-to-all
            out = torch.zeros(tot, dtype=torch.float64, device="cuda")
            rflag = torch.zeros(1, dtype=torch.int32, device="cuda")
            ops.scatter_buckets(torch.from_numpy(np.ascontiguousarray(recv)).cuda(), G, cap,
                                out, rflag)
            assert bool(rflag.item()) == (over and bool((hist[:, q] > cap).any()))
            if not over:
                o = out.cpu().numpy()
                assert np.array_equal(o[:n_loc], want_x[q * n_loc:(q + 1) * n_loc])
                assert np.array_equal(o[n_loc:], want_z[q * m_loc:(q + 1) * m_loc])


@pytest.mark.parametrize("loss", ["hinge", "logistic"])
@pytest.mark.parametrize("d,kx,kz", [(1, 300, 77), (10, 500, 64), (100, 1300, 5000),
                                     (512, 257, 300)])
def test_complete_block_gradient(gpu, loss, d, kx, kz):
    """tw_pair_grad_complete (extension, north_star item (2): per-point pair coefficients then
    X^T c) vs the oracle's restatement, per shard, through SWR-style row tables."""
    from tuplewise import _lib as L, _learn
    rng = np.random.RandomState(d + kx)
    N, nX, nZ = 5, 4000, 6000
    X, Z = rng.normal(size=(nX, d)), rng.normal(0.2, 1, size=(nZ, d))
    w = rng.normal(size=d) / np.sqrt(d)
    rows_x, rows_z = rng.randint(0, nX, size=(N, kx)), rng.randint(0, nZ, size=(N, kz))
    code = L.TW_LOSS_HINGE if loss == "hinge" else L.TW_LOSS_LOGISTIC
    g = _learn.complete_grads_device(L.to_device(X), L.to_device(Z), d, L.to_device(rows_x), kx,
                                     L.to_device(rows_z), kz, N, L.to_device(w), 0.5,
                                     code).cpu().numpy()
    for s in range(N):
        want = O.grad_complete_block(w.reshape(-1, 1), 0.5, loss)(X[rows_x[s]], Z[rows_z[s]])
        np.testing.assert_allclose(g[s], want.ravel(), rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("kx,kz", [(300, 77), (5000, 20000), (4096, 1)])
def test_complete_hinge_search_equals_pair_sums(gpu, kx, kz):
    """Hinge coefficients by threshold search == pair-by-pair sums, bit for bit, on
    integer-valued data where S = 0 exactly for many pairs (the boundary of 1{S > 0}), with
    NaN and +-inf scores and several sorted chunks / LDS groups."""
    from tuplewise import _lib as L, _learn
    rng = np.random.RandomState(kx + kz)
    N, d = 3, 4
    X = rng.randint(-5, 6, size=(kx * N, d)).astype(np.float64)
    Z = rng.randint(-5, 6, size=(kz * N, d)).astype(np.float64)
    X[1, 0], Z[0, 1], X[2, 2] = np.nan, np.inf, -np.inf  # shard 0 only
    w = np.array([1.0, -2.0, 0.5, 3.0])
    args = (L.to_device(X), L.to_device(Z), d, None, kx, None, kz, N, L.to_device(w), 2.0,
            L.TW_LOSS_HINGE)
    g_search = _learn.complete_grads_device(*args).cpu().numpy()
    L.call("tw_pair_grad_complete_set_search", 0)
    try:
        g_pairs = _learn.complete_grads_device(*args).cpu().numpy()
    finally:
        L.call("tw_pair_grad_complete_set_search", 1)
    assert np.array_equal(g_search, g_pairs, equal_nan=True)
    for s in range(1, N):  # finite shards: the oracle's pair-by-pair restatement
        want = O.grad_complete_block(w.reshape(-1, 1), 2.0, "hinge")(
            X[s * kx:(s + 1) * kx], Z[s * kz:(s + 1) * kz])
        np.testing.assert_array_equal(g_search[s], want.ravel())


def test_complete_logistic_large_scores(gpu):
    """Scores beyond +-350 send their (tile, chunk) to the direct-formula path of
    k_logistic_coef (the separated factors could leave the normal range), scores beyond +-40
    to the per-sigma reciprocals (no batched inversion); the gradient still matches the
    oracle, incl. saturated sigmas (S of several hundred)."""
    from tuplewise import _lib as L, _learn
    rng = np.random.RandomState(12)
    N, d, kx, kz = 4, 4, 5000, 1300
    X, Z = rng.normal(size=(kx * N, d)), rng.normal(0.3, 1, size=(kz * N, d))
    X[: kx, :] *= 300.0  # shard 0: |scores| up to ~1000 on the x side
    Z[kz:2 * kz, :] *= 250.0  # shard 1: on the z side
    X[3 * kx:, :] *= 30.0  # shard 3: |scores| in (40, 350] for some tiles (no batched sigmas)
    Z[3 * kz:, :] *= 30.0
    w = np.array([1.0, -0.5, 0.25, 0.8])
    g = _learn.complete_grads_device(L.to_device(X), L.to_device(Z), d, None, kx, None, kz, N,
                                     L.to_device(w), 0.7, L.TW_LOSS_LOGISTIC).cpu().numpy()
    for s in range(N):
        with np.errstate(over="ignore"):  # the oracle's exp saturates, as NumPy's does
            want = O.grad_complete_block(w.reshape(-1, 1), 0.7, "logistic")(
                X[s * kx:(s + 1) * kx], Z[s * kz:(s + 1) * kz])
        np.testing.assert_allclose(g[s], want.ravel(), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("kx,kz", [(300, 77), (5000, 1300), (1, 9000)])
def test_complete_logistic_one_pass_equals_two_pass(gpu, kx, kz):
    """One-pass logistic coefficients (k_logistic_coef + k_apart_final) agree with the two-pass
    pair-by-pair kernel to summation-order rounding."""
    from tuplewise import _lib as L, _learn
    rng = np.random.RandomState(kx * 7 + kz)
    N, d = 3, 6
    X, Z = rng.normal(size=(kx * N, d)), rng.normal(0.3, 1, size=(kz * N, d))
    w = rng.normal(size=d)
    args = (L.to_device(X), L.to_device(Z), d, None, kx, None, kz, N, L.to_device(w), 0.7,
            L.TW_LOSS_LOGISTIC)
    g1 = _learn.complete_grads_device(*args).cpu().numpy()
    L.call("tw_pair_grad_complete_set_search", 0)
    try:
        g2 = _learn.complete_grads_device(*args).cpu().numpy()
    finally:
        L.call("tw_pair_grad_complete_set_search", 1)
    np.testing.assert_allclose(g1, g2, rtol=1e-12, atol=1e-15)


def test_grad_complete_block_drop_in(gpu):
    """compute_stats.grad_complete_block composes with SWR_divide / UN_split like
    grad_inc_block (one launch for all shards), and with ragged user-made shard lists."""
    import tuplewise.compute_stats as cs
    rng = np.random.RandomState(2)
    X, Z = rng.normal(size=(600, 7)), rng.normal(0.5, 1, size=(250, 7))
    w = rng.normal(size=(7, 1))
    for loss in ("hinge", "logistic"):
        np.random.seed(12)
        Xs, Zs = cs.SWR_divide(X, Z, 6)
        g = cs.UN_split(Xs, Zs, cs.grad_complete_block(w, 1, loss=loss))
        np.random.seed(12)
        Xo, Zo = O.SWR_divide(X, Z, 6)
        want = O.UN_split(Xo, Zo, O.grad_complete_block(w, 1, loss))
        np.testing.assert_allclose(g, want, rtol=1e-10, atol=1e-13)
        assert g.shape == (7, 1)
    ragged_x, ragged_z = [X[:100], X[100:350]], [Z[:40], Z[40:41]]
    g = cs.UN_split(ragged_x, ragged_z, cs.grad_complete_block(w, 1))
    want = O.UN_split(ragged_x, ragged_z, O.grad_complete_block(w, 1))
    np.testing.assert_allclose(g, want, rtol=1e-10, atol=1e-13)
    one = cs.grad_complete_block(w, 1, loss="logistic")(X[:50], Z[:30])
    np.testing.assert_allclose(one, O.grad_complete_block(w, 1, "logistic")(X[:50], Z[:30]),
                               rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("dtype_name", ["f64", "i64"])
@pytest.mark.parametrize("pred_name", ["gt", "half"])
@pytest.mark.parametrize("zmax,codes", [(20000, "sort"), (16384, "bucket"), (16384, "sort"),
                                        (16384, "images"), (20000, "images"), (16384, "images1"),
                                        (16384, "images4")])
def test_device_rng_ranked_matches_plain_and_oracle(gpu, dtype_name, pred_name, zmax, codes):
    """tw_count_pairs_rng_ws (float32 images or rank codes in LDS) == tw_count_pairs_rng (score
    gathers) == oracle, on tie-heavy shards with NaN, -0.0/+0.0, +-inf and ragged sizes (incl.
    an empty one); rank codes by bucketing (nz <= 16384) and by sort + search (20000: 2 LDS
    groups); images (the default): every tied pair is decided on the scores."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(21)
    nxs, nzs = [1000, 1, 0, 4097, 3000, 500], [700, 5, 9, zmax, 1, 600]
    L.call("tw_count_rng_set_codes", {"bucket": 1, "sort": 0}.get(codes, 3))
    # images1 / images4: 1 or 4 Philox blocks per thread and iteration (default 2)
    L.call("tw_count_rng_img_set_unroll", int(codes[6:]) if codes[6:] else 2)
    if dtype_name == "f64":
        xs = [rng.randint(-20, 20, n).astype(np.float64) for n in nxs]
        zs = [rng.randint(-20, 20, n).astype(np.float64) for n in nzs]
        xs[0][:50] = np.nan
        zs[0][:30] = np.nan
        xs[3][:100] = -0.0
        zs[3][:100] = 0.0
        xs[4][:3], zs[0][30:33] = [np.inf, -np.inf, 1e300], [np.inf, -np.inf, -1e300]
        xs[5][:], zs[5][:] = 7.0, 7.0  # a degenerate shard: every score equal
        dt = L.TW_F64
    else:
        xs = [rng.randint(-30, 30, n).astype(np.int64) for n in nxs]
        zs = [rng.randint(-30, 30, n).astype(np.int64) for n in nzs]
        dt = L.TW_I64
    pred = L.TW_PRED_GT if pred_name == "gt" else L.TW_PRED_HALF
    X, Z = np.concatenate(xs), np.concatenate(zs)
    xo = np.concatenate([[0], np.cumsum(nxs)]).astype(np.int64)
    zo = np.concatenate([[0], np.cumsum(nzs)]).astype(np.int64)
    dev = lambda a: torch.from_numpy(a).cuda()
    ops = HipOps()
    B, seed, base = 12_345, 0xC0FFEE, 17
    args = (dev(X), dev(xo), dev(Z), dev(zo), len(nxs), B, seed, base, dt, pred)
    assert L.lib().tw_count_pairs_rng_work_bytes(len(nxs), max(nxs), max(nzs), dt, pred) > 0
    try:
        ranked = ops.count_rng(*args, max_nx=max(nxs), max_nz=max(nzs)).cpu().numpy()
    finally:
        L.call("tw_count_rng_set_codes", 3)
        L.call("tw_count_rng_img_set_unroll", 2)
    plain = ops.count_rng(*args).cpu().numpy()
    assert np.array_equal(ranked, plain)
    for s in range(len(nxs)):
        if nxs[s] == 0 or nzs[s] == 0:
            assert ranked[s] == 0
            continue
        i, j = O.rng_pairs(nxs[s], nzs[s], B, seed, base + s)
        a, b = xs[s][i], zs[s][j]
        want = int(np.sum(a > b)) + (int(np.sum(a >= b)) if pred_name == "half" else 0)
        assert ranked[s] == want, s


@pytest.mark.parametrize("kind", ["est_UnNT", "cs_UnNT_prod", "cs_UnNT_gini_SWR", "cs_UnNBT_AUC",
                                  "cs_UnNBT_prod_propSWR"])
def test_repeated_un_one_launch_equals_loop(gpu, kind):
    """UnNT / UnNBT count their T repetitions in one launch (_blocks.run_un_repeated): same
    value, same in-place shuffles and same RNG stream as T separate UN calls."""
    import tuplewise.compute_stats as cs
    import tuplewise.estimation as est
    rng = np.random.RandomState(4)
    X0, Z0 = rng.normal(0.3, 1, 700), rng.normal(0, 1, 500)
    f, loop = {
        "est_UnNT": (lambda X, Z: est.UnNT(X, Z, 7, 3, "SWOR"),
                     lambda X, Z: np.mean([est.UnN(X, Z, 7, "SWOR") for _ in range(3)])),
        "cs_UnNT_prod": (lambda X, Z: cs.UnNT(X, Z, 7, 3, "prop-SWOR", kernel="prod"),
                         lambda X, Z: np.mean([cs.UnN(X, Z, 7, "prop-SWOR", kernel="prod")
                                               for _ in range(3)])),
        "cs_UnNT_gini_SWR": (lambda X, Z: cs.UnNT(X, Z, 5, 2, "prop-SWR", kernel="gini"),
                             lambda X, Z: np.mean([cs.UnN(X, Z, 5, "prop-SWR", kernel="gini")
                                                   for _ in range(2)])),
        "cs_UnNBT_AUC": (lambda X, Z: cs.UnNBT(X, Z, 6, 150, 4, "SWOR", kernel="AUC"),
                         lambda X, Z: np.mean([cs.UnNB(X, Z, 6, 150, "SWOR", kernel="AUC")
                                               for _ in range(4)])),
        "cs_UnNBT_prod_propSWR": (
            lambda X, Z: cs.UnNBT(X, Z, 6, 90, 3, "prop-SWR", kernel="prod"),
            lambda X, Z: np.mean([cs.UnNB(X, Z, 6, 90, "prop-SWR", kernel="prod")
                                  for _ in range(3)])),
    }[kind]
    X1, Z1, X2, Z2 = X0.copy(), Z0.copy(), X0.copy(), Z0.copy()
    np.random.seed(9)
    a = f(X1, Z1)
    s1 = np.random.randint(0, 2**31)
    np.random.seed(9)
    b = loop(X2, Z2)
    s2 = np.random.randint(0, 2**31)
    assert a == b and s1 == s2
    assert np.array_equal(X1, X2) and np.array_equal(Z1, Z2)


@pytest.mark.parametrize("dtype_name", ["f64", "i64"])
@pytest.mark.parametrize("mode", ["gt", "half"])
def test_sorted_count_bucket_equals_sort(gpu, dtype_name, mode):
    """algo="sorted": value buckets (nz <= 16384) == sorted chunks + binary search == oracle,
    on ties, NaN, +-0, +-inf, a degenerate all-equal shard and ragged / empty shards."""
    from tuplewise import _engine as E, _lib as L
    rng = np.random.RandomState(17)
    nxs, nzs = [3000, 1, 0, 16384, 7000, 400], [2500, 3, 11, 16384, 1, 300]
    if dtype_name == "f64":
        xs = [rng.normal(0, 3, n).round(1) for n in nxs]
        zs = [rng.normal(0, 3, n).round(1) for n in nzs]
        xs[0][:40], zs[0][:25] = np.nan, np.nan
        xs[3][:50], zs[3][:50] = -0.0, 0.0
        xs[4][:2], zs[3][60:62] = [np.inf, -np.inf], [np.inf, -np.inf]
        xs[5][:], zs[5][:] = 2.5, 2.5
        dt = L.TW_F64
    else:
        xs = [rng.randint(-50, 50, n).astype(np.int64) for n in nxs]
        zs = [rng.randint(-50, 50, n).astype(np.int64) for n in nzs]
        dt = L.TW_I64
    sh = E.Shards.from_blocks(xs, zs, dt)
    got = []
    for bucket in (1, 0):
        L.call("tw_count_sorted_set_bucket", bucket)
        try:
            got.append(np.asarray(E.count_complete(sh, mode, algo="sorted")))
        finally:
            L.call("tw_count_sorted_set_bucket", 1)
    assert np.array_equal(got[0], got[1])
    for s, (x, z) in enumerate(zip(xs, zs)):
        want = int((x.reshape(-1, 1) > z.reshape(1, -1)).sum())
        if mode == "half":
            want = 2 * want + int((x.reshape(-1, 1) == z.reshape(1, -1)).sum())
        assert int(got[0][s]) == want, s


@pytest.mark.parametrize("n,d", [(1, 1), (1000, 10), (999, 33), (5000, 64), (3001, 101),
                                 (2000, 512), (700, 1000)])
@pytest.mark.parametrize("variant", [1, 0])
def test_gemv_scores_match_numpy(gpu, n, d, variant):
    """tw_gemv_f64 (evaluation_step's X.dot(w), make_exps.py:163, :170-171): a thread per row
    in index order (d <= 32, or variant 0) or one wave per row (d > 32) — both within a few
    ulp-scale of NumPy's BLAS product; odd d, d > 512 and an unaligned view included."""
    import torch
    from tuplewise import _lib as L
    rng = np.random.RandomState(n + d)
    A = rng.normal(size=(n, d))
    w = rng.normal(size=d)
    want = A.dot(w)
    L.call("tw_gemv_set_variant", variant)
    try:
        Ad, wd = torch.from_numpy(A).cuda(), torch.from_numpy(w).cuda()
        out = torch.empty(n, dtype=torch.float64, device="cuda")
        L.call("tw_gemv_f64", L.ptr(Ad), n, d, L.ptr(wd), L.ptr(out), L.stream_handle())
        scale = np.abs(A) @ np.abs(w)  # the dot product's rounding scale
        assert np.all(np.abs(out.cpu().numpy() - want) <= 1e-13 * d * scale + 1e-300)
        # an 8-B-aligned (not 16-B) view of the rows takes the thread-per-row kernel
        big = torch.from_numpy(np.concatenate([[0.0], A.reshape(-1)])).cuda()
        view = big[1:].view(n, d)
        L.call("tw_gemv_f64", L.ptr(view), n, d, L.ptr(wd), L.ptr(out), L.stream_handle())
        assert np.all(np.abs(out.cpu().numpy() - want) <= 1e-13 * d * scale + 1e-300)
    finally:
        L.call("tw_gemv_set_variant", 1)


def _hinge_both(xs, zs, margin):
    from tuplewise import _engine as E, _lib as L
    sh = E.Shards.from_blocks(xs, zs, L.TW_F64)
    srt = E.pair_sum_complete_dev(sh, L.TW_KERN_HINGE, margin, "sorted").cpu().numpy()
    prs = E.pair_sum_complete_dev(sh, L.TW_KERN_HINGE, margin, "pairs").cpu().numpy()
    return srt, prs


@pytest.mark.parametrize("sizes", [[(300, 77)], [(5000, 9000), (0, 10), (10, 0), (4096, 4097)],
                                   [(1, 1), (17000, 3), (3, 12289), (1234, 5678)]])
def test_hinge_sorted_equals_pairs(gpu, sizes):
    """tw_pair_hinge_sum_sorted (top-c sums over sorted z, double-double prefix sums) vs the
    all-pairs kernel and the oracle's conv_AUC (compute_stats.py:129-135) times the pair count,
    on ragged and empty shards, partial sorted chunks and several x-tiles.  Tolerance: rtol
    1e-12 (three summation orders of the same rounded-once terms; see hingesort.hip)."""
    rng = np.random.RandomState(len(sizes) * 31 + sizes[0][0])
    xs = [rng.normal(0.1, 1, nx) for nx, _ in sizes]
    zs = [rng.normal(0, 1, nz) for _, nz in sizes]
    for margin in (1.0, 0.0, -0.5):
        srt, prs = _hinge_both(xs, zs, margin)
        np.testing.assert_allclose(srt, prs, rtol=1e-12, atol=0)
        for s, (x, z) in enumerate(zip(xs, zs)):
            want = O.conv_AUC(margin)(x, z) * len(x) * len(z) if len(x) and len(z) else 0.0
            np.testing.assert_allclose(srt[s], want, rtol=1e-12, atol=1e-300)


def test_hinge_sorted_ties_exact(gpu):
    """Integer-valued scores: S = fl(z - x) + margin is exactly 0 for many pairs (the boundary
    of max(S, 0)) and every partial sum is an exact integer, so sorted == all-pairs == NumPy bit
    for bit; several chunks of equal keys."""
    rng = np.random.RandomState(5)
    xs = [rng.randint(-6, 7, 9000).astype(np.float64), rng.randint(-2, 3, 300).astype(np.float64)]
    zs = [rng.randint(-6, 7, 13000).astype(np.float64), np.zeros(5000)]
    for margin in (0.0, 1.0, 3.0, -2.0):
        srt, prs = _hinge_both(xs, zs, margin)
        assert np.array_equal(srt, prs)
        for s in range(2):
            want = np.maximum(zs[s][None, :] - xs[s][:, None] + margin, 0).sum()
            assert srt[s] == want


def test_hinge_sorted_nonfinite(gpu):
    """NaN / +-inf scores: the sorted path decides NumPy's elementwise outcome from counts (a NaN
    term -> NaN, an infinite term -> +inf, zero terms from x = +inf or z = -inf), one shard per
    case, next to finite shards that must stay exact."""
    inf, nan = np.inf, np.nan
    base_x, base_z = np.array([0.5, -1.0, 2.0]), np.array([1.0, 0.25, -3.0, 4.0])
    cases = [([], []), ([nan], []), ([], [nan]), ([], [inf]), ([-inf], []), ([inf], []),
             ([], [-inf]), ([inf], [inf]), ([-inf], [-inf]), ([inf], [-inf]), ([-inf], [inf])]
    xs = [np.concatenate([base_x, np.array(a, dtype=np.float64)]) for a, _ in cases]
    zs = [np.concatenate([base_z, np.array(b, dtype=np.float64)]) for _, b in cases]
    xs.append(np.array([inf, inf]))  # all x = +inf: every term 0
    zs.append(np.array([1.0, 2.0]))
    for margin in (1.0, 0.0):
        srt, prs = _hinge_both(xs, zs, margin)
        with np.errstate(invalid="ignore"):
            want = np.array([np.maximum(z[None, :] - x[:, None] + margin, 0).sum()
                             for x, z in zip(xs, zs)])
        np.testing.assert_array_equal(srt, want)
        np.testing.assert_array_equal(prs, want)
