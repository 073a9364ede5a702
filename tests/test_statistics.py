"""Statistical properties of the device-RNG draws (tw_count_pairs_rng, include/tuplewise.h).

The device-RNG mode is not NumPy's stream, so its parity is: (1) bit-exact against the
oracle's restatement (tests/test_gpu_parity.py), and (2) the sampling it restates is the
reference's — uniform, with replacement, independent i and j (cs.UB, compute_stats.py:37-42).
(2) is checked here on the restatement (CPU) and on the device estimator's mean (GPU).
"""
import numpy as np
import pytest
from scipy import stats

from oracle import oracle as O


def test_rng_indices_uniform_and_independent():
    nx, nz, B = 97, 61, 400_000
    i, j = O.rng_pairs(nx, nz, B, seed=0xABCDEF, shard=3)
    assert i.min() >= 0 and i.max() < nx and j.min() >= 0 and j.max() < nz
    for idx, n in ((i, nx), (j, nz)):
        p = stats.chisquare(np.bincount(idx, minlength=n)).pvalue
        assert p > 1e-4, p
    # independence of i and j (contingency table of coarse bins)
    tab = np.histogram2d(i, j, bins=(8, 8), range=((0, nx), (0, nz)))[0]
    assert stats.chi2_contingency(tab).pvalue > 1e-4
    # the two pairs of one Philox block are independent as well
    tab2 = np.histogram2d(i[0::2], i[1::2], bins=(8, 8), range=((0, nx), (0, nx)))[0]
    assert stats.chi2_contingency(tab2).pvalue > 1e-4


def test_rng_rejection_path_exact_and_uniform():
    """n = 2^31 + 1: (2^32 mod n) = 2^31 - 1, so about half of the words are rejected and
    redrawn — the multiply-shift without rejection would favour the lower half 2:1."""
    n = (1 << 31) + 1
    i, _ = O.rng_pairs(n, 5, 100_000, seed=77, shard=0)
    assert i.min() >= 0 and i.max() < n
    frac_low = np.mean(i < n // 2)
    assert abs(frac_low - 0.5) < 0.01, frac_low
    # different shards and seeds give different streams
    i2, _ = O.rng_pairs(n, 5, 1000, seed=77, shard=1)
    i3, _ = O.rng_pairs(n, 5, 1000, seed=78, shard=0)
    assert not np.array_equal(i[:1000], i2) and not np.array_equal(i[:1000], i3)


def test_rng_odd_B_prefix_property():
    """Pairs are a deterministic function of (seed, shard, p): B and B+1 share a prefix."""
    a = O.rng_pairs(1000, 800, 777, seed=5, shard=2)
    b = O.rng_pairs(1000, 800, 778, seed=5, shard=2)
    assert np.array_equal(a[0], b[0][:777]) and np.array_equal(a[1], b[1][:777])


@pytest.mark.gpu
def test_device_incomplete_estimator_unbiased(gpu):
    """Mean over seeds of the device UnNB equals the complete UnN of the same shards
    (each incomplete block estimate is unbiased for its complete block value)."""
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(11)
    n, N, B, reps = 20_000, 8, 5_000, 400
    X, Z = rng.normal(0.3, 1, n), rng.normal(0, 1, n)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
    complete = S.values(S.local_counts()).mean()
    ests = np.array([S.UnNB(B, 1000 + r) for r in range(reps)])
    se = ests.std(ddof=1) / np.sqrt(reps)
    assert abs(ests.mean() - complete) < 5 * se, (ests.mean(), complete, se)


@pytest.mark.gpu
def test_device_rng_rejection_path_matches_oracle(gpu):
    """A shard of 2^31 + 1 x-values (17 GB): half the index words take the rejection path;
    the device count equals the oracle's on the same draws."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    n = (1 << 31) + 1
    X = torch.zeros(n, dtype=torch.float64, device="cuda")
    X[n // 2:] = 1.0
    Z = torch.full((3,), 0.5, dtype=torch.float64, device="cuda")
    x_off = torch.tensor([0, n], dtype=torch.int64, device="cuda")
    z_off = torch.tensor([0, 3], dtype=torch.int64, device="cuda")
    B, seed = 20_001, 0x5EED
    out = HipOps().count_rng(X, x_off, Z, z_off, 1, B, seed, 0, L.TW_F64, L.TW_PRED_GT)
    i, _ = O.rng_pairs(n, 3, B, seed, 0)
    assert int(out[0]) == int(np.sum(i >= n // 2))
    del X
    torch.cuda.empty_cache()


# ------------------------------------------------------------ repartition and SWR draws
# The device repartition (csrc/permute.hip, restated by oracle.feistel_perm bit for bit) and
# the learning loop's device draws (tw_swr_rows_rng / tw_pair_grad_rng, oracle._sgd_draw) stand
# in for NumPy's shuffle (compute_stats.py:66-67) and randint (:52-53, :155-156).  Their
# restatements are checked here for the properties those reference calls have.

@pytest.mark.parametrize("n", [10, 1000, 4099])
def test_feistel_positions_uniform_over_keys(n):
    """Over many keys, where element 0 lands and where (0, 1) land jointly are uniform."""
    keys = 6000
    p0, p1 = np.empty(keys, np.int64), np.empty(keys, np.int64)
    for k in range(keys):
        p0[k], p1[k] = O.feistel_perm(np.array([0, 1]), n, 0x51ED + 7919 * k)
    assert np.all(p0 != p1)
    bins = min(n, 20)
    h = np.bincount(p0 * bins // n, minlength=bins)
    assert stats.chisquare(h).pvalue > 1e-4
    if n <= 16:  # the ordered pair (perm(0), perm(1)) uniform over the n(n-1) cells
        cells = np.bincount(p0 * n + p1, minlength=n * n).reshape(n, n)
        assert stats.chisquare(cells[~np.eye(n, dtype=bool)]).pvalue > 1e-4
    else:  # coarse bins: distinctness is a negligible dependence
        tab = np.histogram2d(p0, p1, bins=(8, 8), range=((0, n), (0, n)))[0]
        assert stats.chi2_contingency(tab).pvalue > 1e-4


def test_feistel_full_permutation_bias_small_n_documented():
    """Limitation kept visible: on the tiniest domains the keyed Feistel
    family is NOT uniform over all n! permutations (n = 3 is, n = 4 measurably is not), while
    its low-order marginals stay uniform (above).  No keyed family can reach all n!
    permutations once n! > 2^64 (n >= 21) anyway; the estimators depend on the shard
    composition, whose distribution the variance tests (tests/test_gpu_variance.py) check."""
    from collections import Counter
    c3 = Counter(tuple(O.feistel_perm(np.arange(3), 3, k * 2654435761 + 17)) for k in range(6000))
    assert len(c3) == 6 and stats.chisquare(list(c3.values())).pvalue > 1e-4
    c4 = Counter(tuple(O.feistel_perm(np.arange(4), 4, k * 2654435761 + 17)) for k in range(24000))
    assert len(c4) == 24 and stats.chisquare(list(c4.values())).pvalue < 1e-6


def test_feistel_is_a_bijection_and_keys_independent():
    n = 100_003
    a = O.feistel_perm(np.arange(n), n, 123)
    b = O.feistel_perm(np.arange(n), n, 124)
    assert np.array_equal(np.sort(a), np.arange(n)) and np.array_equal(np.sort(b), np.arange(n))
    assert np.array_equal(O.feistel_perm_inv(a, n, 123), np.arange(n))
    # consecutive keys give unrelated permutations (the repartitions of UnNT's T steps)
    assert abs(stats.spearmanr(a, b).correlation) < 0.02
    assert abs(stats.spearmanr(np.arange(n), a).correlation) < 0.02
    # the fraction of a shard that stays in the same shard is the hypergeometric mean 1/N
    N = 64
    same = np.mean(a * N // n == np.arange(n) * N // n)
    assert abs(same - 1 / N) < 0.003, same


def test_sgd_device_draws_uniform_and_independent():
    """SWR_divide rows (tag 0x40000000) and grad_inc_block pairs (tag 0x80000000) drawn on the
    device: uniform over their ranges, independent across shards and steps."""
    seed, n, k = 0xABC, 9117, 20_000
    rows = [O._mulhi64(O._sgd_draw(seed, 0, np.arange(k), s, 0x40000000)[0], n)
            for s in range(3)]
    for r in rows:
        assert r.min() >= 0 and r.max() < n
        assert stats.chisquare(np.bincount(r * 50 // n, minlength=50)).pvalue > 1e-4
    tab = np.histogram2d(rows[0], rows[1], bins=(8, 8), range=((0, n), (0, n)))[0]
    assert stats.chi2_contingency(tab).pvalue > 1e-4
    u0, v0 = O._sgd_draw(seed, 5, np.arange(k), 2, 0x80000000)
    u1, _ = O._sgd_draw(seed, 6, np.arange(k), 2, 0x80000000)
    i0, j0, i1 = O._mulhi64(u0, 91), O._mulhi64(v0, 7), O._mulhi64(u1, 91)
    assert stats.chisquare(np.bincount(i0, minlength=91)).pvalue > 1e-4
    assert stats.chisquare(np.bincount(j0, minlength=7)).pvalue > 1e-4
    assert stats.chi2_contingency(np.histogram2d(i0, j0, bins=(7, 7))[0]).pvalue > 1e-4
    assert stats.chi2_contingency(np.histogram2d(i0, i1, bins=(7, 7))[0]).pvalue > 1e-4
