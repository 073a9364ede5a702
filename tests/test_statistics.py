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
