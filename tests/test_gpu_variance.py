"""Statistical check of the device repartition against the reference's NumPy shuffle
(VERDICT r01 'Next round' item 1; the reference's own figure, estimation-experiment/main.py:
82-131, is Var(Un), Var(UnN), Var(UnNT) of the Bernoulli experiment against Var_Un / Mean_Un).

ShardedSample's repartition is a keyed Feistel permutation, not NumPy's Fisher-Yates, so it is
not bit-comparable; its estimates must be distributed like the reference's:
  * Bernoulli generators of main.py:97-101 (n = 5000, m = 50, N = 10, T = 4, prop-SWOR):
    the mean of UnNT over 2000 tries matches Mean_Un (main.py:26-27) and its variance is
    statistically equal (Levene) to the drop-in's NumPy-shuffled Monte-Carlo (est.replicate);
  * conditional on ONE data set, the spread of UnN over 2000 repartition keys equals the spread
    over 2000 NumPy shuffles (what a poorly mixing permutation would fail first).
"""
import numpy as np
import pytest
from scipy import stats

pytestmark = pytest.mark.gpu

n, m, N, T = 5000, 50, 10, 4


def _gen(rs, eps):
    return (2 * rs.binomial(1, 1 - eps, n)).astype(np.int64), \
        (2 * rs.binomial(1, eps, m) - 1).astype(np.int64)


@pytest.mark.parametrize("eps", [0.02, 0.1, 0.5])
def test_unnt_device_repartition_matches_reference_distribution(gpu, eps):
    import torch
    import tuplewise.estimation as est
    from tuplewise.device import ShardedSample
    tries = 2000
    rs = np.random.RandomState(int(eps * 1e5) + 1)
    dev = []
    for t in range(tries):
        X, Z = _gen(rs, eps)
        S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
        dev.append(S.UnNT(T, key0=1_000_003 * t))
    dev = np.array(dev)
    np.random.seed(int(eps * 1e5) + 2)
    ref = np.array(est.replicate(est.UnNT, lambda: 2 * np.random.binomial(1, 1 - eps, n),
                                 lambda: 2 * np.random.binomial(1, eps, m) - 1, tries, N, T,
                                 "prop-SWOR"))
    mu = est.Mean_Un(eps)
    for v in (dev, ref):
        assert abs(v.mean() - mu) < 5 * v.std(ddof=1) / np.sqrt(tries), (v.mean(), mu)
    p = stats.levene(dev, ref).pvalue
    assert p > 1e-3, (p, dev.var(), ref.var())


@pytest.mark.parametrize("eps", [0.1, 0.5])
def test_unn_repartition_spread_given_data(gpu, eps):
    import torch
    import tuplewise.estimation as est
    from tuplewise.device import ShardedSample
    reps = 2000
    rs = np.random.RandomState(int(eps * 1e5) + 3)
    X, Z = _gen(rs, eps)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
    dev = np.array(S.UnN_many(range(5000, 5000 + reps)))  # repartition of the current order
    np.random.seed(int(eps * 1e5) + 4)
    Xc, Zc = X.copy(), Z.copy()
    ref = np.array(est.replicate(est.UnN, lambda: Xc, lambda: Zc, reps, N, "prop-SWOR"))
    p = stats.levene(dev, ref).pvalue
    assert p > 1e-3, (p, dev.var(), ref.var())
    assert abs(dev.mean() - ref.mean()) < 5 * np.sqrt(dev.var() / reps + ref.var() / reps)
