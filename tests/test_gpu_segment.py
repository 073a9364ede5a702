"""Wide rows (32 < d <= 512: per-step gradient launches) with the device RNG drawing each
reshuffle's SWR rows in the gradient kernel (learning.SWR_IN_KERNEL) against the row-table
path: the same statistics bit for bit.  (The wide persistent segment kernel these tests once
covered, tw_sgd_segment, measured slower than the per-step launches at C5 and was removed in
round 5.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mod", [1, 3, 10])
def test_wide_swr_in_kernel_equals_row_tables(gpu, mod, monkeypatch):
    """learning.SWR_IN_KERNEL for wide rows (d = 64: per-step gradient launches,
    tw_pair_grad_rng_swr drawing each reshuffle's rows in the kernel, segments cut at
    evaluations only) against the row-table path: the same statistics bit for bit."""
    import tuplewise.learning as lr
    rng = np.random.RandomState(5)
    n, d = 3000, 64
    X = rng.normal(0.3, 1.0, size=(n, d))
    Z = rng.normal(0.0, 1.0, size=(n, d))
    hist = {}
    for swr in (True, False):
        monkeypatch.setattr(lr, "SWR_IN_KERNEL", swr)
        mon = np.random.RandomState(2)
        p = {"N": 8, "B": 64, "margin": 1.0, "reg": 0.01, "learning_rate": 0.05,
             "n_it": 47, "reshuffle_mod": mod, "eval_mod": 20, "w_init": np.full((d, 1), 0.01),
             "test_X": X[:400], "test_Z": Z[:400], "train_X": X, "train_Z": Z,
             "train_mon_pairs": list(zip(mon.randint(0, n, 300), mon.randint(0, n, 300)))}
        np.random.seed(9)
        lr.learning_process(X, Z, p, rng_mode="device")
        hist[swr] = p
    for k in ("norm_w", "bc_AUC", "br_AUC", "tc_AUC", "tr_AUC"):
        assert hist[True][k] == hist[False][k], k
