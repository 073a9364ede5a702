"""The oracle (oracle/oracle.py) against golden vectors produced by the reference itself.
Pins the CPU restatement before it is used as the checker of the HIP path."""
import numpy as np
import pytest

from oracle import oracle as O

CASES = ["gauss", "bern_int64", "ties_int", "edge_float", "n1", "m1", "ragged", "int64_wrap",
         "float32", "col_scores"]


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and (np.array_equal(a, b) or np.array_equal(a, b, equal_nan=True))


@pytest.mark.parametrize("case", CASES)
def test_un_cases(golden, case):
    X, Z = golden[f"un/{case}/X"], golden[f"un/{case}/Z"]
    with np.errstate(all="ignore"):
        assert same(O.est_Un(X, Z), golden[f"un/{case}/est_Un"])
        assert same(O.cs_Un(X, Z, "AUC"), golden[f"un/{case}/cs_AUC"])
        if f"un/{case}/cs_prod" in golden:
            assert same(O.cs_Un(X, Z, "prod"), golden[f"un/{case}/cs_prod"])
            assert same(O.cs_Un(X, Z, "gini"), golden[f"un/{case}/cs_gini"])
            assert same(O.conv_AUC(1)(X, Z), golden[f"un/{case}/conv_AUC"])
    # the integer count behind est.Un
    n = np.asarray(X).size * np.asarray(Z).size
    assert np.float64(O.un_count(X, Z)) / np.float64(n) == golden[f"un/{case}/est_Un"]


def _sharded_fns():
    return {
        "est_UnN_propSWOR": lambda X, Z: O.est_UnN(X, Z, 10, "prop-SWOR"),
        "est_UnN_SWOR": lambda X, Z: O.est_UnN(X, Z, 10, "SWOR"),
        "est_UnN_propSWR": lambda X, Z: O.est_UnN(X, Z, 10, "prop-SWR"),
        "est_UnNT_propSWOR": lambda X, Z: O.est_UnNT(X, Z, 10, 4, "prop-SWOR"),
        "est_UnNT_bern": lambda X, Z: O.est_UnNT(X, Z, 10, 4, "prop-SWOR"),
        "est_UnN_SWOR_degenerate": lambda X, Z: O.est_UnN(X, Z, 40, "SWOR"),
        "est_UnN_prop_degenerate": lambda X, Z: O.est_UnN(X, Z, 40, "prop-SWOR"),
        "cs_UnN_AUC": lambda X, Z: O.cs_UnN(X, Z, 10, "prop-SWOR", "AUC"),
        "cs_UnN_AUC_SWOR": lambda X, Z: O.cs_UnN(X, Z, 10, "SWOR", "AUC"),
        "cs_UnN_prod": lambda X, Z: O.cs_UnN(X, Z, 10, "prop-SWOR"),
        "cs_UnN_gini_SWR": lambda X, Z: O.cs_UnN(X, Z, 10, "prop-SWR", "gini"),
        "cs_UnNB_AUC": lambda X, Z: O.cs_UnNB(X, Z, 10, 500, "prop-SWOR", "AUC"),
        "cs_UnNB_AUC_SWR": lambda X, Z: O.cs_UnNB(X, Z, 10, 300, "prop-SWR", "AUC"),
        "cs_UnNBT_AUC": lambda X, Z: O.cs_UnNBT(X, Z, 10, 200, 3, "SWOR", "AUC"),
        "cs_UnNT_AUC": lambda X, Z: O.cs_UnNT(X, Z, 10, 3, "prop-SWOR", "AUC"),
        "cs_UnNB_prod": lambda X, Z: O.cs_UnNB(X, Z, 10, 400, "prop-SWOR"),
    }


@pytest.mark.parametrize("name", list(_sharded_fns()))
def test_sharded(golden, name):
    fn = _sharded_fns()[name]
    X, Z = golden[f"sh/{name}/X"].copy(), golden[f"sh/{name}/Z"].copy()
    np.random.seed(int(golden[f"sh/{name}/seed"]))
    with np.errstate(all="ignore"), _nowarn():
        val = fn(X, Z)
    assert same(val, golden[f"sh/{name}/value"])
    assert same(X, golden[f"sh/{name}/X_after"]) and same(Z, golden[f"sh/{name}/Z_after"])
    assert np.random.randint(0, 2 ** 31 - 1) == golden[f"sh/{name}/probe"]


class _nowarn:
    def __enter__(self):
        import warnings
        self._c = warnings.catch_warnings()
        self._c.__enter__()
        warnings.simplefilter("ignore")

    def __exit__(self, *a):
        return self._c.__exit__(*a)


def test_indexed(golden):
    X, Z, ix, iz = golden["idx/X"], golden["idx/Z"], golden["idx/ix"], golden["idx/iz"]
    for k in ("AUC", "prod", "gini"):
        assert same(O.UB_indices(X, Z, ix, iz, k), golden[f"idx/UB_indices_{k}"])
    pairs = list(zip(list(ix), list(iz)))
    assert same(O.UB_pairs(X, Z, pairs, "AUC"), golden["idx/UB_pairs_AUC"])
    assert same(O.conv_AUC_deter_pairs(1)(X, Z, pairs), golden["idx/conv_deter"])
    np.random.seed(77)
    assert same(O.UB(X, Z, 1000, "AUC"), golden["idx/UB_AUC_seed77"])


def test_grad(golden):
    X, Z, w = golden["grad/X"], golden["grad/Z"], golden["grad/w"]
    np.random.seed(5)
    assert same(O.grad_inc_block(w, 100, 1)(X, Z), golden["grad/single_seed5"])
    np.random.seed(6)
    Xs, Zs = O.SWR_divide(X, Z, 10)
    assert same(O.UN_split(Xs, Zs, O.grad_inc_block(w, 50, 1)), golden["grad/split_seed6"])


def test_learning_trajectory(golden):
    p = {"n_it": 300, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
         "learning_rate": 0.01, "w_init": golden["learn/w0"]}
    np.random.seed(2024)
    ws, _ = O.learning_trajectory(golden["learn/X"], golden["learn/Z"], p)
    ref = golden["learn/ws"]
    assert len(ws) == len(ref)
    # the reference evaluates (no RNG draws in FIXED_PAIRS mode) -> trajectories identical
    assert np.array_equal(np.stack(ws), ref)


def test_rng_kat(golden):
    np.random.seed(9)
    assert np.array_equal(np.random.randint(0, 1000, 64), golden["rng/randint_seed9"])


def test_exact_large_count_agrees():
    rng = np.random.RandomState(0)
    X, Z = rng.randint(-50, 50, 3000), rng.randint(-50, 50, 2000)
    assert O.count_gt_sorted(X, Z) == O.un_count(X, Z)
    gt = O.un_count(X, Z)
    eq = int((X.reshape(-1, 1) == Z.reshape(1, -1)).sum())
    assert O.count_half_sorted(X, Z) == 2 * gt + eq


def test_theory_matches_monte_carlo():
    """Mean_Un / Var_Un (estimation-experiment/main.py:10-27, :103-104) vs simulation."""
    rng = np.random.RandomState(3)
    n, m, e, tries = 500, 50, 0.1, 3000
    vals = []
    for _ in range(tries):
        X = 2 * rng.binomial(1, 1 - e, n)
        Z = 2 * rng.binomial(1, e, m) - 1
        vals.append(O.count_gt_sorted(X, Z) / (n * m))
    assert abs(np.mean(vals) - O.Mean_Un(e)) < 4 * np.sqrt(O.Var_Un(e, n, m) / tries)
    assert 0.9 < np.var(vals) / O.Var_Un(e, n, m) < 1.1


def test_feistel_is_bijection():
    for n in (1, 2, 3, 17, 1000, 4097):
        p = O.feistel_perm(np.arange(n), n, key=12345)
        assert np.array_equal(np.sort(p), np.arange(n))


def test_feistel_inverse_undoes_forward():
    for n in (1, 2, 3, 17, 1000, 4097, 100_003):
        i = np.arange(n)
        p = O.feistel_perm(i, n, key=777)
        assert np.array_equal(O.feistel_perm_inv(p, n, key=777), i)


def test_logistic_gradient_is_the_derivative_of_its_loss():
    """Row L3 (pairwise logistic, not in the reference: parity unpinned against it): the
    oracle's gradient equals the finite-difference gradient of its own surrogate loss,
    (1/B) sum_b softplus(diff_b . w + margin)."""
    rng = np.random.RandomState(3)
    B, d, margin = 50, 6, 0.7
    diff = rng.normal(size=(B, d))
    w = rng.normal(size=(d, 1))

    def loss(wv):
        return O._surrogate(diff.dot(wv).ravel() + margin, "logistic").sum() / B

    g = O.pair_grad(diff, w, margin, B, "logistic").ravel()
    h = 1e-6
    fd = np.array([(loss(w + h * e[:, None]) - loss(w - h * e[:, None])) / (2 * h)
                   for e in np.eye(d)])
    np.testing.assert_allclose(g, fd, rtol=1e-7, atol=1e-9)
    # and the hinge restatement is the subgradient of its loss away from the kinks
    gh = O.pair_grad(diff, w, margin, B, "hinge").ravel()
    fdh = np.array([(O._surrogate(diff.dot(w + h * e[:, None]).ravel() + margin, "hinge").sum()
                     - O._surrogate(diff.dot(w - h * e[:, None]).ravel() + margin,
                                    "hinge").sum()) / (2 * h * B) for e in np.eye(d)])
    np.testing.assert_allclose(gh, fdh, rtol=1e-6, atol=1e-9)


def test_complete_gradient_factorisation():
    """The complete-block gradient's per-point factorisation (north_star item (2), an extension
    with no reference counterpart) equals the plain double sum over pairs, and for the
    logistic loss the finite-difference gradient of mean_ij softplus(S_ij)."""
    rng = np.random.RandomState(8)
    X, Z = rng.normal(size=(37, 5)), rng.normal(0.3, 1, size=(23, 5))
    w = rng.normal(size=(5, 1))
    for loss, margin in (("hinge", 1.0), ("logistic", 0.4)):
        g = O.grad_complete_block(w, margin, loss)(X, Z).ravel()
        brute = np.zeros(5)
        for i in range(len(X)):
            for j in range(len(Z)):
                dlt = Z[j] - X[i]
                S = dlt.dot(w.ravel()) + margin
                wt = (S > 0) if loss == "hinge" else 1 / (1 + np.exp(-S))
                brute += wt * dlt
        np.testing.assert_allclose(g, brute / (len(X) * len(Z)), rtol=1e-12, atol=1e-15)

    def loss_fn(wv):
        S = Z.dot(wv).ravel()[None, :] - X.dot(wv).ravel()[:, None] + 0.4
        return np.logaddexp(0, S).mean()

    h = 1e-6
    fd = np.array([(loss_fn(w + h * e[:, None]) - loss_fn(w - h * e[:, None])) / (2 * h)
                   for e in np.eye(5)])
    np.testing.assert_allclose(O.grad_complete_block(w, 0.4, "logistic")(X, Z).ravel(), fd,
                               rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("mod", [1, 10000])
def test_learning_trajectory_reference_shape(golden, mod):
    """The reference's own p_learn shape (make_exps.py:210-214: N = 100, B = 100) on the
    shuttle-shaped rows of tests/golden/shapes.py at both ends of the reshuffle sweep
    (learning-experiment/main.py:20): the oracle's loop reproduces the reference's w at every
    step bit for bit."""
    from golden.shapes import shuttle_problem
    X, Z, _, _, w0, _ = shuttle_problem()
    p = {"n_it": 250, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": mod, "reg": 0.05,
         "learning_rate": 0.01, "w_init": w0}
    np.random.seed(3000 + mod)
    ws, _ = O.learning_trajectory(X, Z, p)
    assert np.array_equal(np.stack(ws), golden[f"shuttle_mod{mod}/ws"])
