"""In-repo generator of the shuttle-shaped learning problem (test fixture data, not reference
code).  The reference trains on ODDS shuttle (learning-experiment/make_exps.py:51-93), a
download absent offline; SURVEY.md §8(c) fixes the shapes its `~ind` split gives: 9117 x 10
negatives / 702 x 10 positives for training, 2279 x 10 / 175 x 10 for testing (9 features +
the constant column load_preprocess_data appends).  Seeded legacy RandomState: the same rows on
every NumPy version, so tests/golden/golden.npz stores only what the reference computed on
them (make_golden.py section 5c)."""
import numpy as np

N_X, N_Z, T_X, T_Z, D = 9117, 702, 2279, 175, 9
MONITOR_PAIRS = 20_000  # make_exps.py:216-221 draws 450 000; fewer keep the fixture small


def shuttle_problem(seed: int = 20260):
    rng = np.random.RandomState(seed)

    def rows(n, mu, sd):
        return np.hstack([rng.normal(mu, sd, size=(n, D)), np.ones((n, 1))])

    X, Z = rows(N_X, 0.0, 1.0), rows(N_Z, 0.6, 1.2)
    tX, tZ = rows(T_X, 0.0, 1.0), rows(T_Z, 0.6, 1.2)
    w0 = rng.normal(0, 1, (D + 1, 1))
    mon = list(zip(rng.randint(0, N_X, MONITOR_PAIRS).tolist(),
                   rng.randint(0, N_Z, MONITOR_PAIRS).tolist()))
    return X, Z, tX, tZ, w0, mon


def large_inputs(spec: dict):
    """Inputs of the large-n goldens (make_golden_large.py, tests/test_gpu_large_golden.py):
    `RandomState(data_seed).normal(loc_x, 1, n)` then `.normal(0, 1, m)`, rounded to
    `round` decimals when the case names it (tie-heavy scores).  Regenerated on the GPU box,
    so golden_large.json holds only seeds, values and hashes."""
    rng = np.random.RandomState(spec["data_seed"])
    X = rng.normal(spec["loc_x"], 1, spec["n"])
    Z = rng.normal(0.0, 1, spec["m"])
    if spec.get("round") is not None:
        X, Z = X.round(spec["round"]), Z.round(spec["round"])
    return X, Z
