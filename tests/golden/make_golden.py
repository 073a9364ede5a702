"""Generate golden vectors by running the REFERENCE implementation (this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports /root/reference/{estimation-experiment/main.py, learning-experiment/compute_stats.py,
learning-experiment/make_exps.py} read-only via importlib and records inputs + outputs as
data (golden.npz, no pickles).  Nothing from the reference is copied; only its results.
The GPU box never runs this script (the reference is absent there).
"""
from __future__ import annotations

import importlib.util
import json
import logging
import os
import pathlib
import sys

import numpy as np

REF = pathlib.Path(os.environ.get("TW_REFERENCE", "/root/reference"))
OUT = pathlib.Path(__file__).resolve().parent


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    sys.dont_write_bytecode = True
    est = _load("ref_est_main", REF / "estimation-experiment" / "main.py")
    sys.path.insert(0, str(REF / "learning-experiment"))  # make_exps does `import compute_stats`
    cs = _load("compute_stats", REF / "learning-experiment" / "compute_stats.py")
    sys.modules["compute_stats"] = cs
    me = _load("ref_make_exps", REF / "learning-experiment" / "make_exps.py")

    arrays: dict[str, np.ndarray] = {}
    meta: dict = {"cases": []}

    def put(key, a):
        arrays[key] = np.asarray(a)

    # ---------------------------------------------------------------- 1. complete Un cases
    rng = np.random.RandomState(1234)
    cases = {
        "gauss": (rng.normal(0.5, 1, 700), rng.normal(0, 1, 500)),
        "bern_int64": (2 * rng.binomial(1, 1 - 0.1, 900), 2 * rng.binomial(1, 0.1, 60) - 1),
        "ties_int": (rng.randint(-5, 6, 400), rng.randint(-5, 6, 333)),
        "edge_float": (np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, 1e-320, -1e-320, 5e-324, 1.0,
                                 np.finfo(float).max, -np.finfo(float).max]),
                       np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e-320, 0.0, 1.0,
                                 np.finfo(float).max])),
        "n1": (np.array([0.3]), rng.normal(size=77)),
        "m1": (rng.normal(size=65), np.array([0.1])),
        "ragged": (rng.normal(size=257), rng.normal(size=1029)),
        "int64_wrap": (np.array([2 ** 62, -2 ** 62, 2 ** 63 - 1, -2 ** 63, 5, 0], dtype=np.int64),
                       np.array([-2 ** 62 - 1, 2 ** 62, -1, 1, 0], dtype=np.int64)),
        "float32": (rng.normal(size=300).astype(np.float32), rng.normal(size=200).astype(np.float32)),
        "col_scores": (rng.normal(size=(150, 1)), rng.normal(size=(90, 1))),
    }
    for name, (X, Z) in cases.items():
        put(f"un/{name}/X", X)
        put(f"un/{name}/Z", Z)
        with np.errstate(all="ignore"):
            put(f"un/{name}/est_Un", est.Un(X, Z))
            put(f"un/{name}/cs_AUC", cs.Un(X, Z, kernel="AUC"))
            finite = np.all(np.isfinite(X.astype(float))) and np.all(np.isfinite(Z.astype(float)))
            if finite and X.dtype.kind == "f":
                put(f"un/{name}/cs_prod", cs.Un(X, Z, kernel="prod"))
                put(f"un/{name}/cs_gini", cs.Un(X, Z, kernel="gini"))
                put(f"un/{name}/conv_AUC", cs.conv_AUC(1)(X, Z))
        meta["cases"].append(name)

    # ---------------------------------------------------------------- 2. sharded estimators
    def seeded(seed, fn, X, Z):
        Xc, Zc = X.copy(), Z.copy()
        np.random.seed(seed)
        val = fn(Xc, Zc)
        return val, Xc, Zc, np.random.randint(0, 2 ** 31 - 1)  # RNG-state probe after the call

    Xg, Zg = rng.normal(0.5, 1, 1000), rng.normal(0, 1, 1000)  # config C1 shape
    Xb = 2 * rng.binomial(1, 1 - 0.02, 500)  # Bernoulli (int64) like main.py:97-101
    Zb = 2 * rng.binomial(1, 0.02, 50) - 1
    est_calls = {
        "est_UnN_propSWOR": (lambda X, Z: est.UnN(X, Z, 10, "prop-SWOR"), Xg, Zg),
        "est_UnN_SWOR": (lambda X, Z: est.UnN(X, Z, 10, "SWOR"), Xg, Zg),
        "est_UnN_propSWR": (lambda X, Z: est.UnN(X, Z, 10, "prop-SWR"), Xg, Zg),
        "est_UnNT_propSWOR": (lambda X, Z: est.UnNT(X, Z, 10, 4, "prop-SWOR"), Xg, Zg),
        "est_UnNT_bern": (lambda X, Z: est.UnNT(X, Z, 10, 4, "prop-SWOR"), Xb, Zb),
        "est_UnN_SWOR_degenerate": (lambda X, Z: est.UnN(X, Z, 40, "SWOR"), Xb[:60], Zb[:6]),
        "est_UnN_prop_degenerate": (lambda X, Z: est.UnN(X, Z, 40, "prop-SWOR"), Xb[:30], Zb[:50]),
        "cs_UnN_AUC": (lambda X, Z: cs.UnN(X, Z, 10, "prop-SWOR", kernel="AUC"), Xg, Zg),
        "cs_UnN_AUC_SWOR": (lambda X, Z: cs.UnN(X, Z, 10, "SWOR", kernel="AUC"), Xg, Zg),
        "cs_UnN_prod": (lambda X, Z: cs.UnN(X, Z, 10, "prop-SWOR"), Xg, Zg),
        "cs_UnN_gini_SWR": (lambda X, Z: cs.UnN(X, Z, 10, "prop-SWR", kernel="gini"), Xg, Zg),
        "cs_UnNB_AUC": (lambda X, Z: cs.UnNB(X, Z, 10, 500, "prop-SWOR", kernel="AUC"), Xg, Zg),
        "cs_UnNB_AUC_SWR": (lambda X, Z: cs.UnNB(X, Z, 10, 300, "prop-SWR", kernel="AUC"), Xg, Zg),
        "cs_UnNBT_AUC": (lambda X, Z: cs.UnNBT(X, Z, 10, 200, 3, "SWOR", kernel="AUC"), Xg, Zg),
        "cs_UnNT_AUC": (lambda X, Z: cs.UnNT(X, Z, 10, 3, "prop-SWOR", kernel="AUC"), Xg, Zg),
        "cs_UnNB_prod": (lambda X, Z: cs.UnNB(X, Z, 10, 400, "prop-SWOR"), Xg, Zg),
    }
    meta["sharded"] = []
    for i, (name, (fn, X, Z)) in enumerate(est_calls.items()):
        seed = 100 + i
        val, Xs, Zs, probe = seeded(seed, fn, X, Z)
        put(f"sh/{name}/X", X)
        put(f"sh/{name}/Z", Z)
        put(f"sh/{name}/value", val)
        put(f"sh/{name}/X_after", Xs)
        put(f"sh/{name}/Z_after", Zs)
        put(f"sh/{name}/seed", seed)
        put(f"sh/{name}/probe", probe)
        meta["sharded"].append(name)

    # ---------------------------------------------------------------- 3. indexed estimators
    sx, sz = rng.normal(size=400), rng.normal(size=300)
    ix, iz = rng.randint(0, 400, 5000), rng.randint(0, 300, 5000)
    put("idx/X", sx)
    put("idx/Z", sz)
    put("idx/ix", ix)
    put("idx/iz", iz)
    for k in ("AUC", "prod", "gini"):
        put(f"idx/UB_indices_{k}", cs.UB_indices(sx, sz, ix, iz, k))
    pairs = list(zip(list(ix), list(iz)))
    put("idx/UB_pairs_AUC", cs.UB_pairs(sx, sz, pairs, "AUC"))
    put("idx/conv_deter", cs.conv_AUC_deter_pairs(1)(sx, sz, pairs))
    np.random.seed(77)
    put("idx/UB_AUC_seed77", cs.UB(sx, sz, 1000, kernel="AUC"))

    # ---------------------------------------------------------------- 4. hinge gradient
    d = 10
    GX, GZ = rng.normal(size=(911, d)), rng.normal(0.3, 1, size=(70, d))
    w = rng.normal(size=(d, 1))
    put("grad/X", GX)
    put("grad/Z", GZ)
    put("grad/w", w)
    np.random.seed(5)
    g1 = cs.grad_inc_block(w, 100, 1)(GX, GZ)
    put("grad/single_seed5", g1)
    np.random.seed(6)
    Xs_, Zs_ = cs.SWR_divide(GX, GZ, 10)
    gs = cs.UN_split(Xs_, Zs_, cs.grad_inc_block(w, 50, 1))
    put("grad/split_seed6", gs)

    # ---------------------------------------------------------------- 5. learning trajectory
    lx = rng.normal(size=(911, 9))
    lz = rng.normal(0.7, 1.3, size=(70, 9))
    lx = np.hstack([lx, np.ones((911, 1))])
    lz = np.hstack([lz, np.ones((70, 1))])
    tx = np.hstack([rng.normal(size=(228, 9)), np.ones((228, 1))])
    tz = np.hstack([rng.normal(0.7, 1.3, size=(17, 9)), np.ones((17, 1))])
    w0 = rng.normal(0, 1, (10, 1))
    mon = list(zip(list(rng.randint(0, 911, 4000)), list(rng.randint(0, 70, 4000))))
    p_learn = {"n_it": 300, "margin": 1, "N": 10, "B": 20, "reshuffle_mod": 5, "reg": 0.05,
               "learning_rate": 0.01, "eval_mod": 25, "w_init": w0, "test_X": tx, "test_Z": tz,
               "train_mon_pairs": mon, "train_X": lx, "train_Z": lz}
    captured = []
    orig = cs.grad_inc_block

    def hook(w_, B_, m_):
        captured.append(np.array(w_, copy=True))
        return orig(w_, B_, m_)

    cs.grad_inc_block = hook
    logging.disable(logging.CRITICAL)
    np.random.seed(2024)
    me.learning_process(lx, lz, p_learn)
    cs.grad_inc_block = orig
    put("learn/X", lx)
    put("learn/Z", lz)
    put("learn/test_X", tx)
    put("learn/test_Z", tz)
    put("learn/w0", w0)
    put("learn/mon", np.array(mon, dtype=np.int64))
    put("learn/ws", np.stack(captured))
    for k in ("iter", "norm_w", "bc_AUC", "br_AUC", "tr_AUC", "tc_AUC"):
        put(f"learn/{k}", np.array(p_learn[k]))
    meta["learn"] = {k: v for k, v in p_learn.items()
                     if isinstance(v, (int, float)) and not isinstance(v, bool)}
    meta["learn"]["seed"] = 2024

    # ------------------------------------------- 5b. learning with SAME_AS_BATCH monitoring
    # evaluation_step's other branch (make_exps.py:154-160): the block statistics on the
    # current shards instead of the fixed monitor pairs; the module constant switched for this
    # run only
    me.TYPE_TRAIN_MONITOR = "SAME_AS_BATCH"
    p_sab = {k: v for k, v in p_learn.items()
             if k not in ("iter", "norm_w", "bc_AUC", "br_AUC", "tr_AUC", "tc_AUC")}
    p_sab["n_it"] = 120
    np.random.seed(2025)
    me.learning_process(lx, lz, p_sab)
    me.TYPE_TRAIN_MONITOR = "FIXED_PAIRS"
    for k in ("iter", "norm_w", "bc_AUC", "br_AUC", "tr_AUC", "tc_AUC"):
        put(f"learn_sab/{k}", np.array(p_sab[k]))
    meta["learn_sab"] = {"seed": 2025, "n_it": 120, "TYPE_TRAIN_MONITOR": "SAME_AS_BATCH"}

    # ---------------------------------------------------------------- 7. data preprocessing
    # load_preprocess_data (make_exps.py:51-93) on a synthetic shuttle-like pickle written to
    # a temp dir (the real dataset is a download, absent offline).  Written by us, read by the
    # reference: no reference-shipped file is unpickled.
    import pickle
    import tempfile
    pre_X = np.round(rng.normal(size=(1530, 9)) * 10, 1)
    pre_y = np.where(rng.rand(1530) < 0.08, 1, -1)
    with tempfile.TemporaryDirectory() as td:
        cwd = os.getcwd()
        os.chdir(td)
        try:
            with open("shuttle.pickle", "wb") as fh:
                pickle.dump({"X": pre_X, "y": pre_y}, fh)
            Zt, Xt, Zs, Xs = me.load_preprocess_data()
        finally:
            os.chdir(cwd)
    put("pre/X", pre_X)
    put("pre/y", pre_y)
    for k, v in (("Z_train", Zt), ("X_train", Xt), ("Z_test", Zs), ("X_test", Xs)):
        put(f"pre/{k}", v)

    # ---------------------------------------------------------------- 6. RNG stream KAT
    np.random.seed(9)
    put("rng/randint_seed9", np.random.randint(0, 1000, 64))
    np.random.seed(9)
    perm = np.arange(50)
    np.random.shuffle(perm)
    put("rng/shuffle50_seed9", perm)

    # ------------------------- 5c. learning at the reference's own shape and reshuffle sweep
    # p_learn defaults of make_exps.py:210-214 (N = 100, B = 100, margin 1, reg 0.05, lr 0.01,
    # eval_mod 25) on shuttle-shaped synthetic rows (9117 x 10 / 702 x 10 train, 2279 x 10 /
    # 175 x 10 test: the sizes the `~ind` split gives on ODDS shuttle), at the
    # two ends of the paper's reshuffle sweep (learning-experiment/main.py:20): reshuffle_mod 1
    # (a new SWR draw before every step) and 10000 (one draw for the whole run).  The rows come
    # from the in-repo generator tests/golden/shapes.py (seeded legacy RandomState), so only
    # the trajectories and the evaluation lists are stored.
    from shapes import shuttle_problem
    sx, sz, stx, stz, sw0, smon = shuttle_problem()
    for mod in (1, 10000):
        p_sh = {"n_it": 250, "margin": 1, "N": 100, "B": 100, "reshuffle_mod": mod,
                "reg": 0.05, "learning_rate": 0.01, "eval_mod": 25, "w_init": sw0,
                "test_X": stx, "test_Z": stz, "train_mon_pairs": smon, "train_X": sx,
                "train_Z": sz}
        captured = []
        cs.grad_inc_block = hook
        np.random.seed(3000 + mod)
        me.learning_process(sx, sz, p_sh)
        cs.grad_inc_block = orig
        put(f"shuttle_mod{mod}/ws", np.stack(captured))
        for k in ("iter", "norm_w", "bc_AUC", "br_AUC", "tr_AUC", "tc_AUC"):
            put(f"shuttle_mod{mod}/{k}", np.array(p_sh[k]))
        meta[f"shuttle_mod{mod}"] = {"seed": 3000 + mod, "n_it": 250, "N": 100, "B": 100,
                                     "reshuffle_mod": mod, "eval_mod": 25}

    np.savez_compressed(OUT / "golden.npz", **arrays)
    (OUT / "golden_meta.json").write_text(json.dumps(meta, indent=1, default=float))
    print(f"wrote {len(arrays)} arrays to {OUT / 'golden.npz'}")


if __name__ == "__main__":
    main()
