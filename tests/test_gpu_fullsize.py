"""The BASELINE configs at the sizes they name (VERDICT r01 'Next round' item 1).

C3 (configs[2]): n = 1e6 per class, N = 64 prop-SWOR shards, B = 1e6 pairs per shard, T = 4
repartitions — device-RNG draws (ShardedSample.UnNB_many) with every shard's ranked count equal
to the plain gather kernel's and a few shards per step equal to the oracle's draws exactly;
replay mode through the drop-in cs.UnNBT on host arrays, bit-identical to the oracle's restated
reference (same NumPy RNG stream, same in-place shuffles).
C5 (configs[4]): n = 1e7 rows (5e6 per class), d = 512, N = 256 shards, B = 100, device RNG,
both X layouts — every shard's gradient against the oracle's pair_grad (compute_stats.py:
157-162) on the drawn rows, the SWR row tables against the oracle's draws.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_c3_full_size_device_rng(gpu):
    import torch
    from tuplewise.device import ShardedSample
    n, N, B, T = 1_000_000, 64, 1_000_000, 4
    k = n // N
    rng = np.random.RandomState(33)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    seed0, keys = 0xC3C3_0001, [11, 12, 13, 14]
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo="pairs")
    ests = S.UnNB_many(B, seed0, keys)  # the pipelined call a user makes
    assert len(ests) == T
    S2 = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N)
    ops = S2.ops
    for t, key in enumerate(keys):
        S2.repartition(key)
        seed = seed0 + t
        ranked = S2._count_rng(B, seed)  # rank codes in LDS (tw_count_pairs_rng_ws)
        plain = ops.count_rng(S2.X, S2.x_off_dev, S2.Z, S2.z_off_dev, N, B, seed, 0,
                              S2.dtype, S2.pred)  # the gather kernel (tw_count_pairs_rng)
        assert torch.equal(ranked, plain), f"step {t}: ranked != plain"
        assert np.mean(S2.values(ranked, pairs=B)) == ests[t]
        Xp, Zp = S2.X.cpu().numpy(), S2.Z.cpu().numpy()
        c = ranked.cpu().numpy()
        for s in (t, 21 + t, 42 + t, 63 - t):
            i, j = O.rng_pairs(k, k, B, seed, s)
            want = int((Xp[s * k:(s + 1) * k][i] > Zp[s * k:(s + 1) * k][j]).sum())
            assert int(c[s]) == want, (t, s)


def test_c3_full_size_complete_one_launch_steps(gpu):
    """The bench's step at its size: UnN_many over T = 4 keys, n = 1e6 per class, N = 64, by
    the all-pairs count and by the exact count (algo="sorted": since round 4 the step chains'
    bags counted by tw_count_pairs_chain_bucket, shards of 15625 z) — same estimates; the
    arrays after the last step equal the oracle's chain of permutations; every shard's count
    of the last partition equals an exact searchsorted count."""
    import torch
    from tuplewise.device import ShardedSample
    n, N = 1_000_000, 64
    k = n // N
    rng = np.random.RandomState(35)
    X, Z = rng.normal(0.5, 1, n).round(3), rng.normal(0, 1, n).round(3)  # with ties
    keys = [101, 102, 103, 104]
    res = {}
    for algo in ("pairs", "sorted"):
        S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo=algo)
        res[algo] = (S.UnN_many(keys), S.X.cpu().numpy(), S.Z.cpu().numpy())
    assert res["pairs"][0] == res["sorted"][0]
    Xp, Zp = X, Z
    for key in keys:  # ShardedSample._repartition's key split
        Xp = O.permute_scatter(Xp, (2 * key) % 2 ** 64)
        Zp = O.permute_scatter(Zp, (2 * key + 1) % 2 ** 64)
    for algo in ("pairs", "sorted"):
        assert np.array_equal(res[algo][1], Xp) and np.array_equal(res[algo][2], Zp), algo
    vals = []
    for s in range(N):
        zs = np.sort(Zp[s * k:(s + 1) * k])
        vals.append(np.searchsorted(zs, Xp[s * k:(s + 1) * k], side="left").sum() / (k * k))
    assert res["pairs"][0][-1] == np.mean(np.array(vals, dtype=np.float64))


def test_c3_full_size_replay_drop_in(gpu):
    import tuplewise.compute_stats as cs
    n, N, B, T = 1_000_000, 64, 1_000_000, 2
    rng = np.random.RandomState(34)
    X, Z = rng.normal(0.5, 1, n), rng.normal(0, 1, n)
    Xo, Zo = X.copy(), Z.copy()
    np.random.seed(2024)
    got = cs.UnNBT(X, Z, N, B, T, "prop-SWOR", kernel="AUC")
    probe = np.random.randint(0, 2 ** 31)
    np.random.seed(2024)
    want = O.cs_UnNBT(Xo, Zo, N, B, T, "prop-SWOR", kernel="AUC")
    assert got == want
    assert np.array_equal(X, Xo) and np.array_equal(Z, Zo)  # the in-place shuffles
    assert np.random.randint(0, 2 ** 31) == probe  # the same RNG consumption


@pytest.mark.parametrize("layout", ["replicated", "partitioned"])
def test_c5_full_size_gradients(gpu, layout):
    import torch
    from tuplewise import _lib as L
    from tuplewise.learning import SGDEngine
    n, d, N, B = 5_000_000, 512, 256, 100
    g = torch.Generator(device="cuda").manual_seed(55)
    X = torch.randn((n, d), dtype=torch.float64, device="cuda", generator=g)
    Z = torch.randn((n, d), dtype=torch.float64, device="cuda", generator=g) + 0.3
    w0 = torch.randn((d, 1), dtype=torch.float64, device="cuda", generator=g) / d ** 0.5
    eng = SGDEngine(X, Z, w0, N, B, margin=1, reg=0.05, learning_rate=0.01,
                    optim_type="momentum", x_layout=layout)
    seed = 0xC5C5_C5C5
    eng.enable_device_rng(seed)
    eng.reshuffle_device()
    # one step's per-shard gradients (the launch step_device makes before its update)
    L.call("tw_pair_grad_rng", L.ptr(eng.X), L.ptr(eng.Z), eng.d, L.ptr(eng.rows_x), eng.kx,
           L.ptr(eng.rows_z), eng.kz, eng.N_loc, eng.B, L.ptr(eng.w), eng.margin, eng.loss,
           eng.seed, L.ptr(eng.step_ctr), eng.shard_base, L.ptr(eng.grads_loc),
           L.stream_handle())
    grads = eng.grads_loc.cpu().numpy()
    rx_t = eng.rows_all_x if layout == "partitioned" else eng.rows_x
    rz_t = eng.rows_all_z if layout == "partitioned" else eng.rows_z
    kx, kz = eng.kx, eng.kz
    rows_x, rows_z = rx_t.cpu().numpy(), rz_t.cpu().numpy()
    for s in (0, 101, 255):  # SWR_divide on the device == the oracle's draws
        assert np.array_equal(rows_x[s], O._mulhi64(
            O._sgd_draw(seed, 0, np.arange(kx), s, 0x40000000)[0], n))
        assert np.array_equal(rows_z[s], O._mulhi64(
            O._sgd_draw(seed, 0, np.arange(kz), s, 0x20000000)[0], n))
    rx, rz = np.empty((N, B), np.int64), np.empty((N, B), np.int64)
    for s in range(N):
        u, v = O._sgd_draw(seed, 0, np.arange(B), s, 0x80000000)
        rx[s] = rows_x[s][O._mulhi64(u, kx)]
        rz[s] = rows_z[s][O._mulhi64(v, kz)]
    Xr = X[torch.from_numpy(rx.reshape(-1)).cuda()].cpu().numpy().reshape(N, B, d)
    Zr = Z[torch.from_numpy(rz.reshape(-1)).cuda()].cpu().numpy().reshape(N, B, d)
    w = w0.cpu().numpy()
    flips = 0
    for s in range(N):
        diff = Zr[s] - Xr[s]
        want = O.pair_grad(diff, w, 1.0, B).ravel()
        if not np.allclose(grads[s], want, rtol=1e-10, atol=1e-13):
            S_b = diff.dot(w).ravel() + 1.0
            assert np.min(np.abs(S_b)) < 1e-9, f"shard {s}: gradient differs, no |S| near 0"
            flips += 1  # a hinge filter decided by the last bit of a dot product
    assert flips == 0, f"{flips} shards differ only by hinge-filter sign flips"
