"""The all-pairs count on packed-f32 rank images (csrc/rankimage.hip, round 3) against the
oracle: the images themselves (oracle.rank_records, bit for bit), the one-launch step's counts
against the score-compare kernel and the reference's predicate, its next repartition against
the oracle's permutation, and UnN_many through both paths (estimates and final arrays equal).
Bar: bit-exact (every value is an integer count)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _edge_sample(rng, n, kind):
    if kind == "i64":
        return rng.randint(-40, 40, n).astype(np.int64)
    v = rng.normal(size=n).round(2)
    if kind == "edge" and n > 12:
        v[::7] = np.nan
        v[1::9] = 0.0
        v[2::11] = -0.0
        v[3::13] = np.inf
        v[4::17] = -np.inf
        v[5::19] = 5e-324  # subnormal
        v[6::23] = -5e-324
    return v


@pytest.mark.parametrize("kind", ["gauss", "edge", "i64"])
@pytest.mark.parametrize("n,m", [(1, 1), (0, 5), (7, 0), (300, 257), (5000, 4099),
                                 (200_001, 150_000)])
def test_rank_images_equal_oracle(gpu, kind, n, m):
    """tw_rank_images == oracle.rank_records bit for bit, and every pair satisfies
    x > z  <=>  x_image + z_image >= 1 (NaN, +-0, +-inf, subnormals, ties, int64)."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(n * 7 + m)
    X, Z = _edge_sample(rng, n, kind), _edge_sample(rng, m, kind)
    code = L.TW_I64 if kind == "i64" else L.TW_F64
    xr, zr = HipOps().rank_images(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), code)
    wx, wz = O.rank_records(X, Z)
    assert np.array_equal(xr.cpu().numpy(), wx) and np.array_equal(zr.cpu().numpy(), wz)
    if n and m and n * m <= 5000 * 5000:  # the pair property itself, on all pairs
        gx = (wx.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32)
        nz = (wz.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32)
        with np.errstate(invalid="ignore"):
            assert np.array_equal(gx[:, None] + nz[None, :] >= 1, X[:, None] > Z[None, :])


def test_rank_images_bucket_paths(gpu):
    """The bucketed ranking against the oracle on the layouts that exercise its paths: heavy
    ties (every sampled splitter one of a few values: equality buckets), a sample that sees only
    one value (every other z in the top interval bucket), heavy tails with subnormals (the
    order-key sub-bucket map), and full-range int64 keys."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    ops = HipOps()
    rng = np.random.RandomState(17)
    # heavy ties: 3 values make 95 % of both samples, the rest continuous
    X = np.where(rng.rand(300_000) < 0.95, rng.choice([-1.0, 0.0, 2.5], 300_000),
                 rng.normal(size=300_000))
    Z = np.where(rng.rand(250_000) < 0.95, rng.choice([-1.0, -0.0, 2.5], 250_000),
                 rng.normal(size=250_000))
    # the adversarial layout: Z's sampled positions (i * m // cs) all hold 0.0, every other z a
    # distinct value in (0, 1)
    m, cs = 40_000, 8192
    Za = rng.uniform(1e-6, 1.0, m)
    Za[(np.arange(cs) * m) // cs] = 0.0
    Xa = rng.uniform(-0.5, 1.5, 30_000)
    # heavy tails (the order-key sub-bucket map) and a sample straddling 0 with subnormals
    Xc_, Zc_ = rng.standard_cauchy(200_000), rng.standard_cauchy(180_000)
    Zc_[::1000] = 5e-324
    Xi, Zi = rng.randint(-2 ** 62, 2 ** 62, 100_000), rng.randint(-2 ** 62, 2 ** 62, 90_000)
    for Xc, Zc in ((X, Z), (Xa, Za), (Xc_, Zc_), (Xi, Zi)):
        code = L.TW_I64 if Xc.dtype == np.int64 else L.TW_F64
        xr, zr = ops.rank_images(torch.from_numpy(Xc).cuda(), torch.from_numpy(Zc).cuda(), code)
        wx, wz = O.rank_records(Xc, Zc)
        assert np.array_equal(xr.cpu().numpy(), wx) and np.array_equal(zr.cpu().numpy(), wz)


@pytest.mark.parametrize("m", [100_000, 1_000_000])
def test_rank_images_sorted_and_periodic_z(gpu, m):
    """Z in sorted order and with index-periodic structure (the layouts an
    index-strided splitter sample handled worst) — the hashed sample keeps the interval buckets
    balanced — and Z with heavy ties: images equal the oracle's and one ranking stays within a
    few times its Gaussian cost (sub-bucket scans bounded, long sub-buckets sorted by waves),
    small-Z plan (m = 1e5) and large (1e6)."""
    import time
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    ops = HipOps()
    rng = np.random.RandomState(23)
    X = rng.normal(size=m // 2)
    cases = {"gauss": rng.normal(size=m), "sorted": np.sort(rng.normal(size=m)),
             "periodic": np.tile(np.sort(rng.normal(size=1000)), m // 1000),
             "sawtooth": (np.arange(m) % 4096) * 1e-3,
             # heavy ties: ~m / 5000 and ~m / 1000 copies of each value (long sub-buckets,
             # sorted by one wave each; before, ~20 sequential block sorts per bucket: 1.9 ms)
             "ties5000": rng.randint(0, 5000, size=m).astype(np.float64),
             "ties1000": rng.randint(0, 1000, size=m).astype(np.float64)}
    times = {}
    for name, Z in cases.items():
        Xd, Zd = torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda()
        ops.rank_images(Xd, Zd, L.TW_F64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            xr, zr = ops.rank_images(Xd, Zd, L.TW_F64)
        torch.cuda.synchronize()
        times[name] = (time.perf_counter() - t0) / 5
        wx, wz = O.rank_records(X, Z)
        assert np.array_equal(xr.cpu().numpy(), wx) and np.array_equal(zr.cpu().numpy(), wz), name
    for name, t in times.items():
        assert t < 5 * times["gauss"] + 2e-3, (name, times)


@pytest.mark.parametrize("kind", ["gauss", "edge", "i64"])
@pytest.mark.parametrize("plan", [(0, 0), (8, 0), (16, 0), (8, 8), (16, 24), (8, 1000)])
def test_count_rank_step_fused_repartition(gpu, kind, plan):
    """tw_count_pairs_rank_step on ragged and empty shards: counts == tw_count_pairs (strict)
    == the reference predicate, for every plan (R = 8/16, z chunks 8 / 24 / 1000 / automatic:
    full 16-record groups, 8-groups and single-record tails); the same launch writes the next
    repartition of both record arrays (== the oracle's permutation) and zeroes the next
    counters."""
    import torch
    from tuplewise import _engine as E, _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(31)
    nx = [0, 1, 5, 257, 3000, 1, 4096 + 3, 700, 2048]
    nz = [3, 0, 9, 1000, 2049, 1, 513, 700, 17]
    xs = [_edge_sample(rng, k, kind) for k in nx]
    zs = [_edge_sample(rng, k, kind) for k in nz]
    code = L.TW_I64 if kind == "i64" else L.TW_F64
    sh = E.Shards.from_blocks(xs, zs, code)
    want = np.array([O.un_count(a, b) for a, b in zip(xs, zs)], dtype=np.uint64)
    assert np.array_equal(E.count_complete(sh, "gt", algo="pairs"), want)
    ops = HipOps()
    xr, zr = ops.rank_images(sh.x, sh.z, code)
    xo, zo = sh.offsets_dev()
    out = torch.zeros(len(nx), dtype=torch.int64, device="cuda")
    out_next = torch.full((5,), 77, dtype=torch.int64, device="cuda")
    xn, zn = torch.empty_like(xr), torch.empty_like(zr)
    L.call("tw_count_rank_set_plan", plan[0], plan[1])
    try:
        ops.count_rank_step(xr, xo, zr, zo, len(nx), max(nx), max(nz), out, xn, 11, zn, 12,
                            out_next)
    finally:
        L.call("tw_count_rank_set_plan", 0, 0)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    assert not out_next.cpu().numpy().any()
    assert np.array_equal(xn.cpu().numpy(), O.permute_scatter(xr.cpu().numpy(), 11))
    assert np.array_equal(zn.cpu().numpy(), O.permute_scatter(zr.cpu().numpy(), 12))
    # the scores back in record order
    xs_back = ops.gather_records(sh.x, xn).cpu().numpy()
    assert np.array_equal(xs_back, O.permute_scatter(sh.x.cpu().numpy(), 11),
                          equal_nan=kind != "i64")


@pytest.mark.parametrize("case", ["gauss", "ties_i64", "edge_ragged", "one_shard"])
def test_unn_many_rank_path_equals_score_path(gpu, case):
    """ShardedSample.UnN_many on rank images == the double-compare kernel's steps (estimates,
    final arrays bit for bit, per-step counts), and the last estimate == the oracle's count on
    the oracle's chain of permutations."""
    import torch
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(5)
    if case == "gauss":
        X, Z, N = rng.normal(0.3, 1, 300_000), rng.normal(0, 1, 250_000), 16
    elif case == "ties_i64":
        X, Z, N = rng.randint(0, 50, 160_003), rng.randint(0, 50, 120_000), 12
    elif case == "edge_ragged":
        X, Z, N = _edge_sample(rng, 100_001, "edge"), _edge_sample(rng, 77_777, "edge"), 7
    else:
        X, Z, N = rng.normal(0.5, 1, 20_000), rng.normal(0, 1, 30_000), 1
    keys = [3, 4, 5, 6]
    got = {}
    for rank in (True, False):
        old = D.RANK_IMAGES
        D.RANK_IMAGES = rank
        try:
            S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                              algo="pairs")
            assert S._rank_path_ok() == rank
            est = S.UnN_many(keys)
            got[rank] = (est, S.X.cpu().numpy(), S.Z.cpu().numpy())
        finally:
            D.RANK_IMAGES = old
    assert got[True][0] == got[False][0]
    assert np.array_equal(got[True][1], got[False][1], equal_nan=X.dtype.kind == "f")
    assert np.array_equal(got[True][2], got[False][2], equal_nan=X.dtype.kind == "f")
    # the chain of repartitions and the last step's counts from the oracle
    xa, za = X, Z
    for k in keys:
        xa = O.permute_scatter(xa, (2 * k) & (2 ** 64 - 1))
        za = O.permute_scatter(za, (2 * k + 1) & (2 ** 64 - 1))
    assert np.array_equal(got[True][1], xa, equal_nan=X.dtype.kind == "f")
    x_off, z_off, keep = D.prop_swor_layout(X.size, Z.size, N)
    # the 300k x 250k Gaussian case through the oracle's O(n log m) count (continuous scores, no
    # NaN: #{z < x} by searchsorted is the reference's integer), the others pair by pair
    count = O.count_gt_sorted if case == "gauss" else O.un_count
    vals = [count(xa[x_off[s]:x_off[s + 1]], za[z_off[s]:z_off[s + 1]])
            / ((x_off[s + 1] - x_off[s]) * (z_off[s + 1] - z_off[s])) for s in range(N)
            if keep[s]]
    assert got[True][0][-1] == np.mean(vals)
