"""Step chains (csrc/chain.hip, round 4): est.UnNT's repartition loop walked per element, the
(step, shard) image bags of a chunk of steps counted in one launch.  Checked against the oracle:
the bags hold exactly the images of the oracle's permutation chain shard by shard, the counts
equal the reference predicate on the oracle's permuted arrays (strict and half ties), the
simulated multi-rank exchange (send buckets, an all-to-all done by hand, unpack) gives the
one-process bags, and UnN_many through the chains equals the one-launch-per-step paths
(estimates and final arrays).  Bar: bit-exact (every value is an integer count)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
M64 = 2 ** 64 - 1


def _sample(rng, n, kind):
    if kind == "i64":
        return rng.randint(-40, 40, n).astype(np.int64)
    v = rng.normal(size=n).round(2)
    if kind == "edge" and n > 12:
        v[::7] = np.nan
        v[1::9] = 0.0
        v[2::11] = -0.0
        v[3::13] = np.inf
        v[4::17] = -np.inf
        v[5::19] = 5e-324
    return v


def _chain(a, keys, odd):
    """The oracle's permutation chain: the arrays after each repartition."""
    out = []
    for k in keys:
        a = O.permute_scatter(a, (2 * k + odd) & M64)
        out.append(a)
    return out


def _layout(n, m, N):
    from tuplewise.device import prop_swor_layout
    x_off, z_off, _ = prop_swor_layout(n, m, N)
    return x_off, z_off


@pytest.mark.parametrize("kind", ["gauss", "edge", "i64"])
@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("n,m,N", [(5000, 4099, 7), (20_000, 30_000, 1), (3000, 700, 64),
                                   (1, 1, 1), (4097, 2, 3)])
def test_chain_bags_and_counts_equal_oracle(gpu, kind, half, n, m, N):
    """tw_chain_emit (one process) + tw_count_pairs_chain: each (step, shard) bag is the
    multiset of the oracle's images at that shard's positions after the step's repartition; the
    counts equal the reference predicate (strict: #{x > z}; half: 2 #{x > z} + #{x == z}) on the
    oracle's permuted scores, and tw_count_pairs_chain_bucket's exact counts equal them; the
    chain state after the last step gives the final arrays."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(n + 3 * m + N)
    X, Z = _sample(rng, n, kind), _sample(rng, m, kind)
    code = L.TW_I64 if kind == "i64" else L.TW_F64
    ops = HipOps()
    Xd, Zd = torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda()
    xr, zr = ops.rank_images_query(Zd, Xd, Zd, code, half)
    wx, wz = O.rank_records(X, Z, half=half)
    assert np.array_equal(xr.cpu().numpy(), wx) and np.array_equal(zr.cpu().numpy(), wz)
    keys = [11, 12, 13, 14, 15]
    T = len(keys)
    kx, kz = int(n / N), int((n + m) / N) - int(n / N)
    x_off, z_off = _layout(n, m, N)
    x_bag = torch.empty((T, n), dtype=torch.int64 if half else torch.float32, device="cuda")
    z_bag = torch.empty((T, m), dtype=torch.float32, device="cuda")
    xpos = torch.empty(n, dtype=torch.int32, device="cuda")
    zpos = torch.empty(m, dtype=torch.int32, device="cuda")
    cur = torch.empty(T * 2 * (N + 1), dtype=torch.int32, device="cuda")
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    # two emissions (3 steps, then 2) through the chain state
    ops.chain_emit(xr, zr, half, xpos, zpos, True, 0, 1, kxs[:3], kzs[:3], kx, kz, N,
                   x_bag=x_bag, z_bag=z_bag, cursors=cur)
    ops.chain_emit(xr, zr, half, xpos, zpos, False, 0, 1, kxs[3:], kzs[3:], kx, kz, N,
                   x_bag=x_bag[3:], z_bag=z_bag[3:], cursors=cur)
    xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
    out = torch.full((T, N), 7, dtype=torch.int64, device="cuda")
    ops.count_chain(x_bag, xo, z_bag, zo, N, 3, n, m, kx, kz, half, out[:3])
    ops.count_chain(x_bag[3:], xo, z_bag[3:], zo, N, 2, n, m, kx, kz, half, out[3:])
    # the exact bucket count (algo="sorted") of the same bags: bags of <= 16384 z
    outb = torch.full((T, N), 7, dtype=torch.int64, device="cuda")
    if kz <= 16384:
        ops.count_chain_bucket(x_bag, xo, z_bag, zo, N, T, n, m, kz, m, half, outb)
        assert torch.equal(outb, out)
    xb = x_bag.cpu().numpy()
    zb = z_bag.cpu().numpy()
    got = out.cpu().numpy().view(np.uint64)
    xs, zs = _chain(X, keys, 0), _chain(Z, keys, 1)
    wxs, wzs = _chain(wx, keys, 0), _chain(wz, keys, 1)
    for c in range(T):
        wimg_x = wxs[c] if half else (wxs[c].view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        wimg_z = (wzs[c].view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        gx = xb[c].view(np.int64) if half else xb[c].view(np.uint32)
        gz = zb[c].view(np.uint32)
        for s in range(N):
            a, b = x_off[s], x_off[s + 1]
            assert np.array_equal(np.sort(gx[a:b]), np.sort(wimg_x[a:b]))
            a, b = z_off[s], z_off[s + 1]
            assert np.array_equal(np.sort(gz[a:b]), np.sort(wimg_z[a:b]))
            xa, za = xs[c][x_off[s]:x_off[s + 1]], zs[c][z_off[s]:z_off[s + 1]]
            if xa.dtype.kind == "f":
                xa = xa[~np.isnan(xa)]  # a NaN x is greater than / equal to nothing
            want = O.count_half_sorted(xa, za) if half else O.count_gt_sorted(xa, za)
            assert int(got[c, s]) == want, (c, s)
    Xo, Zo = ops.chain_scatter(Xd, xpos, Zd, zpos)
    assert np.array_equal(Xo.cpu().numpy(), xs[-1], equal_nan=kind != "i64")
    assert np.array_equal(Zo.cpu().numpy(), zs[-1], equal_nan=kind != "i64")


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("G", [2, 3])
def test_chain_exchange_simulated_ranks(gpu, G, half):
    """Several ranks in one process: each rank images its own elements against the whole Z
    (tw_rank_images_query), walks its chains into send buckets (tw_chain_emit, world = G), the
    all-to-all is done by hand (rank r receives every source's chunk for r), tw_chain_unpack
    fills its bags, tw_count_pairs_chain counts them; the ranks' counts equal one process on the
    global layout of G*N shards, and tw_chain_gather's final arrays equal the oracle chain."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(9 + G)
    n_loc, m_loc, N = 3000, 2100, 4
    X, Z = rng.normal(0.3, 1, G * n_loc).round(3), rng.normal(0, 1, G * m_loc).round(3)
    ops = HipOps()
    Zall = torch.from_numpy(Z).cuda()
    Xall = torch.from_numpy(X).cuda()
    keys = [21, 22, 23]
    T = len(keys)
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    kx, kz = int(n_loc / N), int((n_loc + m_loc) / N) - int(n_loc / N)
    tot = n_loc + m_loc
    cap = tot // G + tot // (8 * G) + 1024
    W = 2 if half else 1
    sends = []
    for r in range(G):
        xq = Xall[r * n_loc:(r + 1) * n_loc]
        zq = Zall[r * m_loc:(r + 1) * m_loc]
        xr, zr = ops.rank_images_query(Zall, xq, zq, L.TW_F64, half)
        wx, wz = O.rank_records(X[r * n_loc:(r + 1) * n_loc], Z[r * m_loc:(r + 1) * m_loc],
                                half=half, Z_all=Z)
        assert np.array_equal(xr.cpu().numpy(), wx) and np.array_equal(zr.cpu().numpy(), wz)
        xpos = torch.empty(n_loc, dtype=torch.int32, device="cuda")
        zpos = torch.empty(m_loc, dtype=torch.int32, device="cuda")
        send = torch.empty(G * T * (cap + 1) * W, dtype=torch.int64, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        ops.chain_emit(xr, zr, half, xpos, zpos, True, r, G, kxs, kzs, kx, kz, N, send=send,
                       cap=cap, flag=flag)
        assert int(flag.item()) == 0
        # tw_chain_walk: the same chain state without emitting
        wxp, wzp = torch.empty_like(xpos), torch.empty_like(zpos)
        ops.chain_walk(r * n_loc, n_loc, G * n_loc, r * m_loc, m_loc, G * m_loc, kxs, kzs, wxp,
                       wzp)
        assert torch.equal(wxp, xpos) and torch.equal(wzp, zpos)
        sends.append(send.view(G, -1))
    x_off, z_off = _layout(n_loc, m_loc, N)
    xo, zo = torch.from_numpy(x_off).cuda(), torch.from_numpy(z_off).cuda()
    counts = []
    for r in range(G):
        recv = torch.cat([sends[g][r] for g in range(G)])
        x_bag = torch.empty((T, n_loc), dtype=torch.int64 if half else torch.float32,
                            device="cuda")
        z_bag = torch.empty((T, m_loc), dtype=torch.float32, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        ops.chain_unpack(recv, G, T, cap, half, n_loc, m_loc, x_bag, z_bag, flag, kx, kz, N)
        assert int(flag.item()) == 0
        # (the bags hold their shards' multisets in no particular order: the counts check them)
        out = torch.empty((T, N), dtype=torch.int64, device="cuda")
        ops.count_chain(x_bag, xo, z_bag, zo, N, T, n_loc, m_loc, kx, kz, half, out)
        counts.append(out.cpu().numpy())
        assert int(flag.item()) == 0
        # tw_chain_unpack_count: the same receive side in one call (fresh bags, garbage out)
        xb2, zb2 = torch.empty_like(x_bag), torch.empty_like(z_bag)
        out2 = torch.full((T, N), 12345, dtype=torch.int64, device="cuda")
        ops.chain_unpack_count(recv, G, T, cap, half, n_loc, m_loc, xb2, zb2, flag, kx, kz, N,
                               xo, zo, kx, kz, out2)
        assert int(flag.item()) == 0 and np.array_equal(out2.cpu().numpy(), counts[-1])
        # each shard's region of the receiver's bags (and the tail past the last shard) holds
        # the oracle's permuted images of those positions, as a multiset (runs appended by
        # tw_chain_unpack in no particular order)
        wx, wz = O.rank_records(X, Z, half=half)
        wxs, wzs = _chain(wx, keys, 0), _chain(wz, keys, 1)

        def same_regions(got, want, off, n_all):
            edges = list(off) + ([n_all] if off[-1] < n_all else [])
            for a, b in zip(edges[:-1], edges[1:]):
                assert np.array_equal(np.sort(got[a:b]), np.sort(want[a:b]))
        for c in range(T):
            ex = wxs[c][r * n_loc:(r + 1) * n_loc]
            ez = wzs[c][r * m_loc:(r + 1) * m_loc]
            if half:
                same_regions(x_bag[c].cpu().numpy().view(np.uint64), ex.view(np.uint64), x_off,
                             n_loc)
            else:
                same_regions(x_bag[c].cpu().numpy().view(np.uint32),
                             (ex.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                             x_off, n_loc)
            same_regions(z_bag[c].cpu().numpy().view(np.uint32),
                         (ez.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32), z_off,
                         m_loc)
        Xo, Zo = ops.chain_gather(Xall, Zall, r * n_loc, n_loc, r * m_loc, m_loc, kxs, kzs)
        xs, zs = _chain(X, keys, 0), _chain(Z, keys, 1)
        assert np.array_equal(Xo.cpu().numpy(), xs[-1][r * n_loc:(r + 1) * n_loc])
        assert np.array_equal(Zo.cpu().numpy(), zs[-1][r * m_loc:(r + 1) * m_loc])
    got = np.concatenate(counts, axis=1).view(np.uint64)
    xs, zs = _chain(X, keys, 0), _chain(Z, keys, 1)
    for c in range(T):
        for g in range(G):
            for s in range(N):
                xa = xs[c][g * n_loc + x_off[s]:g * n_loc + x_off[s + 1]]
                za = zs[c][g * m_loc + z_off[s]:g * m_loc + z_off[s + 1]]
                want = (2 * O.un_count(xa, za) + int((xa[:, None] == za[None, :]).sum())
                        if half else O.un_count(xa, za))
                assert int(got[c, g * N + s]) == want


def test_chain_gather_many_steps(gpu):
    """tw_chain_gather over more than 32 steps (chunks walked back through its work array)."""
    import torch
    from tuplewise.device import HipOps
    rng = np.random.RandomState(4)
    G, n_loc, m_loc = 2, 1000, 700
    X, Z = rng.normal(size=G * n_loc), rng.normal(size=G * m_loc)
    keys = list(range(100, 170))
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    xs, zs = _chain(X, keys, 0)[-1], _chain(Z, keys, 1)[-1]
    ops = HipOps()
    for r in range(G):
        Xo, Zo = ops.chain_gather(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(),
                                  r * n_loc, n_loc, r * m_loc, m_loc, kxs, kzs)
        assert np.array_equal(Xo.cpu().numpy(), xs[r * n_loc:(r + 1) * n_loc])
        assert np.array_equal(Zo.cpu().numpy(), zs[r * m_loc:(r + 1) * m_loc])


def test_chain_walk_many_steps(gpu):
    """tw_chain_walk over more than 32 steps (launch chunks) and over none: the oracle's
    Feistel positions of the rank's elements."""
    import torch
    from tuplewise.device import HipOps
    G, n_loc, m_loc = 3, 1000, 700
    keys = list(range(300, 370))
    kxs = [(2 * k) & M64 for k in keys]
    kzs = [(2 * k + 1) & M64 for k in keys]
    ops = HipOps()
    for r in range(G):
        for T in (0, 1, 32, 33, 70):
            xp = torch.empty(n_loc, dtype=torch.int32, device="cuda")
            zp = torch.empty(m_loc, dtype=torch.int32, device="cuda")
            ops.chain_walk(r * n_loc, n_loc, G * n_loc, r * m_loc, m_loc, G * m_loc, kxs[:T],
                           kzs[:T], xp, zp)
            for got, base, nl, ks in ((xp, r * n_loc, n_loc, kxs), (zp, r * m_loc, m_loc, kzs)):
                p = np.arange(base, base + nl)
                for k in ks[:T]:
                    p = O.feistel_perm(p, G * nl, int(k))
                assert np.array_equal(got.cpu().numpy().view(np.uint32), p)


@pytest.mark.parametrize("case", ["gauss", "ties_i64", "edge_ragged", "one_shard", "long"])
@pytest.mark.parametrize("tie_mode", ["strict", "half"])
def test_unn_many_chain_equals_step_paths(gpu, case, tie_mode):
    """ShardedSample.UnN_many through the step chains == the one-launch-per-step paths (rank
    images for strict, the score compare for half ties): estimates and final arrays bit for
    bit; "long" crosses the 32-step chunk boundary."""
    import torch
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(5)
    keys = [3, 4, 5, 6]
    if case == "gauss":
        X, Z, N = rng.normal(0.3, 1, 300_000), rng.normal(0, 1, 250_000), 16
    elif case == "ties_i64":
        X, Z, N = rng.randint(0, 50, 160_003), rng.randint(0, 50, 120_000), 12
    elif case == "edge_ragged":
        X, Z, N = _sample(rng, 100_001, "edge"), _sample(rng, 77_777, "edge"), 7
    elif case == "one_shard":
        X, Z, N = rng.normal(0.5, 1, 20_000), rng.normal(0, 1, 30_000), 1
    else:
        X, Z, N = rng.normal(0.5, 1, 40_000).round(2), rng.normal(0, 1, 30_000).round(2), 5
        keys = list(range(40, 110))
    got = {}
    for chain in (True, False):
        old = D.CHAIN_STEPS
        D.CHAIN_STEPS = chain
        try:
            S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                              algo="pairs", tie_mode=tie_mode)
            assert S._chain_ok() == chain
            got[chain] = (S.UnN_many(keys), S.X.cpu().numpy(), S.Z.cpu().numpy())
        finally:
            D.CHAIN_STEPS = old
    assert got[True][0] == got[False][0]
    eqn = X.dtype.kind == "f"
    assert np.array_equal(got[True][1], got[False][1], equal_nan=eqn)
    assert np.array_equal(got[True][2], got[False][2], equal_nan=eqn)
    xa, za = _chain(X, keys, 0)[-1], _chain(Z, keys, 1)[-1]
    assert np.array_equal(got[True][1], xa, equal_nan=eqn)
    assert np.array_equal(got[True][2], za, equal_nan=eqn)


@pytest.mark.parametrize("case", ["gauss", "ties_i64", "edge_ragged", "one_shard", "long",
                                  "wide"])
@pytest.mark.parametrize("tie_mode", ["strict", "half"])
def test_unn_many_sorted_on_chains_equals_pairs(gpu, case, tie_mode):
    """algo="sorted" through the step chains with the exact bucket count of every bag
    (tw_count_pairs_chain_bucket; shards of <= 16384 z) == the all-pairs chain path: estimates
    and final arrays bit for bit, final arrays == the oracle's permutation chain; "wide" has
    shards past 16384 z and keeps the records path (same values again)."""
    import torch
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(8)
    keys = [3, 4, 5, 6]
    if case == "gauss":
        X, Z, N = rng.normal(0.3, 1, 300_000), rng.normal(0, 1, 250_000), 16
    elif case == "ties_i64":
        X, Z, N = rng.randint(0, 50, 160_003), rng.randint(0, 50, 120_000), 12
    elif case == "edge_ragged":
        X, Z, N = _sample(rng, 100_001, "edge"), _sample(rng, 77_777, "edge"), 7
    elif case == "one_shard":
        X, Z, N = rng.normal(0.5, 1, 20_000), rng.normal(0, 1, 16_000), 1
    elif case == "long":
        X, Z, N = rng.normal(0.5, 1, 40_000).round(2), rng.normal(0, 1, 30_000).round(2), 5
        keys = list(range(40, 110))
    else:
        X, Z, N = rng.normal(0.5, 1, 60_000), rng.normal(0, 1, 50_000), 2
    if tie_mode == "half" and case == "wide":
        pytest.skip("the records path takes the strict predicate only")
    got = {}
    for algo in ("sorted", "pairs"):
        S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N, algo=algo,
                          tie_mode=tie_mode)
        assert S._chain_ok()
        if algo == "sorted":
            assert (S.max_nz <= D.CHAIN_BUCKET_MAX) == (case != "wide")
        got[algo] = (S.UnN_many(keys), S.X.cpu().numpy(), S.Z.cpu().numpy())
    assert got["sorted"][0] == got["pairs"][0]
    eqn = X.dtype.kind == "f"
    assert np.array_equal(got["sorted"][1], got["pairs"][1], equal_nan=eqn)
    assert np.array_equal(got["sorted"][2], got["pairs"][2], equal_nan=eqn)
    xa, za = _chain(X, keys, 0)[-1], _chain(Z, keys, 1)[-1]
    assert np.array_equal(got["sorted"][1], xa, equal_nan=eqn)
    assert np.array_equal(got["sorted"][2], za, equal_nan=eqn)


def test_chain_overflow_flag(gpu):
    """A send bucket past its capacity sets the flag (records dropped, never written out of
    place) and the unpack flags a count past cap."""
    import torch
    from tuplewise import _lib as L
    from tuplewise.device import HipOps
    rng = np.random.RandomState(1)
    G, n, m = 2, 500, 400
    X, Z = rng.normal(size=G * n), rng.normal(size=G * m)
    ops = HipOps()
    Zall = torch.from_numpy(Z).cuda()
    xr, zr = ops.rank_images_query(Zall, torch.from_numpy(X[:n]).cuda(), Zall[:m], L.TW_F64)
    cap = 10
    send = torch.zeros(G * 1 * (cap + 1), dtype=torch.int64, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    xpos = torch.empty(n, dtype=torch.int32, device="cuda")
    zpos = torch.empty(m, dtype=torch.int32, device="cuda")
    ops.chain_emit(xr, zr, False, xpos, zpos, True, 0, G, [5], [6], 50, 40, 10, send=send,
                   cap=cap, flag=flag)
    assert int(flag.item()) == 1
    flag.zero_()
    x_bag = torch.zeros((1, n), dtype=torch.float32, device="cuda")
    z_bag = torch.zeros((1, m), dtype=torch.float32, device="cuda")
    ops.chain_unpack(send, G, 1, cap, False, n, m, x_bag, z_bag, flag, 50, 40, 10)
    assert int(flag.item()) == 1


@pytest.mark.parametrize("kind", ["gauss", "edge", "i64"])
@pytest.mark.parametrize("tie_mode", ["strict", "half"])
def test_local_counts_on_rank_images(gpu, kind, tie_mode, monkeypatch):
    """One-shot counts (ShardedSample.local_counts: est.Un / UnN) on compact rank images ==
    the double-compare kernel == the oracle, shard by shard (ragged shards, NaN/+-0/+-inf,
    int64 ties; strict and half units)."""
    import torch
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(77)
    X, Z, N = _sample(rng, 50_001, kind), _sample(rng, 33_333, kind), 7
    got = {}
    for on in (True, False):
        monkeypatch.setattr(D, "ONESHOT_RANK", on)
        monkeypatch.setattr(D, "ONESHOT_RANK_MIN_PAIRS", 0)
        S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), N,
                          algo="pairs", tie_mode=tie_mode)
        assert S._oneshot_rank_ok() == on
        got[on] = S.local_counts().cpu().numpy()
    assert np.array_equal(got[True], got[False])
    x_off, z_off = _layout(X.size, Z.size, N)
    for s in range(N):
        xa, za = X[x_off[s]:x_off[s + 1]], Z[z_off[s]:z_off[s + 1]]
        if xa.dtype.kind == "f":
            xa = xa[~np.isnan(xa)]
        want = O.count_half_sorted(xa, za) if tie_mode == "half" else O.count_gt_sorted(xa, za)
        assert int(got[True][s]) == want


@pytest.mark.parametrize("tie_mode", ["strict", "half"])
def test_c2_one_shard_on_rank_images(gpu, tie_mode):
    """BASELINE configs[1] (est.Un, n = 1e5/class, one shard: 1e10 pairs) through the rank-image
    one-shot count (taken by default at this size) == the oracle's sorted count."""
    import torch
    from tuplewise.device import ShardedSample
    rng = np.random.RandomState(8)
    X, Z = rng.normal(0.5, 1, 100_000).round(3), rng.normal(0, 1, 100_000).round(3)
    S = ShardedSample(torch.from_numpy(X).cuda(), torch.from_numpy(Z).cuda(), 1, algo="pairs",
                      tie_mode=tie_mode)
    assert S._oneshot_rank_ok()
    got = int(S.local_counts()[0])
    want = O.count_half_sorted(X, Z) if tie_mode == "half" else O.count_gt_sorted(X, Z)
    assert got == want


@pytest.mark.parametrize("tie_mode,algo", [("strict", "pairs"), ("half", "pairs"),
                                           ("strict", "sorted")])
def test_carried_images_equal_fresh_ranking(gpu, tie_mode, algo):
    """device.CARRY_IMAGES: consecutive UnN_many calls on one sample carry the records of the
    final arrays (tw_chain_scatter of the records by the chains' last positions) and skip the
    ranking; every call's estimates and final arrays equal the same calls with a fresh ranking
    each time.  An in-place change of X (its version counter) or an assignment drops them."""
    import torch
    from tuplewise import device as D
    from tuplewise.device import ShardedSample
    gen = torch.Generator(device="cuda").manual_seed(5)
    n = 70_000
    X = (torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.3).round(
        decimals=2)
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen).round(decimals=2)
    calls = [range(3, 7), range(10, 13), range(20, 40), range(50, 54)]

    def run(carry):
        D.CARRY_IMAGES = carry
        try:
            S = ShardedSample(X.clone(), Z.clone(), 16, tie_mode=tie_mode, algo=algo)
            out, seen = [], []
            for i, ks in enumerate(calls):
                if i == 3:
                    S.X.add_(0.0)  # in place: the carried images are dropped
                seen.append(S._carried(tie_mode == "half") is not None)
                out.append(([float(v) for v in S.UnN_many(ks)], S.X.cpu().numpy(),
                            S.Z.cpu().numpy()))
            return out, seen
        finally:
            D.CARRY_IMAGES = True
    got, seen = run(True)
    want, _ = run(False)
    assert seen == [False, True, True, False]
    for (gv, gx, gz), (wv, wx, wz) in zip(got, want):
        assert gv == wv
        assert np.array_equal(gx, wx) and np.array_equal(gz, wz)


@pytest.mark.parametrize("write", ["data_swap", "data_value", "dlpack"])
def test_carried_images_writes_behind_version_counter(gpu, write):
    """writes the version counter cannot see — through `S.X.data`, or a
    DLPack alias of S.Z — still look carried to _carried(), but the arrays' checksum
    (tw_words_checksum, csrc/guard.hip), verified in stream order, sends the call to a recount
    from a fresh ranking: its estimates and final arrays equal a fresh sample's on the written
    arrays, and the next call carries again."""
    import torch
    import torch.utils.dlpack as tdl
    from tuplewise.device import ShardedSample
    gen = torch.Generator(device="cuda").manual_seed(8)
    n, N = 50_000, 16
    X = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen) + 0.3
    Z = torch.randn(n, dtype=torch.float64, device="cuda", generator=gen)
    S = ShardedSample(X.clone(), Z.clone(), N, algo="pairs")
    S.UnN_many(range(3, 7))
    v0x, v0z = S.X._version, S.Z._version
    if write == "data_swap":
        S.X.data[[0, 1, 2]] = S.X.data[[2, 0, 1]].clone()
    elif write == "data_value":
        S.X.data[:1000] += 2.5
    else:
        alias = tdl.from_dlpack(tdl.to_dlpack(S.Z))
        alias[5000:9000] = -alias[5000:9000]
    assert S.X._version == v0x and S.Z._version == v0z  # nothing the counters saw
    assert S._carried(False) is not None
    Xw, Zw = S.X.clone(), S.Z.clone()
    got = [float(v) for v in S.UnN_many(range(10, 14))]
    assert getattr(S, "stale_recounts", 0) == 1
    F = ShardedSample(Xw, Zw, N, algo="pairs")
    want = [float(v) for v in F.UnN_many(range(10, 14))]
    assert got == want
    assert torch.equal(S.X, F.X) and torch.equal(S.Z, F.Z)
    assert S._carried(False) is not None  # carried again, and valid
    assert [float(v) for v in S.UnN_many(range(20, 23))] == [
        float(v) for v in F.UnN_many(range(20, 23))]
    assert S.stale_recounts == 1
