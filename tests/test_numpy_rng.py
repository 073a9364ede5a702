"""tw_np_randint_batch (csrc/numpy_rng.cpp) against np.random itself — no GPU needed."""
import numpy as np
import pytest


@pytest.mark.parametrize("ranges", [
    [(0, 91, 100), (0, 7, 100)] * 50,               # grad_inc_block at C4 (kx=91, kz=7)
    [(0, 9117, 91)] * 100 + [(0, 702, 7)] * 100,    # SWR_divide at C4
    [(0, 1, 5), (3, 4, 2), (0, 2 ** 32, 7), (0, 2 ** 32 - 1, 9), (-5, 2 ** 40, 11),
     (0, 2 ** 62, 13), (-(2 ** 63), 2 ** 63 - 1, 4), (10, 11, 0)],
])
def test_randint_batch_matches_numpy(tw, ranges):
    from tuplewise.numpy_rng import randint_batch
    np.random.seed(1234)
    want = [np.random.randint(lo, hi, n) for lo, hi, n in ranges]
    probe_want = np.random.random()
    np.random.seed(1234)
    got = randint_batch(ranges)
    probe_got = np.random.random()
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.dtype == np.int64 and np.array_equal(g, w)
    assert probe_got == probe_want


def test_randint_batch_empty_range_raises_like_numpy(tw):
    from tuplewise.numpy_rng import randint_batch
    np.random.seed(5)
    with pytest.raises(ValueError):
        randint_batch([(0, 10, 3), (4, 4, 1)])
    after = np.random.random()
    np.random.seed(5)
    np.random.randint(0, 10, 3)
    with pytest.raises(ValueError):
        np.random.randint(4, 4, 1)
    assert np.random.random() == after


@pytest.mark.parametrize("N,kx,kz,B", [(100, 91, 7, 100), (3, 1, 5, 17), (2, 2 ** 33, 3, 4)])
def test_session_pairs_match_grad_inc_block_draws(tw, N, kx, kz, B):
    """Session.pairs == the per-shard randint(0,kx,B), randint(0,kz,B) calls of
    grad_inc_block (compute_stats.py:155-156), and the state written back matches."""
    from tuplewise.numpy_rng import Session
    np.random.seed(99)
    np.random.random(5)  # start mid-block
    want_x, want_z = [], []
    for _ in range(N):
        want_x.append(np.random.randint(0, kx, B))
        want_z.append(np.random.randint(0, kz, B))
    probe_want = np.random.random()
    np.random.seed(99)
    np.random.random(5)
    ix = np.empty((N, B), np.int64)
    iz = np.empty((N, B), np.int64)
    with Session() as s:
        s.pairs(N, kx, kz, B, ix, iz)
    assert np.array_equal(ix, np.stack(want_x)) and np.array_equal(iz, np.stack(want_z))
    assert np.random.random() == probe_want


def test_session_flat_draws_commit_and_reacquire(tw):
    from tuplewise.numpy_rng import Session
    np.random.seed(7)
    a = np.random.randint(0, 9117, 91 * 3)
    mid = np.random.normal()  # foreign draw between session phases (touches has_gauss)
    b = np.random.randint(-3, 702, 50)
    end = np.random.random()
    np.random.seed(7)
    s = Session()
    ga = s.randint_flat([0, 0, 0], [9117] * 3, [91] * 3)
    s.commit()
    gmid = np.random.normal()
    s.acquire()
    gb = s.randint_flat([-3], [702], [50])
    s.commit()
    assert np.array_equal(ga, a) and gmid == mid and np.array_equal(gb, b)
    assert np.random.random() == end


@pytest.mark.parametrize("env", [{"TW_NP_RNG_SCALAR": "1"}, {"TW_NP_RNG_ISA": "avx2"}])
def test_scalar_path_matches_numpy(tw, env):
    """The portable compaction and the AVX2 path (the in-process tests run the widest level the
    CPU has, AVX-512 where present), each forced in a fresh process, against np.random —
    randint pairs and the in-place shuffles."""
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, tuplewise\n"
        "from tuplewise.numpy_rng import Session, randint_batch\n"
        "np.random.seed(3); w=[np.random.randint(0,k,100) for _ in range(40) for k in (91,7)]\n"
        "np.random.seed(3); ix=np.empty((40,100),np.int64); iz=np.empty((40,100),np.int64)\n"
        "s=Session(); s.pairs(40,91,7,100,ix,iz); s.commit()\n"
        "assert np.array_equal(ix, np.stack(w[0::2])) and np.array_equal(iz, np.stack(w[1::2]))\n"
        "np.random.seed(3); o8=np.empty((4,2,10,100),np.uint8); o16=np.empty((4,2,10,100),np.uint16)\n"
        "s=Session(); s.pairs_steps_u8(4,10,91,7,100,o8); s.commit()\n"
        "np.random.seed(3); s=Session(); s.pairs_steps_u16(4,10,91,7,100,o16); s.commit()\n"
        "assert np.array_equal(o8[:, 0].reshape(40, 100), ix) and np.array_equal(o16, o8)\n"
        "from tuplewise.numpy_rng import shuffle_pair\n"
        "X=np.arange(70001.0); Z=np.arange(3000.0); X1=X.copy(); Z1=Z.copy()\n"
        "np.random.seed(8); np.random.shuffle(X1); np.random.shuffle(Z1); p=np.random.rand()\n"
        "np.random.seed(8); shuffle_pair(X, Z)\n"
        "assert np.array_equal(X, X1) and np.array_equal(Z, Z1) and np.random.rand() == p\n"
        "from tuplewise.numpy_rng import shuffle_draws32\n"
        "np.random.seed(8); jx=shuffle_draws32(70001); jz=shuffle_draws32(3000)\n"
        "assert np.random.rand() == p\n"
        "X=np.arange(70001.0); Z=np.arange(3000.0)\n"
        "for a, j in ((X, jx), (Z, jz)):\n"
        "    for i in range(len(a) - 1, 0, -1): a[i], a[j[i]] = a[j[i]], a[i]\n"
        "assert np.array_equal(X, X1) and np.array_equal(Z, Z1)\n"
        "print('ok')\n")
    env = dict(os.environ, **env)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


@pytest.mark.parametrize("nx,nz,shape,dtype", [
    (1000, 700, None, np.float64), (1, 5, None, np.float64), (0, 3, None, np.float64),
    (17, 1, None, np.int64), (300000, 200000, None, np.float64), (1000, 50, "col", np.float64),
    (999, 88, "rows", np.float64), (5000, 3000, None, np.float32), (4097, 4095, None, np.int8),
    (2 ** 20 + 5, 1025, None, np.float64)])
def test_shuffle_pair_matches_numpy(tw, nx, nz, shape, dtype):
    """numpy_rng.shuffle_pair == np.random.shuffle(X); np.random.shuffle(Z): arrays (1-D, (n, 1),
    rows of a 2-D array), every dtype width, and the RNG state after (a probe draw)."""
    from tuplewise.numpy_rng import shuffle_pair
    rs = np.random.RandomState(nx)
    X = rs.normal(size=nx).astype(dtype)
    Z = rs.normal(size=nz).astype(dtype)
    if shape == "col":
        X, Z = X.reshape(-1, 1), Z.reshape(-1, 1)
    elif shape == "rows":
        X, Z = np.repeat(X[:, None], 3, 1).copy(), np.repeat(Z[:, None], 3, 1).copy()
    for seed in (1, 123):
        X1, Z1, X2, Z2 = X.copy(), Z.copy(), X.copy(), Z.copy()
        np.random.seed(seed)
        np.random.randint(0, 5, 3)
        np.random.shuffle(X1)
        np.random.shuffle(Z1)
        want = np.random.randint(0, 2 ** 31, 4)
        np.random.seed(seed)
        np.random.randint(0, 5, 3)
        shuffle_pair(X2, Z2)
        assert np.array_equal(X2, X1) and np.array_equal(Z2, Z1)
        assert np.array_equal(np.random.randint(0, 2 ** 31, 4), want)


def test_shuffle_pair_views_fall_back_to_numpy(tw):
    """A strided view is shuffled by np.random.shuffle itself (the buffer path is restated only
    for contiguous arrays): same result either way."""
    from tuplewise.numpy_rng import shuffle_pair
    base = np.arange(2000.0)
    X, Z = base[::2], np.arange(300.0)
    Xr, Zr = X.copy(), Z.copy()
    np.random.seed(4)
    np.random.shuffle(Xr)
    np.random.shuffle(Zr)
    np.random.seed(4)
    shuffle_pair(X, Z)
    assert np.array_equal(X, Xr) and np.array_equal(Z, Zr)


@pytest.mark.parametrize("alias", ["same", "overlap"])
def test_shuffle_pair_aliased_samples(tw, alias):
    """X and Z sharing memory (the same array, or overlapping contiguous views): the second
    shuffle sees the first one's swaps, exactly as two np.random.shuffle calls in turn — the
    concurrent native path is not taken."""
    from tuplewise.numpy_rng import shuffle_pair
    for n in (1000, 70_000):  # below and above the two-thread size
        base = np.random.RandomState(n).normal(size=2 * n)
        ref = base.copy()
        if alias == "same":
            X, Z, Xr, Zr = base, base, ref, ref
        else:
            X, Z, Xr, Zr = base[:n + n // 2], base[n // 2:], ref[:n + n // 2], ref[n // 2:]
        np.random.seed(8)
        np.random.shuffle(Xr)
        np.random.shuffle(Zr)
        want = np.random.randint(0, 2 ** 31, 4)
        np.random.seed(8)
        shuffle_pair(X, Z)
        assert np.array_equal(base, ref)
        assert np.array_equal(np.random.randint(0, 2 ** 31, 4), want)


def _apply_swaps(a, j):
    """_shuffle_raw's swaps (i = n-1 down to 1: swap a[i], a[j[i]]) in plain Python."""
    for i in range(len(a) - 1, 0, -1):
        k = j[i]
        a[i], a[k] = a[k], a[i]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 17, 1000, 65537, 200003])
def test_shuffle_draws32_are_numpy_shuffle_draws(tw, n):
    """numpy_rng.shuffle_draws32 (the host half of the device shuffle): the draws of
    np.random.shuffle on n items — applying them in _shuffle_raw's order gives NumPy's
    permutation, every j[i] <= i, and the RNG state after is the shuffle's."""
    from tuplewise.numpy_rng import shuffle_draws32
    for seed in (4, 77):
        a = np.arange(n, dtype=np.int64)
        np.random.seed(seed)
        np.random.random(3)
        np.random.shuffle(a)
        probe = np.random.randint(0, 2 ** 31, 3)
        np.random.seed(seed)
        np.random.random(3)
        j = shuffle_draws32(n)
        assert np.array_equal(np.random.randint(0, 2 ** 31, 3), probe)
        assert j.dtype == np.uint32 and len(j) == n
        if n > 1:
            assert np.all(j[1:].astype(np.int64) <= np.arange(1, n))
        b = list(range(n))
        _apply_swaps(b, j.tolist())
        assert np.array_equal(np.array(b, dtype=np.int64), a)


@pytest.mark.parametrize("n", [2, 3, 17, 1000, 65537, 200003])
@pytest.mark.parametrize("cuts", [1, 2, 4, 16, 37])
def test_shuffle_draws32_range_pieces_equal_whole(tw, n, cuts):
    """numpy_rng.shuffle_draws32_range in consecutive ranges (hi = n - 1 down to lo = 1, the
    streamed last shuffle of the drop-in) == one shuffle_draws32(n): the same draws and the
    same RNG state after (cuts 37: ranges that split the mask ranges and SIMD batches)."""
    from tuplewise.numpy_rng import shuffle_draws32, shuffle_draws32_range
    np.random.seed(5)
    np.random.random(7)
    want = shuffle_draws32(n)
    probe = np.random.randint(0, 2 ** 31, 3)
    np.random.seed(5)
    np.random.random(7)
    got = np.zeros(n, dtype=np.uint32)
    edges = sorted({int(e) for e in np.linspace(n - 1, 0, cuts + 1)})[::-1]
    for hi, lo in zip(edges[:-1], edges[1:]):
        hi_i = hi if hi == n - 1 else hi - 1
        if hi_i >= max(lo, 1):
            shuffle_draws32_range(n, hi_i, max(lo, 1), got)
    assert np.array_equal(np.random.randint(0, 2 ** 31, 3), probe)
    assert np.array_equal(got[1:], want[1:])


@pytest.mark.parametrize("in_place", [True, False])
def test_state_in_place_and_copied_paths(tw, in_place, monkeypatch):
    """The native draws advance NumPy's own MT19937 struct in place (numpy_rng._mt_state) or,
    where that is unavailable, a get_state copy committed with set_state: both give NumPy's
    draws and final state, incl. a foreign draw between two Session phases."""
    from tuplewise import numpy_rng as R
    if not in_place:
        monkeypatch.setattr(R, "_mt_state", lambda: None)
    np.random.seed(21)
    a = np.random.randint(0, 97, 50)
    X, W = np.arange(5000.0), np.arange(300.0)
    np.random.shuffle(X)
    np.random.shuffle(W)
    g = np.random.normal()
    b = np.random.randint(-4, 9, 30)
    j = np.arange(700)
    np.random.shuffle(j)
    end = np.random.random()
    np.random.seed(21)
    got_a = R.randint_batch([(0, 97, 50)])[0]
    Y, V = np.arange(5000.0), np.arange(300.0)
    R.shuffle_pair(Y, V)
    s = R.Session()
    gg = np.random.normal()  # foreign draw (touches has_gauss)
    s.acquire()
    got_b = s.randint_flat([-4], [9], [30])
    s.commit()
    jj = R.shuffle_draws32(700)
    k = np.arange(700)
    for i in range(699, 0, -1):
        k[i], k[jj[i]] = k[jj[i]], k[i]
    assert np.array_equal(got_a, a) and np.array_equal(Y, X) and np.array_equal(V, W)
    assert gg == g
    assert np.array_equal(got_b, b) and np.array_equal(k, j)
    assert np.random.random() == end


def test_session_pairs_steps_match_per_step_draws(tw):
    """Session.pairs_steps (one native call for S steps, tw_np_randint_pairs_steps) == S
    steps of grad_inc_block's per-shard randint(0,kx,B), randint(0,kz,B) calls."""
    from tuplewise.numpy_rng import Session
    S, N, kx, kz, B = 7, 5, 91, 7, 33
    np.random.seed(17)
    want = np.empty((S, 2, N, B), np.int64)
    for st in range(S):
        for s in range(N):
            want[st, 0, s] = np.random.randint(0, kx, B)
            want[st, 1, s] = np.random.randint(0, kz, B)
    probe = np.random.random()
    np.random.seed(17)
    out = np.empty((S + 2, 2, N, B), np.int64)
    with Session() as sess:
        sess.pairs_steps(S, N, kx, kz, B, out)
    assert np.array_equal(out[:S], want) and np.random.random() == probe


@pytest.mark.parametrize("kx,kz", [(91, 7), (65536, 3), (40000, 65535)])
def test_session_pairs_steps_u16_match_int64(tw, kx, kz):
    """Session.pairs_steps_u16 (the replay loop's narrowed draws, tw_np_randint_pairs_steps_u16)
    == the int64 draws of pairs_steps, value for value, and leaves the same RNG state; ranges
    beyond 65536 are refused."""
    from tuplewise.numpy_rng import Session
    S, N, B = 5, 4, 37
    np.random.seed(23)
    want = np.empty((S, 2, N, B), np.int64)
    with Session() as sess:
        sess.pairs_steps(S, N, kx, kz, B, want)
    probe = np.random.random()
    np.random.seed(23)
    got = np.empty((S, 2, N, B), np.uint16)
    with Session() as sess:
        sess.pairs_steps_u16(S, N, kx, kz, B, got)
    assert np.array_equal(got.astype(np.int64), want) and np.random.random() == probe
    with Session() as sess, pytest.raises(ValueError):
        sess.pairs_steps_u16(1, N, 65537, kz, B, got)


@pytest.mark.parametrize("kx,kz", [(91, 7), (256, 1), (2, 256), (200, 129)])
def test_session_pairs_steps_u8_match_int64(tw, kx, kz):
    """Session.pairs_steps_u8 (the replay loop's uint8 draws, tw_np_randint_pairs_steps_u8, the
    C4 shape's default) == the int64 draws of pairs_steps, value for value, and leaves the same
    RNG state; ranges beyond 256 are refused."""
    from tuplewise.numpy_rng import Session
    S, N, B = 5, 4, 37
    np.random.seed(29)
    want = np.empty((S, 2, N, B), np.int64)
    with Session() as sess:
        sess.pairs_steps(S, N, kx, kz, B, want)
    probe = np.random.random()
    np.random.seed(29)
    got = np.empty((S, 2, N, B), np.uint8)
    with Session() as sess:
        sess.pairs_steps_u8(S, N, kx, kz, B, got)
    assert np.array_equal(got.astype(np.int64), want) and np.random.random() == probe
    with Session() as sess, pytest.raises(ValueError):
        sess.pairs_steps_u8(1, N, 257, kz, B, got)


@pytest.mark.parametrize("highs", [[9117] * 5 + [702] * 5, [65536, 1, 2, 40000], [3]])
def test_randint_batch_u16_matches_numpy(tw, highs):
    """tw_np_randint_batch_u16 (SWR_divide's rows narrowed for the replay loop's uint16 row
    tables; 64-word AVX-512 VBMI2 compaction where the host has it, else the int64 path
    narrowed) == np.random.randint call for call, leaving the same RNG state; calls beyond
    [0, 65536) are refused with the state untouched."""
    from tuplewise import _lib as L
    from tuplewise.numpy_rng import Session
    cnt = np.array([37 + 11 * i for i in range(len(highs))], np.int64)
    low = np.zeros(len(highs), np.int64)
    high = np.array(highs, np.int64)
    np.random.seed(31)
    want = np.concatenate([np.random.randint(0, h, c) for h, c in zip(highs, cnt)])
    probe = np.random.random()
    np.random.seed(31)
    got = np.empty(int(cnt.sum()), np.uint16)
    with Session() as s:
        assert L.lib().tw_np_randint_batch_u16(s._key, s._pos, len(highs), low.ctypes.data,
                                               high.ctypes.data, cnt.ctypes.data,
                                               got.ctypes.data) == 0
    assert np.array_equal(got.astype(np.int64), want) and np.random.random() == probe
    bad = np.array([65537], np.int64)
    np.random.seed(31)
    with Session() as s:
        assert L.lib().tw_np_randint_batch_u16(s._key, s._pos, 1, low.ctypes.data,
                                               bad.ctypes.data, cnt.ctypes.data,
                                               got.ctypes.data) == 1
    assert np.random.randint(0, highs[0], int(cnt[0]))[0] == want[0]
