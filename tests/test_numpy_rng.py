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


def test_scalar_path_matches_numpy(tw):
    """The portable (non-AVX2) compaction, forced in a fresh process, against np.random."""
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
        "print('ok')\n")
    env = dict(os.environ, TW_NP_RNG_SCALAR="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr
