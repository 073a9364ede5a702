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
