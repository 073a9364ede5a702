"""The host C++ of the C ABI under AddressSanitizer + UBSan (SURVEY.md §5 'Race detection /
sanitizers').  csrc/numpy_rng.cpp (MT19937 + masked-rejection randint,
an AVX2 left-pack with a 256-entry LUT) is built with -fsanitize=address,undefined
(`make -C csrc sanitize`, tests/native/numpy_rng_driver.cpp) and run on the AVX-512 (where the
CPU has it), AVX2 and portable paths; every draw and the advanced state must equal np.random's own, and any
sanitizer report aborts the driver (non-zero exit)."""
import fcntl
import os
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "trade-offs-in-distributed-tuplewise-estimation-and-learning_amd" / "csrc"
EXE = ROOT / "tests" / "native" / "build" / "numpy_rng_asan"


@pytest.fixture(scope="module")
def driver():
    # one build at a time: pytest-xdist workers would otherwise relink the driver under a run
    EXE.parent.mkdir(parents=True, exist_ok=True)
    with open(EXE.parent / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", str(CSRC), "sanitize"], capture_output=True,
                           text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return EXE


def _run(exe, script, scalar):
    """scalar: False (widest SIMD level of the CPU), True (portable), or "avx2" (capped)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    if scalar == "avx2":
        env["TW_NP_RNG_ISA"] = "avx2"
    elif scalar:
        env["TW_NP_RNG_SCALAR"] = "1"
    r = subprocess.run([str(exe)], input=script, capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-2000:]
    vals = np.array(r.stdout.split(), dtype=np.int64)
    return int(vals[0]), vals[1:-625], int(vals[-625]), vals[-624:].astype(np.uint32)


def _state_script(mode, rs):
    _, key, pos, _, _ = rs.get_state()
    return f"{mode}\n{pos}\n" + " ".join(str(int(k)) for k in key) + "\n"


@pytest.mark.parametrize("scalar", [False, "avx2", True])
def test_randint_batch_sanitized_equals_numpy(driver, scalar):
    rs = np.random.RandomState(2024)
    rs.randint(0, 10, 7)  # a mid-block position
    calls = [(0, 1, 5), (0, 2, 33), (-5, 7, 100), (0, 9117, 4000), (3, 3 + 2 ** 31, 50),
             (0, 2 ** 32 + 5, 40), (-(2 ** 40), 2 ** 40, 60), (0, 702, 1), (0, 91, 0),
             (0, 255, 300), (0, 256, 300), (0, 257, 300)]
    script = _state_script("batch", rs) + f"{len(calls)}\n" + "".join(
        f"{lo} {hi} {n}\n" for lo, hi, n in calls)
    rc, got, pos, key = _run(driver, script, scalar)
    want = np.concatenate([rs.randint(lo, hi, n, dtype=np.int64) for lo, hi, n in calls])
    assert rc == 0 and np.array_equal(got, want)
    _, wkey, wpos, _, _ = rs.get_state()
    assert pos == wpos and np.array_equal(key, wkey)


@pytest.mark.parametrize("scalar", [False, "avx2", True])
def test_randint_pairs_sanitized_equals_numpy(driver, scalar):
    """grad_inc_block's draws for every shard of one step (compute_stats.py:155-156)."""
    rs = np.random.RandomState(7)
    N, kx, kz, B = 100, 91, 7, 100
    script = _state_script("pairs", rs) + f"{N} {kx} {kz} {B}\n"
    rc, got, pos, key = _run(driver, script, scalar)
    want = np.concatenate([np.concatenate([rs.randint(0, kx, B), rs.randint(0, kz, B)])
                           for _ in range(N)])
    assert rc == 0 and np.array_equal(got, want)
    _, wkey, wpos, _, _ = rs.get_state()
    assert pos == wpos and np.array_equal(key, wkey)


@pytest.mark.parametrize("scalar", [False, "avx2", True])
@pytest.mark.parametrize("nx,nz", [(1, 1), (2, 17), (1000, 3), (70000, 65537), (300001, 20)])
def test_shuffle_pair_sanitized_equals_numpy(driver, scalar, nx, nz):
    """tw_np_shuffle_pair (the draws, the AVX2 sure-accept batches, the threaded swaps) under
    ASan/UBSan against RandomState.shuffle itself."""
    rs = np.random.RandomState(77 + nx)
    rs.randint(0, 10, 3)
    script = _state_script("shuffle", rs) + f"{nx} {nz}\n"
    rc, got, pos, key = _run(driver, script, scalar)
    x, z = np.arange(nx), np.arange(nz)
    rs.shuffle(x)
    rs.shuffle(z)
    assert rc == 0 and np.array_equal(got, np.concatenate([x, z]))
    _, wkey, wpos, _, _ = rs.get_state()
    assert pos == wpos and np.array_equal(key, wkey)
