"""Parity of tw_count_pairs_idx(32)_ws (explicit index pairs compared on LDS rank codes) with
the plain index kernels tw_count_pairs_idx(32) and with a NumPy count of the same pairs, for
int32 and int64 indices, aligned (16-B vector loads) and misaligned (scalar loads) streams.

Replay mode of UB / UnNB (compute_stats.py:37-42, :104-123): the indices are NumPy randint
draws, absolute positions in the concatenated shard arrays.  Counts are integers: bit-exact.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _np_count(x, z, ix, iz, pair_off, mode):
    out = []
    for s in range(len(pair_off) - 1):
        a = x[ix[pair_off[s]:pair_off[s + 1]]]
        b = z[iz[pair_off[s]:pair_off[s + 1]]]
        if mode == "gt":
            out.append(int(np.sum(a > b)))
        elif mode == "half":
            out.append(int(np.sum(a > b)) + int(np.sum(a >= b)))
        else:  # subgt: (a - b) > 0 with int64 wrap
            with np.errstate(over="ignore", invalid="ignore"):  # inf - inf in the float cases
                out.append(int(np.sum((a - b) > 0)))
    return np.array(out, dtype=np.uint64)


def _sample(kind, rng):
    if kind == "gauss":
        nx = [3000, 2999, 1, 4096, 0, 700]
        nz = [2500, 3001, 5, 4096, 17, 0]
        x = rng.normal(0.5, 1, sum(nx))
        z = rng.normal(0, 1, sum(nz))
    elif kind == "edge_float":
        nx, nz = [400] * 5, [300] * 5
        vals = np.array([np.nan, -0.0, 0.0, np.inf, -np.inf, 1.0, 1.0, -1.0, 5e-324])
        x = rng.choice(vals, sum(nx))
        z = rng.choice(vals, sum(nz))
    elif kind == "ties_int":
        nx, nz = [5000, 4000, 20000], [6000, 3000, 20000]
        x = rng.integers(0, 7, sum(nx)).astype(np.int64)
        z = rng.integers(0, 7, sum(nz)).astype(np.int64)
    elif kind == "int64_wrap":
        nx, nz = [1000, 1000], [1000, 1000]
        big = np.array([2 ** 62, -(2 ** 62), 2 ** 63 - 1, -(2 ** 63), 0, 1], dtype=np.int64)
        x = rng.choice(big, sum(nx))
        z = rng.choice(big, sum(nz))
    elif kind == "large_shard":  # nz >= 65536: codes do not apply, the plain kernel runs
        nx, nz = [70000], [70000]
        x = rng.normal(0.5, 1, sum(nx))
        z = rng.normal(0, 1, sum(nz))
    else:
        raise ValueError(kind)
    x_off = np.concatenate([[0], np.cumsum(nx)]).astype(np.int64)
    z_off = np.concatenate([[0], np.cumsum(nz)]).astype(np.int64)
    return x, x_off, z, z_off


def _pairs(x_off, z_off, B, rng, stray=False):
    ix, iz, po = [], [], [0]
    for s in range(len(x_off) - 1):
        nx, nz = x_off[s + 1] - x_off[s], z_off[s + 1] - z_off[s]
        if nx == 0 or nz == 0:
            po.append(po[-1])
            continue
        a = x_off[s] + rng.integers(0, nx, B)
        b = z_off[s] + rng.integers(0, nz, B)
        if stray:  # indices outside the shard's span (allowed by tw_count_pairs_idx)
            a[::7] = rng.integers(0, x_off[-1], len(a[::7]))
            b[::5] = rng.integers(0, z_off[-1], len(b[::5]))
        ix.append(a)
        iz.append(b)
        po.append(po[-1] + B)
    return (np.concatenate(ix).astype(np.int64), np.concatenate(iz).astype(np.int64),
            np.array(po, dtype=np.int64))


def _idx(L, a, width, misalign):
    """Device index column of the given width; misalign = start 1 element into the buffer, so
    the base pointer is not 16-B aligned and the kernel takes its scalar-load path."""
    dt = np.int32 if width == 32 else np.int64
    if not misalign:
        return L.to_device(a, dt)
    return L.to_device(np.concatenate([[0], a]), dt)[1:]


@pytest.mark.parametrize("kind", ["gauss", "edge_float", "ties_int", "int64_wrap",
                                  "large_shard"])
@pytest.mark.parametrize("stray", [False, True])
@pytest.mark.parametrize("width,misalign", [(32, False), (64, False), (32, True)])
@pytest.mark.parametrize("codes", [3, 2])
def test_idx_ranked_matches_plain_and_numpy(gpu, kind, stray, width, misalign, codes):
    """codes 3: float32 images in LDS (default); 2: 16-bit rank codes (value buckets)."""
    from tuplewise import _engine as E, _lib as L
    L.call("tw_count_rng_set_codes", codes)
    try:
        _check_idx(E, L, kind, stray, width, misalign)
    finally:
        L.call("tw_count_rng_set_codes", 3)


def _check_idx(E, L, kind, stray, width, misalign):
    rng = np.random.default_rng(zlib.crc32(f"{kind}{stray}".encode()))
    x, x_off, z, z_off = _sample(kind, rng)
    ix, iz, po = _pairs(x_off, z_off, 20011, rng, stray)
    ixd, izd = _idx(L, ix, width, misalign), _idx(L, iz, width, misalign)
    code = L.TW_F64 if x.dtype == np.float64 else L.TW_I64
    xd, zd = L.to_device(x), L.to_device(z)
    xo, zo = L.to_device(x_off), L.to_device(z_off)
    max_nx, max_nz = int(np.diff(x_off).max()), int(np.diff(z_off).max())
    modes = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF, "subgt": L.TW_PRED_SUBGT}
    for mode, pred in modes.items():
        want = _np_count(x, z, ix, iz, po, mode)
        plain = E.count_indexed_dev(xd, zd, code, ixd, izd, po, pred).cpu().numpy().view(np.uint64)
        ranked = E.count_indexed_ranked_dev(xd, xo, zd, zo, max_nx, max_nz, code, ixd, izd, po,
                                            pred).cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(plain, want, err_msg=f"plain {kind} {mode}")
        np.testing.assert_array_equal(ranked, want, err_msg=f"ranked {kind} {mode}")


@pytest.mark.parametrize("codes,parts", [(3, 0), (3, 2), (3, 8), (2, 0), (2, 8), (2, 32)])
def test_idx_ranked_bench_shape(gpu, codes, parts):
    """The bench / C3 shape: 64 shards of 15625 x 15625, 1e6 int32 index pairs per shard, a
    512-block grid through xcd_block; every shard against a torch gather-compare."""
    import torch
    from tuplewise import _engine as E, _lib as L
    k, N, B = 15625, 64, 1_000_000
    g = torch.Generator(device="cuda").manual_seed(77 + parts)
    X = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g) + 0.5
    Z = torch.randn(N * k, dtype=torch.float64, device="cuda", generator=g)
    base = (torch.arange(N, device="cuda", dtype=torch.int64) * k).repeat_interleave(B)
    ix = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
    iz = (base + torch.randint(0, k, (N * B,), device="cuda", generator=g)).to(torch.int32)
    off = np.arange(N + 1, dtype=np.int64) * k
    po = np.arange(N + 1, dtype=np.int64) * B
    offd = L.to_device(off)
    want = (X[ix.long()] > Z[iz.long()]).view(N, B).sum(1).cpu().numpy().astype(np.uint64)
    L.call("tw_count_rng_set_codes", codes)
    L.call("tw_count_idx_set_parts", parts)
    L.call("tw_count_img_set_plan", parts, 2 if parts == 2 else 9)
    try:
        got = E.count_indexed_ranked_dev(X, offd, Z, offd, k, k, L.TW_F64, ix, iz, po,
                                         L.TW_PRED_GT).cpu().numpy().view(np.uint64)
    finally:
        L.call("tw_count_idx_set_parts", 0)
        L.call("tw_count_img_set_plan", 0, 9)
        L.call("tw_count_rng_set_codes", 3)
    np.testing.assert_array_equal(got, want)


def test_idx_ranked_codes_sorted_path(gpu):
    """The sort + binary-search rank codes (tw_count_rng_set_codes(0)) give the same counts."""
    from tuplewise import _engine as E, _lib as L
    rng = np.random.default_rng(5)
    x, x_off, z, z_off = _sample("gauss", rng)
    ix, iz, po = _pairs(x_off, z_off, 9999, rng)
    xd, zd = L.to_device(x), L.to_device(z)
    xo, zo = L.to_device(x_off), L.to_device(z_off)
    want = _np_count(x, z, ix, iz, po, "half")
    L.call("tw_count_rng_set_codes", 0)
    try:
        got = E.count_indexed_ranked_dev(xd, xo, zd, zo, int(np.diff(x_off).max()),
                                         int(np.diff(z_off).max()), L.TW_F64, ix, iz, po,
                                         L.TW_PRED_HALF).cpu().numpy().view(np.uint64)
    finally:
        L.call("tw_count_rng_set_codes", 3)
    np.testing.assert_array_equal(got, want)
