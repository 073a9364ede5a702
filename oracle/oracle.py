"""ORACLE — test infrastructure only.  CPU restatement of the reference's hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker (or, for cpu_baseline, as the timed CPU port).  The product package
never imports it; the product path fails loudly without the HIP library.

Every function restates one reference function (RobinVogel/Trade-offs-in-Distributed-
Tuplewise-Estimation-and-Learning) with NumPy, citing file:line.  Parity is PINNED: the
restatement is checked against golden vectors produced by the reference itself
(tests/golden/make_golden.py imports the reference read-only; tests/test_oracle_golden.py).

Beyond the reference (the device-only paths, whose results NumPy never produced):
  feistel_perm / philox4x32_10 restate csrc/permute.hip and csrc/count.hip bit for bit so the
  device-RNG repartition and incomplete paths can be checked exactly on small inputs.
  loss="logistic" (the pairwise-logistic loss BASELINE.json names) has
  no reference implementation: PARITY UNPINNED against the reference.  Its restatement is
  pinned only by its own definition — tests/test_oracle_golden.py checks the gradient against
  finite differences of the loss.
"""
from __future__ import annotations

import numpy as np

# ----------------------------------------------------------------- estimators (reference)


def un_count(X, Z) -> int:
    """#{(i,j): X_i > Z_j}: the integer behind est.Un (estimation-experiment/main.py:29-31)."""
    return int((np.asarray(X).reshape((-1, 1)) > np.asarray(Z).reshape((1, -1))).sum())


def est_Un(X, Z):
    """estimation-experiment/main.py:29-31"""
    return (X.reshape((-1, 1)) > Z.reshape((1, -1))).mean()


def cs_Un(X, Z, kernel="prod"):
    """learning-experiment/compute_stats.py:10-19"""
    X_col = X.reshape((-1, 1))
    Z_row = Z.reshape((1, -1))
    assert kernel in ["prod", "gini", "AUC"]
    if kernel == "prod":
        return (X_col.dot(Z_row)).mean()
    if kernel == "gini":
        return np.mean(np.abs(X_col - Z_row))
    return np.mean((X_col - Z_row > 0).astype(int))


def UB_indices(X, Z, ind_X, ind_Z, kernel):
    """compute_stats.py:22-30"""
    X_select = X[ind_X]
    Z_select = Z[ind_Z]
    assert kernel in ["prod", "gini", "AUC"]
    if kernel == "prod":
        return np.mean(X_select * Z_select)
    if kernel == "gini":
        return np.mean(np.abs(X_select - Z_select))
    return np.mean((X_select - Z_select > 0).astype(int))


def UB_pairs(X, Z, indices, kernel):
    """compute_stats.py:32-35"""
    idx = np.asarray(indices).reshape(-1, 2)
    return UB_indices(X, Z, idx[:, 0], idx[:, 1], kernel)


def UB(X, Z, B, kernel="prod"):
    """compute_stats.py:37-42 (draw order: X indices, then Z indices)"""
    return UB_indices(X, Z, np.random.randint(0, X.shape[0], B),
                      np.random.randint(0, Z.shape[0], B), kernel)


def UN(X, Z, N, f_block, sampling_type="SWOR", variant="cs"):
    """compute_stats.py:56-92 (variant "cs") / estimation-experiment/main.py:33-69 ("est").
    The two differ only for degenerate blocks (k in (0, tau)): cs asserts SWOR and appends 0;
    est appends 0 for SWOR and skips the block otherwise."""
    vals = []
    X_rem, Z_rem = X, Z
    np.random.shuffle(X_rem)
    np.random.shuffle(Z_rem)
    n_X, n_Z = X_rem.shape[0], Z_rem.shape[0]
    tau = int((n_X + n_Z) / N)
    for _ in range(N):
        if sampling_type != "prop-SWR":
            if sampling_type.startswith("prop"):
                k = int(n_X / N)
            else:
                n_X, n_Z = X_rem.shape[0], Z_rem.shape[0]
                k = np.random.binomial(tau, n_X / (n_X + n_Z))
            if k in (0, tau):
                if variant == "cs":
                    assert sampling_type == "SWOR"
                    vals.append(0)
                elif sampling_type == "SWOR":
                    vals.append(0)
            else:
                vals.append(f_block(X_rem[:k], Z_rem[:(tau - k)]))
            X_rem = X_rem[k:]
            Z_rem = Z_rem[(tau - k):]
        elif sampling_type == "prop-SWR":
            vals.append(f_block(X_rem[np.random.randint(0, n_X, int(n_X / N))],
                                Z_rem[np.random.randint(0, n_Z, int(n_Z / N))]))
    return np.mean(vals)


def est_UnN(X, Z, N, sampling_type):
    """estimation-experiment/main.py:72-74"""
    return UN(X, Z, N, est_Un, sampling_type, variant="est")


def est_UnNT(X, Z, N, T, sampling_type):
    """estimation-experiment/main.py:76-79"""
    return np.mean([est_UnN(X, Z, N, sampling_type) for _ in range(T)])


def cs_UnN(X, Z, N, sampling_type, kernel="prod"):
    """compute_stats.py:95-101"""
    return UN(X, Z, N, lambda x, z: cs_Un(x, z, kernel=kernel), sampling_type, "cs")


def cs_UnNB(X, Z, N, B, sampling_type, kernel="prod"):
    """compute_stats.py:104-110"""
    return UN(X, Z, N, lambda x, z: UB(x, z, B, kernel=kernel), sampling_type, "cs")


def cs_UnNT(X, Z, N, T, sampling_type, kernel="prod"):
    """compute_stats.py:113-116"""
    return np.mean([cs_UnN(X, Z, N, sampling_type, kernel) for _ in range(T)])


def cs_UnNBT(X, Z, N, B, T, sampling_type, kernel="prod"):
    """compute_stats.py:119-123"""
    return np.mean([cs_UnNB(X, Z, N, B, sampling_type, kernel) for _ in range(T)])


def SWR_divide(X, Z, N):
    """compute_stats.py:48-54 (all N X-draws first, then all N Z-draws)"""
    n_X, n_Z = X.shape[0], Z.shape[0]
    X_s = [X[np.random.randint(0, n_X, int(n_X / N))] for _ in range(N)]
    Z_s = [Z[np.random.randint(0, n_Z, int(n_Z / N))] for _ in range(N)]
    return X_s, Z_s


def UN_split(X_s, Z_s, f_block):
    """compute_stats.py:44-46"""
    return np.mean([f_block(X, Z) for X, Z in zip(X_s, Z_s)], axis=0)


def _surrogate(t, loss):
    """Pair loss of the convexified 1-AUC: hinge max(t, 0) (compute_stats.py:135) or, for the
    row-L3 extension (NOT in the reference; parity unpinned against it), the logistic
    softplus(t) = log(1 + e^t), evaluated as NumPy's stable logaddexp(0, t)."""
    if loss == "hinge":
        return np.maximum(t, 0)
    if loss == "logistic":
        return np.logaddexp(0, t)
    raise ValueError(loss)


def conv_AUC(margin, loss="hinge"):
    """compute_stats.py:129-135"""
    def res_function(X, Z):
        return _surrogate(Z.reshape((1, -1)) - X.reshape((-1, 1)) + margin, loss).mean()
    return res_function


def conv_AUC_deter_pairs(margin, loss="hinge"):
    """compute_stats.py:137-144"""
    def res(X, Z, indices):
        idx = np.asarray(indices).reshape(-1, 2)
        return _surrogate(Z[idx[:, 1]] - X[idx[:, 0]] + margin, loss).mean()
    return res


def pair_grad(diff, w, margin, B, loss="hinge"):
    """The body of grad_inc_block after the draws (compute_stats.py:157-162): hinge sums the
    filtered rows in row order; logistic (row L3 extension) weights every row by
    sigma(S) = 1 / (1 + e^-S), the derivative of softplus(S), and sums in row order."""
    S_diff = diff.dot(w) + margin
    if loss == "hinge":
        filt = (S_diff > 0).ravel()
        return (diff[filt].sum(axis=0) / B).reshape([-1, 1])
    if loss == "logistic":
        wgt = 1.0 / (1.0 + np.exp(-S_diff.ravel()))
        return ((wgt[:, None] * diff).sum(axis=0) / B).reshape([-1, 1])
    raise ValueError(loss)


def grad_complete_block(w, margin, loss="hinge"):
    """Extension, NOT in the reference (BASELINE.json north_star item (2)): the surrogate's
    gradient over ALL pairs of a block, (1/(kx kz)) sum_ij phi'(S_ij) (z_j - x_i) with
    S_ij = z_j.w - x_i.w + margin, factorised into per-point coefficients
    a_j = sum_i phi'(S_ij), b_i = sum_j phi'(S_ij) and (a.Z - b.X) / (kx kz).  Pinned in
    tests/test_oracle_golden.py against the unfactorised double sum and, for the logistic loss,
    finite differences of the complete surrogate."""
    def res(X, Z):
        sx, sz = X.dot(w).ravel(), Z.dot(w).ravel()
        S = sz[None, :] - sx[:, None] + margin
        if loss == "hinge":
            P = (S > 0).astype(np.float64)
        elif loss == "logistic":
            P = 1.0 / (1.0 + np.exp(-S))
        else:
            raise ValueError(loss)
        a, b = P.sum(axis=0), P.sum(axis=1)
        return ((a.dot(Z) - b.dot(X)) / (len(sx) * len(sz))).reshape([-1, 1])
    return res


def grad_inc_block(w, B, margin, loss="hinge"):
    """compute_stats.py:146-162"""
    def res(X, Z):
        X_sel = X[np.random.randint(0, X.shape[0], B)]
        Z_sel = Z[np.random.randint(0, Z.shape[0], B)]
        return pair_grad(Z_sel - X_sel, w, margin, B, loss)
    return res


def sgd_step(w, delta_w, gradient_mean, reg, learning_rate, optim_type="momentum"):
    """learning-experiment/make_exps.py:130-141"""
    gradient = gradient_mean + reg * w
    if optim_type == "SGD":
        delta_w = learning_rate * gradient
    if optim_type == "momentum":
        delta_w = 0.9 * delta_w + learning_rate * gradient
    return w - delta_w, delta_w


def learning_trajectory(X, Z, p_learn, capture_every=1, loss="hinge", optim_type="momentum"):
    """learning_process (make_exps.py:96-141) without evaluation: returns the w before every
    gradient step (the values the reference passes to grad_inc_block at :130)."""
    N, B = p_learn["N"], p_learn["B"]
    w = p_learn["w_init"]
    ws = []
    X_s, Z_s = SWR_divide(X, Z, N)
    delta_w = 0
    for i in range(p_learn["n_it"]):
        if i % p_learn["reshuffle_mod"] == 0:
            X_s, Z_s = SWR_divide(X, Z, N)
        if i % capture_every == 0:
            ws.append(np.array(w, copy=True))
        g = UN_split(X_s, Z_s, grad_inc_block(w, B, p_learn["margin"], loss))
        w, delta_w = sgd_step(w, delta_w, g, p_learn["reg"], p_learn["learning_rate"],
                              optim_type)
    return ws, w


# ----------------------------------------------------------------- theory (reference)
def Mean_Un(e):
    """estimation-experiment/main.py:26-27 with p(e)=e, q(e)=1-e (:10-14)"""
    return (1 - e) + e * (1 - e)


def Var_Un(e, n, m):
    """estimation-experiment/main.py:16-23, :103-104"""
    p, q = e, 1 - e
    s1 = (p ** 2) * q * (1 - q)
    s2 = ((1 - q) ** 2) * p * (1 - p)
    s0 = p * q * (1 - p) * (1 - q)
    return s1 / n + s2 / m + s0 / (n * m)


# ----------------------------------------------------------------- exact large-n count
def count_gt_sorted(X, Z) -> int:
    """#{(i,j): X_i > Z_j} in O((n+m) log m) (NaN-free inputs): for each x, the number of z
    strictly below it.  Same integer as un_count; feasible at n = 1e6 where the reference's
    n*m boolean temporary is not."""
    zs = np.sort(np.asarray(Z).reshape(-1))
    return int(np.searchsorted(zs, np.asarray(X).reshape(-1), side="left").sum())


def count_half_sorted(X, Z) -> int:
    """2*#{x>z} + #{x==z} (tie_mode="half" half-units)."""
    zs = np.sort(np.asarray(Z).reshape(-1))
    x = np.asarray(X).reshape(-1)
    lo = np.searchsorted(zs, x, side="left")
    hi = np.searchsorted(zs, x, side="right")
    return int((lo + hi).sum())


# ----------------------------------------------------------------- device-RNG restatements
_M32 = np.uint64(0xFFFFFFFF)


def _mix32(v):
    v = v & _M32
    v ^= v >> np.uint64(16)
    v = (v * np.uint64(0x85EBCA6B)) & _M32
    v ^= v >> np.uint64(13)
    v = (v * np.uint64(0xC2B2AE35)) & _M32
    v ^= v >> np.uint64(16)
    return v


def _feistel_keys(n: int, key: int):
    bits = 2
    while bits < 62 and (1 << bits) < n:
        bits += 1
    if bits & 1:
        bits += 1
    half = bits // 2
    st = (key ^ 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
    ks = []
    for _ in range(6):
        st = (st + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2 ** 64 - 1)
        z ^= z >> 31
        ks.append(z & 0xFFFFFFFF)
    return half, ks


def feistel_perm(idx, n: int, key: int) -> np.ndarray:
    """Restates csrc/permute.hip feistel_perm: keyed bijection of [0, n)."""
    half, ks = _feistel_keys(n, key)
    mask = np.uint64((1 << half) - 1)
    hb = np.uint64(half)

    def once(v):
        L = (v >> hb) & mask
        R = v & mask
        for k in ks:
            nL = R
            R = (L ^ _mix32((R * np.uint64(0x9E3779B1) + np.uint64(k)) & _M32)) & mask
            L = nL
        return (L << hb) | R

    v = once(np.asarray(idx, dtype=np.uint64))
    while True:
        bad = v >= np.uint64(n)
        if not bad.any():
            return v.astype(np.int64)
        v[bad] = once(v[bad])


def feistel_perm_inv(pos, n: int, key: int) -> np.ndarray:
    """Restates csrc/permute.hip feistel_perm_inv: the inverse bijection (rounds reversed,
    cycle walking backwards)."""
    half, ks = _feistel_keys(n, key)
    mask = np.uint64((1 << half) - 1)
    hb = np.uint64(half)

    def once_inv(v):
        L = (v >> hb) & mask
        R = v & mask
        for k in reversed(ks):
            pR = L
            L = (R ^ _mix32((pR * np.uint64(0x9E3779B1) + np.uint64(k)) & _M32)) & mask
            R = pR
        return (L << hb) | R

    v = once_inv(np.asarray(pos, dtype=np.uint64))
    while True:
        bad = v >= np.uint64(n)
        if not bad.any():
            return v.astype(np.int64)
        v[bad] = once_inv(v[bad])


def order_keys(v) -> np.ndarray:
    """Restates csrc/sortkeys.h order_key: order-preserving uint64 keys (NaN above every
    value, -0.0 == +0.0; int64 by flipping the sign bit)."""
    v = np.asarray(v).reshape(-1)
    if v.dtype == np.int64:
        return v.view(np.uint64) ^ np.uint64(1 << 63)
    v = v.astype(np.float64)
    b = v.view(np.uint64).copy()
    b[v == 0] = 0
    neg = (b >> np.uint64(63)) == 1
    k = np.where(neg, ~b, b | np.uint64(1 << 63))
    k[np.isnan(v)] = np.uint64(2 ** 64 - 1)
    return k


def rank_records(X, Z, half=False, Z_all=None):
    """Restates csrc/rankimage.hip tw_rank_images (the round-3 all-pairs count on packed f32
    images; not a reference function): every element's image is the number of Z-scores whose
    order key is below its own, g(v) = #{z : key(z) < key(v)} (NaN x: -2^25); z images are
    stored negated.  Records: low word the f32 image bits, high word the element's index.  For
    every pair, X_i > Z_j  <=>  x_image + z_image >= 1.
    tw_rank_images_query: Z_all (default Z) is the Z the images count; half=True puts
    h(x) = #{z : key(z) <= key(x)} (NaN x: -2^25) in the X records' high word instead of the
    index, so that X_i >= Z_j  <=>  h_image + z_image >= 1."""
    X, Z = np.asarray(X).reshape(-1), np.asarray(Z).reshape(-1)
    n, m = X.size, Z.size
    zk = np.sort(order_keys(Z if Z_all is None else np.asarray(Z_all).reshape(-1)))
    gx = np.searchsorted(zk, order_keys(X), side="left").astype(np.float32)
    gz = np.searchsorted(zk, order_keys(Z), side="left").astype(np.float32)
    hi = np.arange(n, dtype=np.uint64)
    if half:
        hx = np.searchsorted(zk, order_keys(X), side="right").astype(np.float32)
        if X.dtype != np.int64:
            hx[np.isnan(X)] = np.float32(-2.0 ** 25)
        hi = hx.view(np.uint32).astype(np.uint64)
    if X.dtype != np.int64:
        gx[np.isnan(X)] = np.float32(-2.0 ** 25)
    xr = gx.view(np.uint32).astype(np.uint64) | (hi << np.uint64(32))
    zr = (-gz).view(np.uint32).astype(np.uint64) | (np.arange(m, dtype=np.uint64)
                                                    << np.uint64(32))
    return xr.view(np.int64), zr.view(np.int64)


def permute_scatter(vals: np.ndarray, key: int) -> np.ndarray:
    """out[perm(i)] = vals[i] (tw_permute_scatter)."""
    out = np.empty_like(vals)
    out[feistel_perm(np.arange(len(vals)), len(vals), key)] = vals
    return out


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 (Salmon et al. 2011), vectorised; restates csrc/count.hip."""
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = 0x9E3779B9, 0xBB67AE85
    a, b, c, d = (np.asarray(v, dtype=np.uint64) & _M32 for v in (c0, c1, c2, c3))
    for _ in range(10):
        p0 = a * M0
        p1 = c * M1
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        a, b, c, d = (hi1 ^ b ^ np.uint64(k0)) & _M32, lo1, (hi0 ^ d ^ np.uint64(k1)) & _M32, lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return a, b, c, d


def _mulhi64(a: np.ndarray, n: int) -> np.ndarray:
    return np.array([(int(v) * n) >> 64 for v in a], dtype=np.int64)


def _lemire(words: np.ndarray, n: int, q: np.ndarray, shard: int, w: int, seed: int):
    """Lemire's multiply-shift with rejection (csrc/count.hip lemire_index): (r * n) >> 32,
    a rejected word replaced by word w of the Philox block at counter word 3 = 1, 2, ..."""
    m = words.astype(np.uint64) * np.uint64(n)
    t = np.uint64(((1 << 32) - n) % n)
    bad = (m & _M32) < t
    att = 1
    while bad.any():
        qb = q[bad]
        r = philox4x32_10(qb & _M32, qb >> np.uint64(32), np.full(qb.size, shard, np.uint64),
                          np.full(qb.size, att, np.uint64), seed & 0xFFFFFFFF,
                          (seed >> 32) & 0xFFFFFFFF)[w]
        m[bad] = r * np.uint64(n)
        bad = (m & _M32) < t
        att += 1
    return (m >> np.uint64(32)).astype(np.int64)


def rng_pairs(nx: int, nz: int, B: int, seed: int, shard: int):
    """The (i, j) pairs tw_count_pairs_rng draws for one shard (global shard index):
    Philox block q gives pairs 2q (words 0, 1) and 2q+1 (words 2, 3) (csrc/count.hip
    k_count_rng); shards of >= 2^32 values use one block per pair and 64-bit multiply-high."""
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    if nx >= 1 << 32 or nz >= 1 << 32:
        p = np.arange(B, dtype=np.uint64)
        a, b, c, d = philox4x32_10(p & _M32, p >> np.uint64(32), np.full(B, shard, np.uint64),
                                   np.zeros(B, np.uint64), k0, k1)
        return (_mulhi64((b << np.uint64(32)) | a, nx), _mulhi64((d << np.uint64(32)) | c, nz))
    q = np.arange((B + 1) // 2, dtype=np.uint64)
    a, b, c, d = philox4x32_10(q & _M32, q >> np.uint64(32), np.full(q.size, shard, np.uint64),
                               np.zeros(q.size, np.uint64), k0, k1)
    i = np.empty(2 * q.size, np.int64)
    j = np.empty(2 * q.size, np.int64)
    i[0::2] = _lemire(a, nx, q, shard, 0, seed)
    j[0::2] = _lemire(b, nz, q, shard, 1, seed)
    i[1::2] = _lemire(c, nx, q, shard, 2, seed)
    j[1::2] = _lemire(d, nz, q, shard, 3, seed)
    return i[:B], j[:B]


def _sgd_draw(seed, step, idx, shard, tag):
    """Restates csrc/hinge.hip sgd_draw: Philox counter (idx, shard, step lo, tag|step hi)."""
    idx = np.asarray(idx, dtype=np.uint64)
    n = idx.size
    a, b, c, d = philox4x32_10(idx, np.full(n, shard, np.uint64),
                               np.full(n, step & 0xFFFFFFFF, np.uint64),
                               np.full(n, tag | (step >> 32), np.uint64),
                               seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return (b << np.uint64(32)) | a, (d << np.uint64(32)) | c


def device_rng_learning_trajectory(X, Z, p_learn, seed, optim_type="momentum", loss="hinge"):
    """learning_process (make_exps.py:96-141) with the device-RNG draws of
    tw_swr_rows_rng / tw_hinge_grad_rng (tags 0x40000000 / 0x20000000 / 0x80000000) and the
    reference's gradient/update arithmetic; returns w before every step."""
    N, B = p_learn["N"], p_learn["B"]
    n_X, n_Z = X.shape[0], Z.shape[0]
    kx, kz = int(n_X / N), int(n_Z / N)
    w = p_learn["w_init"]
    delta_w = 0
    ws = []
    rows_x = rows_z = None
    for i in range(p_learn["n_it"]):
        if i % p_learn["reshuffle_mod"] == 0:
            rows_x = [_mulhi64(_sgd_draw(seed, i, np.arange(kx), s, 0x40000000)[0], n_X)
                      for s in range(N)]
            rows_z = [_mulhi64(_sgd_draw(seed, i, np.arange(kz), s, 0x20000000)[0], n_Z)
                      for s in range(N)]
        ws.append(np.array(w, copy=True))
        grads = []
        for s in range(N):
            u, v = _sgd_draw(seed, i, np.arange(B), s, 0x80000000)
            ix, iz = _mulhi64(u, kx), _mulhi64(v, kz)
            diff = Z[rows_z[s]][iz] - X[rows_x[s]][ix]
            grads.append(pair_grad(diff, w, p_learn["margin"], B, loss))
        g = np.mean(grads, axis=0)
        w, delta_w = sgd_step(w, delta_w, g, p_learn["reg"], p_learn["learning_rate"],
                              optim_type)
    return ws, w
