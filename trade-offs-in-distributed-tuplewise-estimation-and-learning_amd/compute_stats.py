"""Drop-in replacement for learning-experiment/compute_stats.py on MI355X.

Same names, signatures, defaults, RNG consumption, side effects and exceptions as the
reference module; the pair arithmetic runs in libtuplewise.so's HIP kernels.  Block functions
returned here (the fun_block closures of UnN/UnNB, conv_AUC's result, grad_inc_block's
result) stay ordinary callables, and additionally carry a ``_tw_block`` spec that lets UN /
UN_split evaluate every block in one device launch.
"""
from __future__ import annotations

import numpy as np

from . import _blocks as Bk
from . import _lib as L
from . import _learn
from .numpy_rng import randint_batch

_KERNELS = ["prod", "gini", "AUC"]


# ---------- Definitions of the estimators --------

def Un(X, Z, kernel="prod"):
    """Computes Un, full two-sample U-statistic.  (compute_stats.py:10-19)"""
    assert kernel in _KERNELS
    X = np.asarray(X)
    Z = np.asarray(Z)
    blk = Bk.whole(X, Z)
    if kernel == "AUC":
        return Bk.CompleteCount(literal_sub=True).evaluate(X, Z, [blk])[0]
    kern = L.TW_KERN_PROD if kernel == "prod" else L.TW_KERN_GINI
    return Bk.CompleteSum(kern).evaluate(X, Z, [blk])[0]


def UB_indices(X, Z, ind_X, ind_Z, kernel):
    """Mean of `kernel` over the given index pairs.  (compute_stats.py:22-30)"""
    X = np.asarray(X)
    Z = np.asarray(Z)
    ind_X = _check_index(np.asarray(ind_X), X.shape[0])
    ind_Z = _check_index(np.asarray(ind_Z), Z.shape[0])
    assert kernel in _KERNELS
    if ind_X.shape != ind_Z.shape:
        raise ValueError(f"operands could not be broadcast together with shapes "
                         f"{ind_X.shape} {ind_Z.shape}")
    rs = Bk._row_size(X)
    if Bk._row_size(Z) != rs:
        raise ValueError(f"operands could not be broadcast together with shapes "
                         f"{X[ind_X].shape} {Z[ind_Z].shape}")
    ix, iz = ind_X.reshape(-1), ind_Z.reshape(-1)
    if rs > 1:  # X[ind_X] - Z[ind_Z] on whole rows: element pairs column by column
        ix = (ix[:, None] * rs + np.arange(rs)).reshape(-1)
        iz = (iz[:, None] * rs + np.arange(rs)).reshape(-1)
    off = np.array([0, ix.size], dtype=np.int64)
    return Bk.indexed_values(X.reshape(-1), Z.reshape(-1), ix, iz, off, kernel)[0]


def UB_pairs(X, Z, indices, kernel):
    """Computes incomplete two-sample U-statistic for given pairs.  (compute_stats.py:32-35)"""
    idx = np.asarray(list(indices) if not isinstance(indices, (list, np.ndarray)) else indices,
                     dtype=np.int64).reshape(-1, 2)
    return UB_indices(X, Z, idx[:, 0], idx[:, 1], kernel)


def UB(X, Z, B, kernel="prod"):
    """Computes incomplete two-sample U-statistic.  (compute_stats.py:37-42)"""
    n_X = X.shape[0]
    n_Z = Z.shape[0]
    return UB_indices(X, Z, np.random.randint(0, n_X, B), np.random.randint(0, n_Z, B), kernel)


def UN_split(X_s, Z_s, f_block):
    """Computes UN for all of the blocks in X_s, Z_s.  (compute_stats.py:44-46)"""
    spec = getattr(f_block, "_tw_block", None)
    if spec is not None and hasattr(spec, "evaluate_split"):
        return spec.evaluate_split(X_s, Z_s)
    return np.mean([f_block(X, Z) for X, Z in zip(X_s, Z_s)], axis=0)


def SWR_divide(X, Z, N):
    """Divides the sample with sampling with replacement.  (compute_stats.py:48-54)

    Returns lists of row copies like the reference; the lists also remember the drawn row
    indices so device consumers (UN_split with grad_inc_block) can gather on the GPU."""
    n_X = X.shape[0]
    n_Z = Z.shape[0]
    rows = randint_batch([(0, n_X, int(n_X / N))] * N + [(0, n_Z, int(n_Z / N))] * N)
    rows_x, rows_z = rows[:N], rows[N:]
    return (_learn.ShardList([X[r] for r in rows_x], X, rows_x),
            _learn.ShardList([Z[r] for r in rows_z], Z, rows_z))


def UN(X, Z, N, f_block, sampling_type="SWOR"):
    """Computes complete or incomplete (depending on f_block) two-sample U-statistic on each
    worker and averages them.  Cuts the dataset X,Z in N splits.  sampling_type can be SWOR,
    prop-SWOR or prop-SWR.  (compute_stats.py:56-92)"""
    return Bk.run_un(X, Z, N, f_block, sampling_type, variant="cs")


def _block_fn(spec, fn):
    fn._tw_block = spec
    return fn


def UnN(X, Z, N, sampling_type, kernel="prod"):
    """Computes block-wise complete U-statistic.  (compute_stats.py:95-101)"""

    def fun_block(x, z):
        return Un(x, z, kernel=kernel)

    assert kernel in _KERNELS
    if kernel == "AUC":
        spec = Bk.CompleteCount(literal_sub=True)
    else:
        spec = Bk.CompleteSum(L.TW_KERN_PROD if kernel == "prod" else L.TW_KERN_GINI)
    return UN(X, Z, N, _block_fn(spec, fun_block), sampling_type=sampling_type)


def UnNB(X, Z, N, B, sampling_type, kernel="prod"):
    """Computes block-wise incomplete U-statistic.  (compute_stats.py:104-110)"""

    def fun_block(x, z):
        return UB(x, z, B, kernel=kernel)

    assert kernel in _KERNELS
    return UN(X, Z, N, _block_fn(Bk.Incomplete(B, kernel), fun_block),
              sampling_type=sampling_type)


def UnNT(X, Z, N, T, sampling_type, kernel="prod"):
    """Computes reshuffled block-wise complete U-statistic.  (compute_stats.py:113-116)
    The T repetitions' blocks are counted in one launch (_blocks.run_un_repeated)."""
    assert kernel in _KERNELS
    if kernel == "AUC":
        spec = Bk.CompleteCount(literal_sub=True)
    else:
        spec = Bk.CompleteSum(L.TW_KERN_PROD if kernel == "prod" else L.TW_KERN_GINI)
    v = Bk.run_un_repeated(X, Z, N, spec, sampling_type, "cs", T)
    if v is not None:
        return v
    return np.mean([UnN(X, Z, N, sampling_type=sampling_type, kernel=kernel)
                    for _ in range(T)])


def UnNBT(X, Z, N, B, T, sampling_type, kernel="prod"):
    """Computes reshuffled block-wise incomplete U-statistic.  (compute_stats.py:119-123)
    The T repetitions' blocks are counted in one launch (_blocks.run_un_repeated)."""
    assert kernel in _KERNELS
    v = Bk.run_un_repeated(X, Z, N, Bk.Incomplete(B, kernel), sampling_type, "cs", T)
    if v is not None:
        return v
    return np.mean([UnNB(X, Z, N, B, sampling_type=sampling_type, kernel=kernel)
                    for _ in range(T)])

# -------- End of the definition of the estimators -------

# ---------- Gradient descent functions ----------


_LOSSES = {"hinge": (L.TW_KERN_HINGE, L.TW_LOSS_HINGE),
           "logistic": (L.TW_KERN_LOGISTIC, L.TW_LOSS_LOGISTIC)}


def _loss_codes(loss):
    if loss not in _LOSSES:
        raise ValueError(f"loss must be 'hinge' or 'logistic', not {loss!r}")
    return _LOSSES[loss]


def conv_AUC(margin, *, loss="hinge"):
    """Complete hinge surrogate of 1-AUC.  (compute_stats.py:129-135)

    loss="logistic" (keyword-only extension; not in the reference):
    softplus(z - x + margin) instead of max(z - x + margin, 0)."""
    kern = _loss_codes(loss)[0]

    def res_function(X, Z):
        """Computes the convexification of the 1-AUC that we minimize."""
        X = np.asarray(X)
        Z = np.asarray(Z)
        blk = Bk.whole(X, Z)
        return Bk.CompleteSum(kern, float(margin)).evaluate(X, Z, [blk])[0]
    return _block_fn(Bk.CompleteSum(kern, float(margin)), res_function)


def conv_AUC_deter_pairs(margin, *, loss="hinge"):
    """Returns function that computes the convex loss on incomplete U-stat.
    (compute_stats.py:137-144); loss as in conv_AUC."""
    _loss_codes(loss)

    def res(X, Z, indices):
        """Computes the convexification of the 1-AUC that we minimize."""
        idx = np.asarray(indices, dtype=np.int64).reshape(-1, 2)
        X = np.asarray(X)
        Z = np.asarray(Z)
        ix = _check_index(idx[:, 0], X.shape[0])
        iz = _check_index(idx[:, 1], Z.shape[0])
        off = np.array([0, len(ix)], dtype=np.int64)
        return Bk.indexed_values(_columns(X), _columns(Z), ix, iz, off, loss,
                                 float(margin))[0]
    return res


def grad_inc_block(w, B, margin, *, loss="hinge"):
    """Returns a function that computes the gradient on incomplete U-stat.
    (compute_stats.py:146-162)

    loss="logistic" (keyword-only extension, row L3): every drawn pair's diff is weighted by
    sigma(diff . w + margin), the gradient of softplus, instead of the hinge filter."""
    return _learn.grad_block(w, B, margin, _loss_codes(loss)[1])

def grad_complete_block(w, margin, *, loss="hinge"):
    """Extension (not in the reference; BASELINE.json north_star item (2)): a block function
    returning the surrogate's gradient over ALL pairs of the block,
    1/(n_X n_Z) sum_ij phi'(S_ij) (Z_j - X_i), S_ij = w.(Z_j - X_i) + margin, computed on the
    device as per-point pair-coefficient reductions followed by X^T c.  Composes with UN_split
    like grad_inc_block (one launch for all shards)."""
    return _learn.complete_grad_block(w, margin, _loss_codes(loss)[1])

# ---------- End gradient descent functions ----------


def _check_index(ind: np.ndarray, n: int) -> np.ndarray:
    ind = np.asarray(ind)
    if ind.dtype == np.bool_:
        raise NotImplementedError("boolean masks are not pair indices")
    ind = ind.astype(np.int64, copy=False)
    if ind.size:
        lo, hi = int(ind.min()), int(ind.max())
        if lo < -n or hi >= n:
            bad = hi if hi >= n else lo
            raise IndexError(f"index {bad} is out of bounds for axis 0 with size {n}")
        if lo < 0:
            ind = np.where(ind < 0, ind + n, ind)
    return ind


def _columns(A: np.ndarray) -> np.ndarray:
    """Score vectors as 1-D: (n,) or (n, 1) like evaluation_step's `X.dot(w)` columns."""
    A = np.asarray(A)
    if A.ndim == 2 and A.shape[1] == 1:
        return A[:, 0]
    if A.ndim == 1:
        return A
    raise NotImplementedError(f"pair indices into a {A.shape} array (one score per row only)")
