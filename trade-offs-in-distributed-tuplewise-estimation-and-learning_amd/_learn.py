"""Pairwise hinge gradient on shards — host side.

grad_inc_block(w, B, margin) (learning-experiment/compute_stats.py:146-162) returns a closure;
UN_split (compute_stats.py:44-46) calls it once per shard and averages with np.mean(axis=0).
The closure returned here draws the same randint pairs in the same order and evaluates the
gradient with tw_hinge_grad; UN_split recognises it and evaluates all shards in one launch.
"""
from __future__ import annotations

import numpy as np

from . import _blocks as Bk
from . import _lib as L
from .numpy_rng import randint_batch


class ShardList(list):
    """list of shard row-copies (what the reference's SWR_divide returns) that also remembers
    the source matrix and the drawn row indices, so device code can gather rows on the GPU."""

    def __init__(self, items, source=None, rows=None):
        super().__init__(items)
        self.source = source
        self.rows = rows


def _as_matrix(A) -> np.ndarray:
    A = np.asarray(A, dtype=np.float64)
    return A.reshape(-1, 1) if A.ndim == 1 else A


def hinge_grads_device(Xd, Zd, d, rows_x, kx, rows_z, kz, ixd, izd, n_shards, B, wd, margin,
                       loss=L.TW_LOSS_HINGE):
    """Per-shard gradients (n_shards, d) on the device via tw_pair_grad."""
    t = L.torch()
    out = L.empty((n_shards, d), t.float64)
    L.call("tw_pair_grad", L.ptr(Xd), L.ptr(Zd), int(d), L.ptr(rows_x), int(kx), L.ptr(rows_z),
           int(kz), L.ptr(ixd), L.ptr(izd), int(n_shards), int(B), L.ptr(wd), float(margin),
           int(loss), L.ptr(out), L.stream_handle())
    return out


class GradSpec(Bk.BlockSpec):
    def __init__(self, w, B, margin, loss=L.TW_LOSS_HINGE):
        self.w = np.asarray(w, dtype=np.float64)
        self.B = int(B)
        self.margin = margin
        self.loss = loss

    def draw(self, nx, nz):
        ix = np.random.randint(0, nx, self.B)
        iz = np.random.randint(0, nz, self.B)
        return ix, iz

    def _grads(self, X_s, Z_s):
        N = min(len(X_s), len(Z_s))
        if N == 0:
            return []
        # every shard's two randint calls (X then Z, shard by shard) in one native batch
        calls = []
        for x, z in zip(X_s, Z_s):
            calls += [(0, np.asarray(x).shape[0], self.B), (0, np.asarray(z).shape[0], self.B)]
        out = randint_batch(calls)
        ix = np.stack(out[0::2])
        iz = np.stack(out[1::2])
        d = _as_matrix(X_s[0]).shape[1]

        def side(S, draws_idx):
            rows = getattr(S, "rows", None)
            src = getattr(S, "source", None)
            if rows is not None and src is not None and len({len(r) for r in rows}) == 1:
                return (L.to_device(_as_matrix(src)), L.to_device(np.stack(rows).astype(np.int64)),
                        len(rows[0]), draws_idx)
            mats = [_as_matrix(a) for a in S]
            off = np.concatenate([[0], np.cumsum([m.shape[0] for m in mats])])[:-1]
            absolute = draws_idx + off[:, None]  # rows of the concatenated shards
            return L.to_device(np.concatenate(mats)), None, 0, absolute

        Xd, rx, kx, ixa = side(X_s, ix)
        Zd, rz, kz, iza = side(Z_s, iz)
        wd = L.to_device(self.w.reshape(-1))
        out = hinge_grads_device(Xd, Zd, d, rx, kx, rz, kz, L.to_device(ixa), L.to_device(iza),
                                 N, self.B, wd, self.margin, self.loss)
        return [g.reshape(-1, 1) for g in out.cpu().numpy()]

    def evaluate_split(self, X_s, Z_s):
        return np.mean(self._grads(X_s, Z_s), axis=0)


def grad_block(w, B, margin, loss=L.TW_LOSS_HINGE):
    spec = GradSpec(w, B, margin, loss)

    def res(X, Z):
        """
            Returns:
            1/B sum_{i,j in D_B} I{w^T(Z_j - X_i + margin > 0)}(Z_j - X_i)
        """
        return spec._grads([X], [Z])[0]

    res._tw_block = spec
    return res


def complete_grads_device(Xd, Zd, d, rows_x, kx, rows_z, kz, n_shards, wd, margin,
                          loss=L.TW_LOSS_HINGE):
    """Per-shard complete-block gradients (n_shards, d) via tw_pair_grad_complete."""
    t = L.torch()
    out = L.empty((n_shards, d), t.float64)
    work = L.empty((max(1, int(L.lib().tw_pair_grad_complete_work_bytes(n_shards, kx, kz,
                                                                          d))),), t.uint8)
    L.call("tw_pair_grad_complete", L.ptr(Xd), L.ptr(Zd), int(d), L.ptr(rows_x), int(kx),
           L.ptr(rows_z), int(kz), int(n_shards), L.ptr(wd), float(margin), int(loss),
           L.ptr(work), L.ptr(out), L.stream_handle())
    return out


class CompleteGradSpec(Bk.BlockSpec):
    """The complete-block gradient (extension): all pairs of each block, per-point pair
    coefficients then X^T c on the device."""

    def __init__(self, w, margin, loss=L.TW_LOSS_HINGE):
        self.w = np.asarray(w, dtype=np.float64)
        self.margin = margin
        self.loss = loss

    def _grads(self, X_s, Z_s):
        N = min(len(X_s), len(Z_s))
        if N == 0:
            return []
        X_s, Z_s = list(X_s)[:N], list(Z_s)[:N]
        d = _as_matrix(X_s[0]).shape[1]
        wd = L.to_device(self.w.reshape(-1))
        sizes_x = {_as_matrix(a).shape[0] for a in X_s}
        sizes_z = {_as_matrix(a).shape[0] for a in Z_s}
        if len(sizes_x) == 1 and len(sizes_z) == 1:  # one launch for all shards
            def side(S, full):
                rows = getattr(full, "rows", None)
                src = getattr(full, "source", None)
                if rows is not None and src is not None and len(rows) >= N:
                    return (L.to_device(_as_matrix(src)),
                            L.to_device(np.stack(rows[:N]).astype(np.int64)))
                return L.to_device(np.concatenate([_as_matrix(a) for a in S])), None
            Xd, rx = side(X_s, getattr(self, "_full_x", None))
            Zd, rz = side(Z_s, getattr(self, "_full_z", None))
            out = complete_grads_device(Xd, Zd, d, rx, sizes_x.pop(), rz, sizes_z.pop(), N,
                                        wd, self.margin, self.loss)
            return [g.reshape(-1, 1) for g in out.cpu().numpy()]
        res = []  # ragged shards: one launch each
        for x, z in zip(X_s, Z_s):
            xm, zm = _as_matrix(x), _as_matrix(z)
            out = complete_grads_device(L.to_device(xm), L.to_device(zm), d, None,
                                        xm.shape[0], None, zm.shape[0], 1, wd, self.margin,
                                        self.loss)
            res.append(out.cpu().numpy()[0].reshape(-1, 1))
        return res

    def evaluate_split(self, X_s, Z_s):
        self._full_x, self._full_z = X_s, Z_s  # SWR_divide's row tables, when present
        try:
            return np.mean(self._grads(X_s, Z_s), axis=0)
        finally:
            self._full_x = self._full_z = None


def complete_grad_block(w, margin, loss=L.TW_LOSS_HINGE):
    spec = CompleteGradSpec(w, margin, loss)

    def res(X, Z):
        """
            Returns:
            1/(n_X n_Z) sum_{i,j} phi'(w^T(Z_j - X_i) + margin)(Z_j - X_i)
        """
        return spec._grads([X], [Z])[0]

    res._tw_block = spec
    return res
