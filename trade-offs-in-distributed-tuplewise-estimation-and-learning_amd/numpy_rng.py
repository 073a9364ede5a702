"""Bulk replay of NumPy's legacy global RNG through libtuplewise.so (tw_np_randint_batch).

randint_batch([(low, high, size), ...]) returns exactly what the same sequence of
np.random.randint(low, high, size) calls would return, and leaves np.random in exactly the
state those calls would leave it — in one native call instead of one Python call each.
Only the MT19937-backed legacy global RandomState is supported (what the reference uses).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def randint_batch(calls) -> list:
    """[np.random.randint(lo, hi, n) for lo, hi, n in calls], one native call."""
    calls = list(calls)
    if not calls:
        return []
    name, key, pos, has_gauss, gauss = np.random.get_state(legacy=True)
    if name != "MT19937":
        raise NotImplementedError("only the MT19937 legacy RandomState is supported")
    key = np.ascontiguousarray(key, dtype=np.uint32).copy()
    pos_c = ctypes.c_int32(int(pos))
    low = np.array([c[0] for c in calls], dtype=np.int64)
    high = np.array([c[1] for c in calls], dtype=np.int64)
    cnt = np.array([int(c[2]) for c in calls], dtype=np.int64)
    out = np.empty(int(cnt.sum()), dtype=np.int64)
    rc = L.lib().tw_np_randint_batch(key.ctypes.data, ctypes.byref(pos_c), len(calls),
                                     low.ctypes.data, high.ctypes.data, cnt.ctypes.data,
                                     out.ctypes.data)
    bad = rc != 0
    # commit the advanced state (even on error: NumPy has consumed the earlier calls' draws)
    np.random.set_state((name, key, pos_c.value, has_gauss, gauss))
    if bad:
        raise ValueError("high <= low")
    offs = np.concatenate([[0], np.cumsum(cnt)])
    return [out[offs[i]:offs[i + 1]] for i in range(len(cnt))]


def _shuffle_items(a):
    """(items, item bytes) when np.random.shuffle(a) is the buffer path this module restates:
    a C-contiguous, non-object ndarray (rows of a 2-D array are items); else None."""
    if not isinstance(a, np.ndarray) or a.ndim == 0 or a.dtype.hasobject:
        return None
    if not a.flags.c_contiguous or a.size == 0:
        return None
    return a.shape[0], a.itemsize * (a.size // a.shape[0])


def shuffle_pair(X, Z) -> None:
    """np.random.shuffle(X); np.random.shuffle(Z) (compute_stats.py:66-67, estimation-experiment/
    main.py:46-47): the same index draws from the same legacy MT19937 stream, the same swaps,
    the same final RNG state — the swaps of X on a second native thread while Z's draws and
    swaps run.  Arrays the buffer path does not cover (views, object arrays, other RNGs) go
    to np.random.shuffle itself."""
    ix, iz = _shuffle_items(X), _shuffle_items(Z)
    state = np.random.get_state(legacy=True)
    if ix is None or iz is None or state[0] != "MT19937":
        np.random.shuffle(X)
        np.random.shuffle(Z)
        return
    name, key, pos, has_gauss, gauss = state
    key = np.ascontiguousarray(key, dtype=np.uint32).copy()
    pos_c = ctypes.c_int32(int(pos))
    jbuf = np.empty(ix[0] + iz[0], dtype=np.int64)
    rc = L.lib().tw_np_shuffle_pair(key.ctypes.data, ctypes.byref(pos_c), X.ctypes.data,
                                    ix[0], ix[1], Z.ctypes.data, iz[0], iz[1],
                                    jbuf.ctypes.data)
    if rc:
        raise RuntimeError(f"tw_np_shuffle_pair failed ({rc})")
    np.random.set_state((name, key, pos_c.value, has_gauss, gauss))


def shuffle_draws32(n: int, out=None) -> np.ndarray:
    """The index draws np.random.shuffle makes on n items (n <= 2^31), without the swaps: a
    uint32 array j with j[i] for i = n-1 down to 1 (j[0] = 0), the global legacy state advanced
    exactly as the shuffle would advance it (the host half of _engine.DeviceShuffles).
    out: a C-contiguous 4-byte array of n entries to draw into (e.g. pinned memory)."""
    name, key, pos, has_gauss, gauss = np.random.get_state(legacy=True)
    if name != "MT19937":
        raise ValueError("shuffle_draws32 restates the legacy MT19937 RandomState only")
    key = np.ascontiguousarray(key, dtype=np.uint32).copy()
    pos_c = ctypes.c_int32(int(pos))
    if out is None:
        j = np.zeros(max(int(n), 0), dtype=np.uint32)
    else:
        j = out.view(np.uint32)
        if j.shape != (max(int(n), 0),) or not j.flags.c_contiguous:
            raise ValueError("shuffle_draws32: out must be a contiguous array of n 4-byte items")
        if n > 0:
            j[0] = 0
    rc = L.lib().tw_np_shuffle_draws32(key.ctypes.data, ctypes.byref(pos_c), int(n),
                                       j.ctypes.data)
    if rc:
        raise ValueError(f"tw_np_shuffle_draws32 failed ({rc}) for n = {n}")
    np.random.set_state((name, key, pos_c.value, has_gauss, gauss))
    return j


class Session:
    """NumPy's legacy global MT19937 state held in native code for a run of draws.

    While a session is open nothing else may draw from np.random; commit() writes the
    advanced state back (and is called on exit).  acquire() re-reads it after foreign draws.
    Every draw equals the corresponding np.random.randint call bit for bit."""

    def __init__(self):
        self.acquire()

    def acquire(self):
        name, key, pos, self._has_gauss, self._gauss = np.random.get_state(legacy=True)
        if name != "MT19937":
            raise NotImplementedError("only the MT19937 legacy RandomState is supported")
        self._key = np.ascontiguousarray(key, dtype=np.uint32).copy()
        self._pos = ctypes.c_int32(int(pos))

    def commit(self):
        np.random.set_state(("MT19937", self._key, self._pos.value, self._has_gauss,
                             self._gauss))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.commit()
        return False

    def randint_flat(self, low, high, cnt, out=None) -> np.ndarray:
        """Consecutive randint(low[c], high[c], cnt[c]) calls, concatenated."""
        low = np.ascontiguousarray(low, dtype=np.int64)
        high = np.ascontiguousarray(high, dtype=np.int64)
        cnt = np.ascontiguousarray(cnt, dtype=np.int64)
        if out is None:
            out = np.empty(int(cnt.sum()), dtype=np.int64)
        rc = L.lib().tw_np_randint_batch(self._key.ctypes.data, ctypes.byref(self._pos),
                                         len(cnt), low.ctypes.data, high.ctypes.data,
                                         cnt.ctypes.data, out.ctypes.data)
        if rc:
            raise ValueError("high <= low")
        return out

    def pairs(self, N, kx, kz, B, ix, iz):
        """grad_inc_block's draws of all N shards into int64 arrays ix, iz of shape (N, B)."""
        assert ix.flags.c_contiguous and iz.flags.c_contiguous
        rc = L.lib().tw_np_randint_pairs(self._key.ctypes.data, ctypes.byref(self._pos),
                                         int(N), int(kx), int(kz), int(B), ix.ctypes.data,
                                         iz.ctypes.data)
        if rc:
            raise ValueError("high <= low")

    def pairs_steps(self, S, N, kx, kz, B, out):
        """S consecutive steps of grad_inc_block's draws: out[s, 0] and out[s, 1] ((N, B)
        int64 each) receive step s's X and Z indices, in the reference's draw order."""
        assert out.flags.c_contiguous and out.shape[0] >= S
        lib = L.lib()
        key, pos = self._key.ctypes.data, ctypes.byref(self._pos)
        for st in range(S):
            rc = lib.tw_np_randint_pairs(key, pos, int(N), int(kx), int(kz), int(B),
                                         out[st, 0].ctypes.data, out[st, 1].ctypes.data)
            if rc:
                raise ValueError("high <= low")
