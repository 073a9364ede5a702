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

_RK_STATE_LEN = 624
_MT = {"bg": None, "ptrs": None}


def _mt_state():
    """(key, pos) pointers into the global legacy RandomState's MT19937 state — NumPy's own
    mt19937_state struct (uint32 key[624]; int pos), which the native draws then advance IN
    PLACE, with no get_state/set_state copies (~40 us a pair).  The layout is checked once
    against get_state.  None when the global generator is not an MT19937."""
    bg = getattr(np.random.mtrand._rand, "_bit_generator", None)
    if type(bg) is not np.random.MT19937:
        return None
    if _MT["bg"] is not bg:
        addr = int(bg.ctypes.state_address)
        key = np.ctypeslib.as_array((ctypes.c_uint32 * _RK_STATE_LEN).from_address(addr))
        pos = ctypes.c_int.from_address(addr + 4 * _RK_STATE_LEN)
        name, k, p = np.random.get_state(legacy=True)[:3]
        if name != "MT19937" or p != pos.value or not np.array_equal(k, key):
            return None
        _MT.update(bg=bg, ptrs=(ctypes.c_void_p(addr),
                                ctypes.c_void_p(addr + 4 * _RK_STATE_LEN)))
    return _MT["ptrs"]


class _CopiedState:
    """get_state/set_state around a native call: the fallback when _mt_state() is None."""

    def __init__(self):
        name, key, pos, self.has_gauss, self.gauss = np.random.get_state(legacy=True)
        if name != "MT19937":
            raise NotImplementedError("only the MT19937 legacy RandomState is supported")
        self.key = np.ascontiguousarray(key, dtype=np.uint32).copy()
        self.pos = ctypes.c_int32(int(pos))

    def ptrs(self):
        return ctypes.c_void_p(self.key.ctypes.data), ctypes.byref(self.pos)

    def commit(self):
        np.random.set_state(("MT19937", self.key, self.pos.value, self.has_gauss, self.gauss))


def _native_draws(fn):
    """Run fn(key_ptr, pos_ptr) on the global MT19937 state (in place when possible) and
    return its status; the state is committed even on error (NumPy would have consumed the
    draws made before the failing call)."""
    ptrs = _mt_state()
    if ptrs is not None:
        return fn(*ptrs)
    st = _CopiedState()
    rc = fn(*st.ptrs())
    st.commit()
    return rc


def randint_batch(calls) -> list:
    """[np.random.randint(lo, hi, n) for lo, hi, n in calls], one native call."""
    calls = list(calls)
    if not calls:
        return []
    low = np.array([c[0] for c in calls], dtype=np.int64)
    high = np.array([c[1] for c in calls], dtype=np.int64)
    cnt = np.array([int(c[2]) for c in calls], dtype=np.int64)
    out = np.empty(int(cnt.sum()), dtype=np.int64)
    rc = _native_draws(lambda key, pos: L.lib().tw_np_randint_batch(
        key, pos, len(calls), low.ctypes.data, high.ctypes.data, cnt.ctypes.data,
        out.ctypes.data))
    if rc:
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
    # aliasing X and Z (the same array or overlapping views): the second shuffle must see the
    # first one's swaps, which the concurrent native path does not give
    if ix is None or iz is None or np.shares_memory(X, Z) or (
            _mt_state() is None and np.random.get_state(legacy=True)[0] != "MT19937"):
        np.random.shuffle(X)
        np.random.shuffle(Z)
        return
    jbuf = np.empty(ix[0] + iz[0], dtype=np.int64)
    rc = _native_draws(lambda key, pos: L.lib().tw_np_shuffle_pair(
        key, pos, X.ctypes.data, ix[0], ix[1], Z.ctypes.data, iz[0], iz[1], jbuf.ctypes.data))
    if rc:
        raise RuntimeError(f"tw_np_shuffle_pair failed ({rc})")


def shuffle_draws32(n: int, out=None) -> np.ndarray:
    """The index draws np.random.shuffle makes on n items (n <= 2^31), without the swaps: a
    uint32 array j with j[i] for i = n-1 down to 1 (j[0] = 0), the global legacy state advanced
    exactly as the shuffle would advance it (the host half of _engine.DeviceShuffles).
    out: a C-contiguous 4-byte array of n entries to draw into (e.g. pinned memory)."""
    if out is None:
        j = np.zeros(max(int(n), 0), dtype=np.uint32)
    else:
        j = out.view(np.uint32)
        if j.shape != (max(int(n), 0),) or not j.flags.c_contiguous:
            raise ValueError("shuffle_draws32: out must be a contiguous array of n 4-byte items")
        if n > 0:
            j[0] = 0
    rc = _native_draws(lambda key, pos: L.lib().tw_np_shuffle_draws32(key, pos, int(n),
                                                                       j.ctypes.data))
    if rc:
        raise ValueError(f"tw_np_shuffle_draws32 failed ({rc}) for n = {n}")
    return j


def shuffle_draws32_range(n: int, hi: int, lo: int, out) -> None:
    """shuffle_draws32's draws for i = hi down to lo only (1 <= lo <= hi < n), into out (the
    shuffle's whole n-entry 4-byte array; other entries untouched), the global legacy state
    advanced past them: consecutive ranges from hi = n - 1 down to lo = 1 make exactly
    shuffle_draws32(n)'s draws (_engine.DeviceShuffles streams the drop-in's last shuffle)."""
    j = out.view(np.uint32)
    if j.shape != (int(n),) or not j.flags.c_contiguous:
        raise ValueError("shuffle_draws32_range: out must be a contiguous array of n items")
    rc = _native_draws(lambda key, pos: L.lib().tw_np_shuffle_draws32_range(
        key, pos, int(n), int(hi), int(lo), j.ctypes.data))
    if rc:
        raise ValueError(f"tw_np_shuffle_draws32_range failed ({rc}) for n={n}, [{lo}, {hi}]")


class Session:
    """NumPy's legacy global MT19937 state held in native code for a run of draws.

    The draws advance NumPy's own MT19937 state in place (_mt_state), so foreign draws between
    them need nothing; where that is unavailable the session holds a copy, nothing else may
    draw from np.random while it is open, commit() writes it back (and is called on exit) and
    acquire() re-reads it after foreign draws.  Every draw equals the corresponding
    np.random.randint call bit for bit."""

    def __init__(self):
        self.acquire()

    def acquire(self):
        ptrs = _mt_state()
        self._copy = None if ptrs is not None else _CopiedState()
        self._key, self._pos = ptrs if ptrs is not None else self._copy.ptrs()

    def commit(self):
        if self._copy is not None:
            self._copy.commit()

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
        rc = L.lib().tw_np_randint_batch(self._key, self._pos, len(cnt), low.ctypes.data,
                                         high.ctypes.data, cnt.ctypes.data, out.ctypes.data)
        if rc:
            raise ValueError("high <= low")
        return out

    def pairs(self, N, kx, kz, B, ix, iz):
        """grad_inc_block's draws of all N shards into int64 arrays ix, iz of shape (N, B)."""
        assert ix.flags.c_contiguous and iz.flags.c_contiguous
        rc = L.lib().tw_np_randint_pairs(self._key, self._pos, int(N), int(kx), int(kz),
                                         int(B), ix.ctypes.data, iz.ctypes.data)
        if rc:
            raise ValueError("high <= low")

    def pairs_steps_u16(self, S, N, kx, kz, B, out):
        """pairs_steps into a uint16 array (kx, kz <= 65536): the same indices, narrowed."""
        assert out.flags.c_contiguous and out.shape[0] >= S
        assert out.shape[1:] == (2, N, B) and out.dtype == np.uint16
        rc = L.lib().tw_np_randint_pairs_steps_u16(self._key, self._pos, int(S), int(N),
                                                   int(kx), int(kz), int(B), out.ctypes.data)
        if rc:
            raise ValueError("high <= low or an index range beyond 65536")

    def pairs_steps_u8(self, S, N, kx, kz, B, out):
        """pairs_steps into a uint8 array (kx, kz <= 256): the same indices, narrowed."""
        assert out.flags.c_contiguous and out.shape[0] >= S
        assert out.shape[1:] == (2, N, B) and out.dtype == np.uint8
        rc = L.lib().tw_np_randint_pairs_steps_u8(self._key, self._pos, int(S), int(N),
                                                  int(kx), int(kz), int(B), out.ctypes.data)
        if rc:
            raise ValueError("high <= low or an index range beyond 256")

    def pairs_steps(self, S, N, kx, kz, B, out):
        """S consecutive steps of grad_inc_block's draws: out[s, 0] and out[s, 1] ((N, B)
        int64 each) receive step s's X and Z indices, in the reference's draw order."""
        assert out.flags.c_contiguous and out.shape[0] >= S
        assert out.shape[1:] == (2, N, B) and out.dtype == np.int64
        rc = L.lib().tw_np_randint_pairs_steps(self._key, self._pos, int(S), int(N), int(kx),
                                               int(kz), int(B), out.ctypes.data)
        if rc:
            raise ValueError("high <= low")
