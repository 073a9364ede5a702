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
    return np.split(out, np.cumsum(cnt)[:-1])
