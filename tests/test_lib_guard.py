"""The C-ABI binding's lifetime guard (VERDICT r05 'Next round' item 5).

Round 5's aperture violation in k_row_table_remote came from `L.ptr(L.to_device(a))` inside
one ctypes argument list: the temporary died when ptr() returned, the caching allocator handed
its block to the next temporary, and two table arguments aliased.  `_lib.ptr` now refuses an
unreferenced temporary, and `_lib.call` accepts tensors themselves and holds them until the
entry point returns.  CPU tensors stand in for device ones (the guard is allocator-agnostic).
"""
import gc
import weakref

import pytest
import torch

from tuplewise import _lib as L


def test_ptr_refuses_temporaries():
    with pytest.raises(L.TuplewiseError, match="unreferenced temporary"):
        L.ptr(torch.zeros(8))
    with pytest.raises(L.TuplewiseError, match="unreferenced temporary"):
        L.ptr(torch.zeros(8)[2:])  # a view whose base nobody else holds


def test_ptr_accepts_held_tensors():
    class Holder:
        pass

    a = torch.zeros(8)
    h = Holder()
    h.t = torch.ones(4, 4)
    rows = [torch.zeros(3), torch.zeros(5)]
    assert L.ptr(a).value == a.data_ptr()
    assert L.ptr(h.t).value == h.t.data_ptr()
    assert L.ptr(a[2:]).value == a[2:].data_ptr()  # a view of a named tensor
    assert L.ptr(h.t[1]).value == h.t[1].data_ptr()
    assert L.ptr(rows[1]).value == rows[1].data_ptr()
    assert L.ptr(a if a.numel() else None).value == a.data_ptr()
    assert L.ptr(None).value is None


def test_call_holds_tensor_arguments(monkeypatch):
    """Two temporaries in one argument list reach the entry point as distinct, live blocks."""
    seen = []

    class FakeLib:
        def tw_fake(self_, *args):  # noqa: N805
            ptrs = [a.value for a in args if hasattr(a, "value")]
            seen.append((ptrs, [r() is not None for r in refs]))
            return L.TW_OK

    refs = []

    def temp(n):
        t = torch.full((n,), 7.0)
        refs.append(weakref.ref(t))
        return t

    monkeypatch.setattr(L, "_lib", FakeLib())
    monkeypatch.setattr(L, "_TENSOR", torch.Tensor)
    fake = FakeLib()
    monkeypatch.setattr(L, "lib", lambda: fake)
    L.call("tw_fake", temp(1 << 16), 5, temp(1 << 16), None)
    ptrs, alive = seen[0]
    assert len(ptrs) == 2 and ptrs[0] != ptrs[1]
    assert alive == [True, True]  # both blocks still held while the entry point runs
    gc.collect()
    assert all(r() is None for r in refs)  # and released afterwards
