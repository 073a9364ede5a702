"""Device dispatch for the tuplewise hot path.

Host side of the drop-in API: it turns NumPy inputs into device tensors (PyTorch-ROCm is used
only for allocation, copies and the stream), describes shards by offset arrays, and calls the
C ABI of libtuplewise.so (include/tuplewise.h).  All pair arithmetic happens in the HIP
kernels; this file only does bookkeeping, NumPy dtype promotion and the final exact division.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L

# ----------------------------------------------------------------------------- dtype rules
_INT64_MIN = np.int64(-(2 ** 63))


def compare_operands(X: np.ndarray, Z: np.ndarray):
    """Operands of NumPy's `X > Z` as (x, z, dtype code) with identical ordering.

    NumPy compares in np.result_type(X, Z): float kinds compare as float64 (exact for every
    float input), signed/bool integers as int64, uint64 vs uint64 as unsigned (mapped to int64
    keys by flipping the sign bit, an order isomorphism), uint64 vs signed as float64.
    """
    X = np.asarray(X)
    Z = np.asarray(Z)
    rt = np.result_type(X.dtype, Z.dtype)
    if rt.kind == "f":
        return X.astype(np.float64, copy=False), Z.astype(np.float64, copy=False), L.TW_F64
    if rt.kind in "bi":
        return X.astype(np.int64, copy=False), Z.astype(np.int64, copy=False), L.TW_I64
    if rt.kind == "u":  # both unsigned
        xk = X.astype(np.uint64, copy=False).view(np.int64) ^ _INT64_MIN
        zk = Z.astype(np.uint64, copy=False).view(np.int64) ^ _INT64_MIN
        return xk, zk, L.TW_I64
    raise TypeError(f"unsupported dtypes for a pair comparison: {X.dtype}, {Z.dtype}")


def subtract_gt_operands(X: np.ndarray, Z: np.ndarray):
    """Operands + predicate for cs.Un's literal `(X - Z) > 0` (compute_stats.py:19, :30).

    Returns (x, z, dtype code, mode) with mode in {"gt", "subgt", "ne"}:
      float result  -> `x > z` (identical for IEEE doubles)
      int64 result  -> wrapping int64 subtraction then `> 0`             ("subgt")
      narrower signed ints that cannot wrap -> `x > z`
      unsigned result -> (x - z) wraps to >= 0, so `> 0` means `x != z`  ("ne")
      bool          -> NumPy raises TypeError for boolean subtract; so do we.
    """
    X = np.asarray(X)
    Z = np.asarray(Z)
    if X.dtype == np.bool_ and Z.dtype == np.bool_:
        raise TypeError("numpy boolean subtract, the `-` operator, is not supported")
    rt = np.result_type(X.dtype, Z.dtype)
    if rt.kind == "f":
        return X.astype(np.float64, copy=False), Z.astype(np.float64, copy=False), L.TW_F64, "gt"
    if rt.kind == "u":
        x, z, code = compare_operands(X, Z)
        return x, z, code, "ne"
    if rt.kind == "i":
        x = X.astype(np.int64, copy=False)
        z = Z.astype(np.int64, copy=False)
        if rt.itemsize == 8:
            if x.size and z.size:  # no wrap possible -> plain ordered comparison
                lo = int(x.min()) - int(z.max())
                hi = int(x.max()) - int(z.min())
                if -(2 ** 63) <= lo and hi <= 2 ** 63 - 1:
                    return x, z, L.TW_I64, "gt"
            return x, z, L.TW_I64, "subgt"
        info = np.iinfo(rt)
        lo = int(x.min()) - int(z.max()) if x.size and z.size else 0
        hi = int(x.max()) - int(z.min()) if x.size and z.size else 0
        if info.min <= lo and hi <= info.max:
            return x, z, L.TW_I64, "gt"
        raise NotImplementedError(
            f"(X - Z) > 0 wraps in {rt}; only int64 wrap-around is reproduced on the device")
    raise TypeError(f"unsupported dtypes for X - Z: {X.dtype}, {Z.dtype}")


# ----------------------------------------------------------------------------- shard layout
class Shards:
    """Concatenated shard data on the device + host-side offsets.

    x_off/z_off are int64 host arrays of length n_shards+1; shard s owns x[x_off[s]:x_off[s+1]].
    """

    def __init__(self, x_dev, x_off: np.ndarray, z_dev, z_off: np.ndarray, dtype_code: int):
        self.x = x_dev
        self.z = z_dev
        self.x_off = np.asarray(x_off, dtype=np.int64)
        self.z_off = np.asarray(z_off, dtype=np.int64)
        self.dtype = dtype_code
        self.n_shards = len(self.x_off) - 1
        self._x_off_dev = None
        self._z_off_dev = None

    @property
    def nx(self) -> np.ndarray:
        return np.diff(self.x_off)

    @property
    def nz(self) -> np.ndarray:
        return np.diff(self.z_off)

    def offsets_dev(self):
        if self._x_off_dev is None:
            self._x_off_dev = L.to_device(self.x_off)
            self._z_off_dev = L.to_device(self.z_off)
        return self._x_off_dev, self._z_off_dev

    @classmethod
    def from_host(cls, x: np.ndarray, x_off, z: np.ndarray, z_off, dtype_code: int):
        return cls(L.to_device(x), x_off, L.to_device(z), z_off, dtype_code)

    @classmethod
    def from_blocks(cls, xs, zs, dtype_code: int):
        xs = [np.asarray(a).reshape(-1) for a in xs]
        zs = [np.asarray(a).reshape(-1) for a in zs]
        x_off = np.concatenate([[0], np.cumsum([len(a) for a in xs])]).astype(np.int64)
        z_off = np.concatenate([[0], np.cumsum([len(a) for a in zs])]).astype(np.int64)
        x = np.concatenate(xs) if xs else np.zeros(0)
        z = np.concatenate(zs) if zs else np.zeros(0)
        return cls.from_host(x, x_off, z, z_off, dtype_code)


def _counts_to_host(out) -> np.ndarray:
    return out.cpu().numpy().view(np.uint64)


SORTED_MIN_PAIRS = 1 << 22  # "auto": per-shard pair count above which sort+search wins


def pick_algo(algo: str, max_nx: int, max_nz: int, mode: str) -> str:
    if algo == "auto":
        return "sorted" if (mode in ("gt", "half", "ne")
                            and max_nx * max_nz >= SORTED_MIN_PAIRS) else "pairs"
    if algo not in ("pairs", "sorted"):
        raise ValueError(f"algo must be 'auto', 'pairs' or 'sorted', not {algo!r}")
    if algo == "sorted" and mode == "subgt":
        raise ValueError("algo='sorted' needs an ordered predicate (no int64 wrap-around)")
    return algo


# one element of the sorted count (LDS buckets / sort + search, csrc/rankcount.hip) costs about
# as much device time as 750 compares of the all-pairs kernel (measured at the C3 shape:
# 2e6 elements in ~45 us against 3.3e13 compared pairs/s)
SORTED_ELEMENT_COST = 750


def count_work(nx: int, nz: int, mode: str) -> int:
    """Device work of one block's count in all-pairs compare equivalents, for the algorithm
    'auto' picks: nx*nz compares, or (nx + nz) sorted-element steps."""
    if pick_algo("auto", nx, nz, mode) == "sorted":
        return (nx + nz) * SORTED_ELEMENT_COST
    return nx * nz


def count_launch(x_dev, x_off_dev, z_dev, z_off_dev, n, max_nx, max_nz, dtype, pred, algo):
    """Enqueue one count of all shards (no host sync); returns the int64 device tensor."""
    t = L.torch()
    out = L.empty((n,), t.int64)
    if algo == "sorted":
        work = L.empty((int(L.lib().tw_count_pairs_sorted_work_bytes(n, max_nz)),), t.uint8)
        L.call("tw_count_pairs_sorted", L.ptr(x_dev), L.ptr(x_off_dev), L.ptr(z_dev),
               L.ptr(z_off_dev), n, max_nx, max_nz, dtype, pred, L.ptr(work), L.ptr(out),
               L.stream_handle())
    else:
        L.call("tw_count_pairs", L.ptr(x_dev), L.ptr(x_off_dev), L.ptr(z_dev), L.ptr(z_off_dev),
               n, max_nx, max_nz, dtype, pred, L.ptr(out), L.stream_handle())
    return out


def count_complete(sh: Shards, mode: str = "gt", algo: str = "auto") -> np.ndarray:
    """Per-shard exact counts (uint64) of the predicate over all pairs of each shard.

    mode: "gt" (#x>z), "half" (2#x>z + #x==z), "subgt" (#(x-z)>0 with int64 wrap),
    "ne" (#x!=z, derived on the device from the half and gt counts).
    algo: "pairs" (all-pairs VALU kernel), "sorted" (sort + binary search), "auto"."""
    n = sh.n_shards
    if n == 0:
        return np.zeros(0, dtype=np.uint64)
    xo, zo = sh.offsets_dev()
    max_nx = int(sh.nx.max())
    max_nz = int(sh.nz.max())
    algo = pick_algo(algo, max_nx, max_nz, mode)

    def run(pred):
        return count_launch(sh.x, xo, sh.z, zo, n, max_nx, max_nz, sh.dtype, pred, algo)

    if mode == "ne":
        half = _counts_to_host(run(L.TW_PRED_HALF)).astype(object)
        gt = _counts_to_host(run(L.TW_PRED_GT)).astype(object)
        pairs = (sh.nx.astype(object) * sh.nz.astype(object))
        return np.array(pairs - (half - 2 * gt), dtype=np.uint64)
    pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF, "subgt": L.TW_PRED_SUBGT}[mode]
    return _counts_to_host(run(pred))


_I32_LIMIT = 2 ** 31  # arrays up to this many elements take int32 pair indices


def _idx_dev(a, bound=None):
    """Pair-index array on the device.  Device tensors pass through (callers cache them);
    host arrays go up as int32 when every valid index fits (bound = the indexed array's
    length, <= 2^31; the indices were bound-checked or drawn in range by the caller), which is
    the 8 B/pair replay contract and halves the upload, else as int64."""
    t = L.torch()
    if isinstance(a, t.Tensor):
        return a
    a = np.asarray(a)
    if bound is not None and bound <= _I32_LIMIT:
        return L.to_device(a, np.int32)
    return L.to_device(a, np.int64)


def _idx_pair(ix, iz, bx=None, bz=None):
    """(ixd, izd) of one index width: int32 when both fit, else both int64."""
    t = L.torch()
    ixd, izd = _idx_dev(ix, bx), _idx_dev(iz, bz)
    if ixd.dtype != izd.dtype:
        ixd, izd = ixd.to(t.int64), izd.to(t.int64)
    if ixd.dtype not in (t.int32, t.int64):
        raise TypeError(f"pair indices must be int32 or int64, not {ixd.dtype}")
    return ixd, izd


def _off_dev(pair_off, pair_off_dev):
    return pair_off_dev if pair_off_dev is not None else L.to_device(
        np.asarray(pair_off, dtype=np.int64))


def count_indexed_dev(x_dev, z_dev, dtype_code: int, ix, iz, pair_off: np.ndarray, pred: int,
                      pair_off_dev=None):
    """Per-shard counts over index pairs gathered from the scores (no shard spans), enqueued
    only: the (n_shards,) int64 device tensor (uint64 semantics)."""
    t = L.torch()
    n = len(pair_off) - 1
    ixd, izd = _idx_pair(ix, iz, x_dev.numel(), z_dev.numel())
    pod = _off_dev(pair_off, pair_off_dev)
    max_pairs = int(np.diff(pair_off).max()) if n else 0
    out = L.empty((max(n, 1),), t.int64)[:n]
    name = "tw_count_pairs_idx32" if ixd.dtype == t.int32 else "tw_count_pairs_idx"
    L.call(name, L.ptr(x_dev), L.ptr(z_dev), L.ptr(ixd), L.ptr(izd), L.ptr(pod), n, max_pairs,
           dtype_code, pred, L.ptr(out), L.stream_handle())
    return out


def count_indexed_ranked_dev(x_dev, x_off_dev, z_dev, z_off_dev, max_nx: int, max_nz: int,
                             dtype_code: int, ix, iz, pair_off: np.ndarray, pred: int,
                             pair_off_dev=None, work=None):
    """count_indexed_dev for shard-contiguous samples (shard s = x[x_off[s]:x_off[s+1]]): the
    same integers, compared on 16-bit rank codes in LDS (tw_count_pairs_idx(32)_ws; it runs the
    plain kernel where codes do not apply).  `work` may be a cached uint8 device buffer of
    tw_count_pairs_rng_work_bytes bytes."""
    t = L.torch()
    n = len(pair_off) - 1
    ixd, izd = _idx_pair(ix, iz, x_dev.numel(), z_dev.numel())
    pod = _off_dev(pair_off, pair_off_dev)
    max_pairs = int(np.diff(pair_off).max()) if n else 0
    wpred = L.TW_PRED_GT if (pred == L.TW_PRED_SUBGT and dtype_code == L.TW_F64) else pred
    wb = int(L.lib().tw_count_pairs_rng_work_bytes(n, max_nx, max_nz, dtype_code, wpred))
    if wb > 0 and (work is None or work.numel() < wb):
        work = L.empty((wb,), t.uint8)
    out = L.empty((max(n, 1),), t.int64)[:n]
    name = "tw_count_pairs_idx32_ws" if ixd.dtype == t.int32 else "tw_count_pairs_idx_ws"
    L.call(name, L.ptr(x_dev), L.ptr(x_off_dev), L.ptr(z_dev), L.ptr(z_off_dev), n, max_nx,
           max_nz, L.ptr(ixd), L.ptr(izd), L.ptr(pod), max_pairs, dtype_code, pred,
           L.ptr(work if wb > 0 else None), wb, L.ptr(out), L.stream_handle())
    return out


def count_indexed(x_dev, z_dev, dtype_code: int, ix, iz, pair_off: np.ndarray,
                  mode: str = "gt", pair_off_dev=None, spans=None) -> np.ndarray:
    """Per-shard counts over explicit (absolute) index pairs (host or device index arrays).
    spans = (x_off, z_off): shard s draws (mostly) from x[x_off[s]:x_off[s+1]] and
    z[z_off[s]:z_off[s+1]]; the counts then run on LDS rank codes (count_indexed_ranked_dev),
    the same integers for any indices.  Without spans the pairs gather the scores."""
    n = len(pair_off) - 1
    if n == 0:
        return np.zeros(0, dtype=np.uint64)
    ixd, izd = _idx_pair(ix, iz, x_dev.numel(), z_dev.numel())
    pod = _off_dev(pair_off, pair_off_dev)
    if spans is not None:
        xo, zo = (np.asarray(a, dtype=np.int64) for a in spans)
        xod, zod = L.to_device(xo), L.to_device(zo)
        mx, mz = int(np.diff(xo).max()), int(np.diff(zo).max())

    def run(pred):
        if spans is not None:
            return _counts_to_host(count_indexed_ranked_dev(x_dev, xod, z_dev, zod, mx, mz,
                                                            dtype_code, ixd, izd, pair_off,
                                                            pred, pod))
        return _counts_to_host(count_indexed_dev(x_dev, z_dev, dtype_code, ixd, izd, pair_off,
                                                 pred, pod))

    if mode == "ne":
        half = run(L.TW_PRED_HALF).astype(object)
        gt = run(L.TW_PRED_GT).astype(object)
        pairs = np.diff(pair_off).astype(object)
        return np.array(pairs - (half - 2 * gt), dtype=np.uint64)
    pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF, "subgt": L.TW_PRED_SUBGT}[mode]
    return run(pred)


def pair_sum_complete(sh: Shards, kern: int, margin: float = 0.0) -> np.ndarray:
    """Per-shard float64 sums of kern(x_i, z_j) over all pairs."""
    if sh.n_shards == 0:
        return np.zeros(0)
    return pair_sum_complete_dev(sh, kern, margin).cpu().numpy()


_SH_STREAMS = {}  # per device: the X and Z shuffle streams of DeviceShuffles
_SIDE_STREAMS = {}  # (device, name) -> a stream of the drop-in's own (counts, write-backs)


class _Launcher:
    """A worker thread per device that runs the drop-in's enqueue work (the draws' uploads, the
    swap rounds' launches, the per-step counts) in submission order, so the host thread making
    the draws (native code, GIL released) never waits for a launch: each shuffle enqueues ~20
    kernels, ~0.1 ms of host time, and the draws are the call's critical path."""

    def __init__(self, dev):
        import queue
        import threading
        self.q = queue.Queue()
        self.err = None
        self.dev = dev
        threading.Thread(target=self._loop, daemon=True).start()

    def _loop(self):
        L.torch().cuda.set_device(self.dev)
        while True:
            fn = self.q.get()
            try:
                if self.err is None:
                    fn()
            except BaseException as e:  # raised to the submitting thread at drain()
                self.err = e
            finally:
                self.q.task_done()

    def submit(self, fn) -> None:
        self.q.put(fn)

    def drain(self) -> None:
        """Wait until every submitted task has run; re-raise the first failure."""
        self.q.join()
        if self.err is not None:
            e, self.err = self.err, None
            raise e


_LAUNCHERS = {}


def launcher(dev, name: str = "launch") -> _Launcher:
    """The device's worker thread of that name (made once)."""
    if (dev, name) not in _LAUNCHERS:
        _LAUNCHERS[(dev, name)] = _Launcher(dev)
    return _LAUNCHERS[(dev, name)]


def side_stream(name: str):
    """A named side stream of the current device, made once (torch.cuda.Stream)."""
    t = L.torch()
    key = (t.cuda.current_device(), name)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = t.cuda.Stream()
    return _SIDE_STREAMS[key]

_SH_BUFFERS = {}  # (device, nx, nz, T, dtype) -> the buffers of the last reuse=True instance


class DeviceShuffles:
    """T successive np.random.shuffle's of two arrays of 8-byte items, every state kept on the
    device: xs[k] = x0 after the swaps of shuffles 0..k (likewise zs).  The host draws each
    shuffle's indices in NumPy's order (numpy_rng.shuffle_draws32) straight into pinned buffers
    (draw_x, draw_z); push_x() / push_z() upload them asynchronously and enqueue that side's
    swap rounds (csrc/devshuffle.hip: the sequential loop's permutation, bit for bit) on the
    side's own stream, so X's shuffle k runs while the host draws Z's, and Z's while the host
    draws X's shuffle k+1 — the last shuffle on the critical path is Z's alone (round 5: the two
    sides shared every launch before, and the last pair ran after the last draw).
    x0 / z0: device tensors, or host arrays (1-D float64) uploaded by a helper thread while the
    host makes the first draws.  finish() reads the pending counts (one sync); a side whose
    batch of rounds did not finish (rare) is resumed and its later shuffles are redone.
    reuse=True (the drop-in's own calls, whose snapshots die with the call): the pinned draw
    buffers, snapshots and workspaces of the previous call of the same shape are used again
    (their allocation was ~0.35 ms of a 7-ms call).
    Returns the (T, nx) and (T, nz) device tensors."""

    def __init__(self, x0, z0, T: int, reuse: bool = False, threaded: bool = False):
        import threading
        t = L.torch()
        lib = L.lib()
        self.t = t
        self.T = T
        host = not isinstance(x0, t.Tensor)
        self.nx = int(np.asarray(x0).size if host else x0.numel())
        self.nz = int(np.asarray(z0).size if host else z0.numel())
        dev = t.cuda.current_device()
        dt = t.float64 if host else x0.dtype
        key = (dev, self.nx, self.nz, T, dt)
        buf = _SH_BUFFERS.get(key) if reuse else None
        if dev not in _SH_STREAMS:
            _SH_STREAMS[dev] = (t.cuda.Stream(), t.cuda.Stream())
        self.sx, self.sz = _SH_STREAMS[dev]
        main = t.cuda.current_stream()
        self.sx.wait_stream(main)
        self.sz.wait_stream(main)
        self._up = None
        if host:
            self.x0 = buf["x0"] if buf else L.empty((self.nx,), t.float64)
            self.z0 = buf["z0"] if buf else L.empty((self.nz,), t.float64)

            def upload():  # pageable H2D copies, GIL released; the streams order the shuffles
                with t.cuda.device(dev):
                    with t.cuda.stream(self.sx):
                        self.x0.copy_(t.from_numpy(np.ascontiguousarray(x0).reshape(-1)))
                    with t.cuda.stream(self.sz):
                        self.z0.copy_(t.from_numpy(np.ascontiguousarray(z0).reshape(-1)))
            if threaded:  # the launcher's first task: before every push, beside the draws
                launcher(dev).submit(upload)
            else:
                self._up = threading.Thread(target=upload)
                self._up.start()
        else:
            assert x0.element_size() == 8 and z0.element_size() == 8
            self.x0, self.z0 = x0.reshape(-1), z0.reshape(-1)
        self.rounds = (int(lib.tw_shuffle_swaps_rounds(self.nx, 0)),
                       int(lib.tw_shuffle_swaps_rounds(0, self.nz)))
        if buf is None:
            nbx = max(int(lib.tw_shuffle_swaps_work_bytes(self.nx, 0)), 1)
            nbz = max(int(lib.tw_shuffle_swaps_work_bytes(0, self.nz)), 1)
            buf = {"xs": L.empty((T, self.nx), dt), "zs": L.empty((T, self.nz), dt),
                   "hx": t.empty((T, self.nx), dtype=t.int32, pin_memory=True),
                   "hz": t.empty((T, self.nz), dtype=t.int32, pin_memory=True),
                   "jx": L.empty((T, self.nx), t.int32), "jz": L.empty((T, self.nz), t.int32),
                   "work": (L.empty((T, nbx), t.uint8), L.empty((T, nbz), t.uint8)),
                   "pend": L.empty((2, max(T, 1)), t.int32),
                   "x0": self.x0 if host else None, "z0": self.z0 if host else None}
            if reuse:
                _SH_BUFFERS.clear()  # one shape kept: the previous shape's memory goes back
                _SH_BUFFERS[key] = buf
        self.xs, self.zs, self.hx, self.hz = buf["xs"], buf["zs"], buf["hx"], buf["hz"]
        self.jx, self.jz, self.work, self.pend = buf["jx"], buf["jz"], buf["work"], buf["pend"]
        self.kx = self.kz = 0
        # threaded: uploads and launches run on the device's launcher thread (submit), in order
        self._launcher = launcher(dev) if threaded else None

    def submit(self, fn) -> None:
        """Run fn after every push so far (on the launcher thread when threaded)."""
        if self._launcher is None:
            fn()
        else:
            self._launcher.submit(fn)

    def drain(self) -> None:
        if self._launcher is not None:
            self._launcher.drain()

    def _uploaded(self):
        if self._up is not None:
            self._up.join()
            self._up = None

    def draw_x(self):
        return self.hx[self.kx].numpy()

    def draw_z(self):
        return self.hz[self.kz].numpy()

    def push_x(self) -> None:
        k = self.kx
        self.kx += 1

        def task():
            self._uploaded()
            with self.t.cuda.stream(self.sx):
                self.jx[k].copy_(self.hx[k], non_blocking=True)
                self._start(0, k)
        self.submit(task)

    def push_z(self) -> None:
        k = self.kz
        self.kz += 1

        def task():
            self._uploaded()
            with self.t.cuda.stream(self.sz):
                self.jz[k].copy_(self.hz[k], non_blocking=True)
                self._start(1, k)
        self.submit(task)

    def push(self) -> None:
        self.push_x()
        self.push_z()

    def draw_push_z_streamed(self, pieces: int = 4) -> None:
        """Z's next shuffle drawn AND pushed in `pieces` parts (the call's last shuffle, whose
        swap rounds would otherwise all run after its last draw): the draws of a group of
        windows (tw_shuffle_swaps_windows, in the host's draw order), their upload, and the
        rounds those windows allow (tw_shuffle_swaps_part) — the device swaps the first windows
        while the host draws the next.  Same draws, same rounds, same permutation."""
        from .numpy_rng import shuffle_draws32_range
        t, k, n = self.t, self.kz, self.nz
        self.kz += 1
        hz = self.hz[k].numpy()
        W = int(L.lib().tw_shuffle_swaps_windows())
        p = -(-(n - 1) // W) if n > 1 else 0
        pieces = max(1, min(int(pieces), W))
        r0 = 0
        for q in range(pieces):
            c0, c1 = q * W // pieces, (q + 1) * W // pieces
            last = q == pieces - 1
            hi, lo = n - c0 * p - 1, max(1, n - c1 * p)
            if n > 1 and hi >= lo:
                shuffle_draws32_range(n, hi, lo, hz)
            # windows [0, c1) are up: rounds to c1 - 2 (round r reads windows <= r + 1)
            r1 = max(r0, c1 - 1) if not last else r0

            def part(q=q, hi=hi, lo=lo, r0=r0, r1=r1, last=last):
                if q == 0:
                    self._uploaded()
                with t.cuda.stream(self.sz):
                    if q == 0:
                        self.zs[k].copy_(self.z0 if k == 0 else self.zs[k - 1])
                    if n > 1 and hi >= lo:
                        self.jz[k][lo:hi + 1].copy_(self.hz[k][lo:hi + 1], non_blocking=True)
                    L.call("tw_shuffle_swaps_part", None, 0, L.ptr(self.zs[k]), n, None,
                           L.ptr(self.jz[k]), r0, r1, int(last), L.ptr(self.work[1][k]),
                           L.ptr(self.pend[1, k:k + 1]), L.stream_handle())
            self.submit(part)
            r0 = r1

    def order_after(self, stream) -> None:
        """`stream` waits for every shuffle enqueued so far (both sides; call it on the
        launcher thread, or after drain(), to include every push)."""
        stream.wait_stream(self.sx)
        stream.wait_stream(self.sz)

    def _run(self, side, k, first, round0):
        if side == 0:
            L.call("tw_shuffle_swaps", L.ptr(self.xs[k]), self.nx, None, 0, L.ptr(self.jx[k]),
                   None, int(first), round0, L.ptr(self.work[0][k]),
                   L.ptr(self.pend[0, k:k + 1]), L.stream_handle())
        else:
            L.call("tw_shuffle_swaps", None, 0, L.ptr(self.zs[k]), self.nz, None,
                   L.ptr(self.jz[k]), int(first), round0, L.ptr(self.work[1][k]),
                   L.ptr(self.pend[1, k:k + 1]), L.stream_handle())

    def _start(self, side, k):  # on the side's stream
        xs = self.xs if side == 0 else self.zs
        xs[k].copy_((self.x0 if side == 0 else self.z0) if k == 0 else xs[k - 1])
        self._run(side, k, True, 0)

    def write_back_x_async(self, x_host) -> None:
        """Copy X's last state into the host array x_host on the device's write-back thread, as
        soon as X's last shuffle has run — while this thread draws Z's last shuffle (threaded
        only; drain_write_back() waits for it)."""
        t, T = self.t, self.T
        wb = launcher(self._launcher.dev, "writeback")
        stream = side_stream("x-writeback")
        out = t.from_numpy(x_host).reshape(-1)

        def record():  # on the launcher thread, after X's last push was enqueued
            ev = t.cuda.Event()
            ev.record(self.sx)

            def copy():
                stream.wait_event(ev)
                with t.cuda.stream(stream):
                    out.copy_(self.xs[T - 1])
            wb.submit(copy)
        self.submit(record)
        self._wb = wb

    def drain_write_back(self) -> None:
        wb = getattr(self, "_wb", None)
        if wb is not None:
            self.drain()  # the record task ran, so the copy is queued
            wb.drain()
            self._wb = None

    def last_x(self):
        """The X side's last state, ordered on the current stream after its shuffles (a
        caller may copy it out while Z's last shuffle runs); finish() says whether it held."""
        self.drain()
        self.t.cuda.current_stream().wait_stream(self.sx)
        return self.xs[self.T - 1]

    def finish(self):
        """Sync on the pending counts; resume the rare unfinished side.  Returns (xs, zs) and
        leaves the current stream ordered after both sides.  self.redone: the sides whose
        states changed after a resumption."""
        T, t = self.T, self.t
        assert self.kx == T and self.kz == T, "every shuffle must be pushed before finish()"
        self.drain()
        main = t.cuda.current_stream()
        main.wait_stream(self.sx)
        main.wait_stream(self.sz)
        pend = self.pend[:, :T].cpu().numpy()
        self.redone = set()
        for side in (0, 1):
            left = np.nonzero(pend[side])[0]
            if not len(left):
                continue
            self.redone.add(side)
            k = int(left[0])
            while k < T:  # finish shuffle k, then redo the later ones one at a time
                r0 = self.rounds[side]
                while int(self.pend[side, k].item()):
                    self._run(side, k, False, r0)
                    r0 += self.rounds[side]
                k += 1
                if k < T:
                    self._start(side, k)
        return self.xs, self.zs


def shuffle_snapshots_device(x0, z0, jx, jz):
    """DeviceShuffles over draws already made (uint32 host arrays, one per shuffle)."""
    ds = DeviceShuffles(x0, z0, len(jx))
    for a, b in zip(jx, jz):
        ds.draw_x()[...] = np.asarray(a).view(np.int32)
        ds.draw_z()[...] = np.asarray(b).view(np.int32)
        ds.push()
    return ds.finish()


# hinge sums of shards with at least this many pairs use the O((n+m) log m) path
HINGE_SORTED_MIN_PAIRS = 1 << 27


def pair_sum_complete_dev(sh: Shards, kern: int, margin: float = 0.0, algo: str = "auto"):
    """pair_sum_complete, enqueued only: the (n_shards,) float64 device tensor.  The hinge
    kernel on float64 scores takes the sorted path (tw_pair_hinge_sum_sorted: top-c sums from
    double-double prefix sums of the sorted z) when a shard has >= HINGE_SORTED_MIN_PAIRS
    pairs (algo="auto") or always (algo="sorted"); algo="pairs" forces the all-pairs kernel."""
    n = sh.n_shards
    t = L.torch()
    xo, zo = sh.offsets_dev()
    max_nx, max_nz = int(sh.nx.max()), int(sh.nz.max())
    if (kern == L.TW_KERN_HINGE and sh.dtype == L.TW_F64 and algo != "pairs"
            and (algo == "sorted" or max_nx * max_nz >= HINGE_SORTED_MIN_PAIRS)):
        nb = int(L.lib().tw_pair_hinge_sum_sorted_work_bytes(n, max_nx, max_nz))
        work = L.empty((max(nb, 1),), t.uint8)
        out = L.empty((n,), t.float64)
        L.call("tw_pair_hinge_sum_sorted", L.ptr(sh.x), L.ptr(xo), L.ptr(sh.z), L.ptr(zo), n,
               max_nx, max_nz, float(margin), L.ptr(work), L.ptr(out), L.stream_handle())
        return out
    per = int(L.lib().tw_pair_sum_work_per_shard(max_nx, max_nz))
    work = L.empty((per * n,), t.float64)
    out = L.empty((n,), t.float64)
    L.call("tw_pair_sum_f64", L.ptr(sh.x), L.ptr(xo), L.ptr(sh.z), L.ptr(zo), n, max_nx, max_nz,
           kern, float(margin), L.ptr(work), L.ptr(out), L.stream_handle())
    return out


def pair_sum_indexed(x_dev, z_dev, ix, iz, pair_off, kern: int, margin: float = 0.0,
                     pair_off_dev=None):
    if len(pair_off) - 1 == 0:
        return np.zeros(0)
    return pair_sum_indexed_dev(x_dev, z_dev, ix, iz, pair_off, kern, margin,
                                pair_off_dev).cpu().numpy()


def pair_sum_indexed_dev(x_dev, z_dev, ix, iz, pair_off, kern: int, margin: float = 0.0,
                         pair_off_dev=None, count_out=None):
    """pair_sum_indexed, enqueued only: the (n_shards,) float64 device tensor.  count_out
    (int32 indices only): an (n_shards,) int64 device tensor that receives #{x > z} over the
    same pairs from the same pass (tw_pair_sum_idx32_f64)."""
    n = len(pair_off) - 1
    t = L.torch()
    ixd, izd = _idx_pair(ix, iz, x_dev.numel(), z_dev.numel())
    pod = _off_dev(pair_off, pair_off_dev)
    max_pairs = int(np.diff(pair_off).max())
    per = int(L.lib().tw_pair_sum_idx_work_per_shard(max_pairs))
    work = L.empty((per * n,), t.float64)
    out = L.empty((n,), t.float64)
    if ixd.dtype == t.int32:
        L.call("tw_pair_sum_idx32_f64", L.ptr(x_dev), L.ptr(z_dev), L.ptr(ixd), L.ptr(izd),
               L.ptr(pod), n, max_pairs, kern, float(margin), L.ptr(work), L.ptr(out),
               L.ptr(count_out), L.stream_handle())
    else:
        if count_out is not None:
            raise ValueError("count_out needs int32 pair indices")
        L.call("tw_pair_sum_idx_f64", L.ptr(x_dev), L.ptr(z_dev), L.ptr(ixd), L.ptr(izd),
               L.ptr(pod), n, max_pairs, kern, float(margin), L.ptr(work), L.ptr(out),
               L.stream_handle())
    return out


def ratio(count, pairs) -> np.float64:
    """NumPy's mean of a 0/1 array: float64(sum) / float64(count), bit for bit."""
    return np.float64(np.float64(int(count)) / np.float64(int(pairs)))
