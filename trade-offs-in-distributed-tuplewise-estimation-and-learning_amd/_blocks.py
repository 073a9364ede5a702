"""The block protocol of the reference and its one-launch dispatch.

The reference's distributed estimator is a serial loop over N simulated workers (UN,
learning-experiment/compute_stats.py:56-92 and estimation-experiment/main.py:33-69): shuffle
the caller's arrays in place, cut consecutive blocks (or resample them), call
``f_block(X_block, Z_block)`` per block, and average.  Here the loop still runs on the host —
it owns the NumPy global RNG, whose draws must happen in exactly the reference's order — but
it only *plans*: block boundaries, index draws and degenerate-block handling.  The block
functions this package returns carry a ``_tw_block`` spec; ``run_un`` hands all planned
blocks of such a spec to one device launch and then averages with the reference's own
``np.mean``.  A user-supplied f_block without a spec is called block by block, exactly as the
reference does (that is the reference protocol, not a fallback of our kernels).
"""
from __future__ import annotations

import numpy as np

from . import _engine as E
from . import _lib as L
from . import _multi as M
from .numpy_rng import shuffle_pair


class Block:
    """One planned block: x/z are either (start, stop) slices of the shuffled arrays or index
    arrays (prop-SWR resampling); aux holds RNG draws the block function made."""
    __slots__ = ("x", "z", "aux")

    def __init__(self, x, z, aux=None):
        self.x, self.z, self.aux = x, z, aux

    def nx(self) -> int:
        return (self.x[1] - self.x[0]) if isinstance(self.x, tuple) else len(self.x)

    def nz(self) -> int:
        return (self.z[1] - self.z[0]) if isinstance(self.z, tuple) else len(self.z)


def _flat(a: np.ndarray) -> np.ndarray:
    return np.asarray(a).reshape(-1)


def _row_size(a) -> int:
    a = np.asarray(a)
    return int(np.prod(a.shape[1:], dtype=np.int64)) if a.ndim > 1 else 1


def whole(X, Z) -> "Block":
    """One block spanning every row of X and Z (blocks are in rows; see _elements)."""
    nx = X.shape[0] if X.ndim else 1
    nz = Z.shape[0] if Z.ndim else 1
    return Block((0, nx), (0, nz))


def _elements(blocks, side: str, rs: int) -> list:
    """Blocks' row selections (slices or row-index arrays) of a (n, ...) array whose rows
    hold rs elements, as selections of the flattened array (what Un's reshape(-1) sees)."""
    if rs == 1:
        return blocks
    out = []
    for b in blocks:
        sel = getattr(b, side)
        if isinstance(sel, tuple):
            e = (sel[0] * rs, sel[1] * rs)
        else:
            e = (np.asarray(sel, dtype=np.int64)[:, None] * rs + np.arange(rs)).reshape(-1)
        nb = Block(e, b.z, b.aux) if side == "x" else Block(b.x, e, b.aux)
        out.append(nb)
    return out


def _slice_offsets(blocks, side: str):
    """int64 offsets (len(blocks)+1) when the blocks' parts are consecutive slices of one
    array (the usual SWOR / prop-SWOR plan), else None."""
    parts = [getattr(b, side) for b in blocks]
    if not parts or not all(isinstance(p, tuple) for p in parts):
        return None
    starts = np.array([p[0] for p in parts], dtype=np.int64)
    stops = np.array([p[1] for p in parts], dtype=np.int64)
    if not np.all(starts[1:] == stops[:-1]):
        return None
    return np.concatenate([starts[:1], stops]).astype(np.int64)


def _layout(arr_dev, blocks, side: str):
    """Device array + int64 offsets (len(blocks)+1) for the blocks' x or z parts."""
    parts = [getattr(b, side) for b in blocks]
    if all(isinstance(p, tuple) for p in parts):
        # consecutive slices (possibly of length 0) of one array: offsets straight into it
        starts = np.array([p[0] for p in parts], dtype=np.int64)
        stops = np.array([p[1] for p in parts], dtype=np.int64)
        if len(parts) == 0 or np.all(starts[1:] == stops[:-1]):
            off = np.concatenate([starts[:1], stops]).astype(np.int64)
            return arr_dev, off
    # resampled blocks: gather on the device into one concatenated array
    t = L.torch()
    idx = [np.arange(p[0], p[1], dtype=np.int64) if isinstance(p, tuple)
           else np.asarray(p, dtype=np.int64) for p in parts]
    off = np.concatenate([[0], np.cumsum([len(i) for i in idx])]).astype(np.int64)
    cat = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
    gathered = arr_dev.index_select(0, t.from_numpy(cat).to(arr_dev.device))
    return gathered, off


def _upload_blocks(host, blocks, side: str):
    """The part of a host array a group of blocks reads, on the current device, + int64 offsets
    (len(blocks)+1): one contiguous slice for consecutive slice blocks (no host copy), else the
    blocks' selections concatenated on the host.  (Multi-device path: each slot uploads only
    its group's data.)"""
    parts = [getattr(b, side) for b in blocks]
    if all(isinstance(p, tuple) for p in parts) and all(
            a[1] == b[0] for a, b in zip(parts, parts[1:])):
        lo, hi = parts[0][0], parts[-1][1]
        off = np.array([p[0] - lo for p in parts] + [hi - lo], dtype=np.int64)
        return L.to_device(np.ascontiguousarray(host[lo:hi])), off
    pieces = [host[p[0]:p[1]] if isinstance(p, tuple) else host[np.asarray(p, dtype=np.int64)]
              for p in parts]
    off = np.concatenate([[0], np.cumsum([len(q) for q in pieces])]).astype(np.int64)
    cat = np.concatenate(pieces) if pieces else host[:0]
    return L.to_device(np.ascontiguousarray(cat)), off


class BlockSpec:
    """Descriptor of a package block function (see module docstring)."""

    def draw(self, nx: int, nz: int):
        """RNG draws the reference block function makes on a block of this shape."""
        return None

    def evaluate(self, X: np.ndarray, Z: np.ndarray, blocks: list) -> list:
        raise NotImplementedError

    def work(self, nx: int, nz: int, dtype) -> int:
        """Device work of one block in all-pairs compare equivalents (what the multi-device
        split weighs; default: every pair once)."""
        return nx * nz


class CompleteCount(BlockSpec):
    """Un-type block: exact count of a comparison predicate over all pairs, divided by nx*nz.

    literal_sub=False: est.Un ``X > Z`` (estimation-experiment/main.py:31)
    literal_sub=True : cs.Un AUC ``(X - Z) > 0`` (compute_stats.py:19)
    tie_mode="half" : opt-in +0.5 on ties (BASELINE.json); value = half-units / (2 nx nz)."""

    def __init__(self, literal_sub: bool, tie_mode: str = "strict"):
        self.literal_sub = literal_sub
        self.tie_mode = tie_mode

    def operands(self, X, Z):
        if self.literal_sub:
            x, z, code, mode = E.subtract_gt_operands(X, Z)
        else:
            (x, z, code), mode = E.compare_operands(X, Z), "gt"
        if self.tie_mode == "half":
            if mode != "gt" and mode != "subgt":
                raise NotImplementedError("tie_mode='half' needs an ordered comparison")
            mode = "half"
        return x, z, code, mode

    def _mode(self, dtype) -> str:
        if self.literal_sub and np.issubdtype(np.dtype(dtype), np.integer):
            return "subgt"  # int64 wrap-around: all pairs only
        return "half" if self.tie_mode == "half" else "gt"

    def work(self, nx, nz, dtype):
        """the count 'auto' runs: (nx + nz) sorted-element steps or nx*nz compares"""
        return E.count_work(nx, nz, self._mode(dtype))

    def evaluate(self, X, Z, blocks):
        x, z, code, mode = self.operands(_flat(X), _flat(Z))
        blocks = _elements(_elements(blocks, "x", _row_size(X)), "z", _row_size(Z))
        wmode = mode if mode != "ne" else "gt"
        work = sum(E.count_work(b.nx(), b.nz(), wmode) for b in blocks)
        if mode != "ne" and M.slots_for(work, len(blocks)):
            pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF, "subgt": L.TW_PRED_SUBGT}[mode]

            def enqueue(sub):  # this slot's blocks: upload their data, count (in flight)
                xa, xo = _upload_blocks(x, sub, "x")
                za, zo = _upload_blocks(z, sub, "z")
                sh = E.Shards(xa, xo, za, zo, code)
                xod, zod = sh.offsets_dev()
                mx, mz = int(sh.nx.max()), int(sh.nz.max())
                return E.count_launch(xa, xod, za, zod, len(sub), mx, mz, code, pred,
                                      E.pick_algo("auto", mx, mz, mode))

            counts = M.gather(M.spread(blocks, lambda b: E.count_work(b.nx(), b.nz(), wmode),
                                       enqueue))
            counts = counts.astype(np.int64).view(np.uint64)
        else:
            xo, zo = _slice_offsets(blocks, "x"), _slice_offsets(blocks, "z")
            if xo is not None and zo is not None:  # the usual plan: one upload for all four
                xa, za, xod, zod = L.to_device_many([x, z, xo, zo])
                sh = E.Shards(xa, xo, za, zo, code)
                sh._x_off_dev, sh._z_off_dev = xod, zod
            else:
                xd, zd = L.to_device(x), L.to_device(z)
                xa, xo = _layout(xd, blocks, "x")
                za, zo = _layout(zd, blocks, "z")
                sh = E.Shards(xa, xo, za, zo, code)
            counts = E.count_complete(sh, mode)
        out = []
        for b, c in zip(blocks, counts):
            pairs = b.nx() * b.nz()
            out.append(E.ratio(c, 2 * pairs) if mode == "half" else E.ratio(c, pairs))
        return out


    def evaluate_device(self, xd, zd, blocks):
        """evaluate() on float64 device arrays (the device-shuffle path of run_un_repeated):
        `X > Z` and the literal `(X - Z) > 0` are the same ordered comparison on doubles."""
        done = self.enqueue_device(xd, zd, blocks)
        if done is not None:
            return done()
        mode = "half" if self.tie_mode == "half" else "gt"
        xa, xo = _layout(xd, blocks, "x")
        za, zo = _layout(zd, blocks, "z")
        sh = E.Shards(xa, xo, za, zo, L.TW_F64)
        sh._x_off_dev, sh._z_off_dev = L.to_device_many([xo, zo])  # one upload for both
        return self._ratios(E.count_complete(sh, mode), xo, zo, mode)

    def enqueue_device(self, xd, zd, blocks, stream=None, after=()):
        """evaluate_device in two halves, for blocks that are consecutive slices of xd / zd
        (the SWOR / prop-SWOR plans; None otherwise): the offsets go up on the current stream,
        then the count is enqueued — on `stream` when given, ordered after the upload and the
        streams in `after` (the arrays' producers); returns done() -> the values (one sync,
        ordered after the count on the caller's current stream)."""
        t = L.torch()
        xo, zo = _slice_offsets(blocks, "x"), _slice_offsets(blocks, "z")
        if xo is None or zo is None:
            return None
        mode = "half" if self.tie_mode == "half" else "gt"
        xod, zod = L.to_device_many([xo, zo], pinned=stream is not None)
        mx, mz = int(np.diff(xo).max()), int(np.diff(zo).max())
        pred = L.TW_PRED_HALF if mode == "half" else L.TW_PRED_GT
        algo = E.pick_algo("auto", mx, mz, mode)
        if stream is None:
            dev = E.count_launch(xd, xod, zd, zod, len(blocks), mx, mz, L.TW_F64, pred, algo)
        else:
            stream.wait_stream(t.cuda.current_stream())
            for s in after:
                stream.wait_stream(s)
            with t.cuda.stream(stream):
                for a in (xod, zod, xd, zd):
                    a.record_stream(stream)  # read there; the caller may drop them meanwhile
                dev = E.count_launch(xd, xod, zd, zod, len(blocks), mx, mz, L.TW_F64, pred,
                                     algo)

        def done():
            if stream is not None:
                t.cuda.current_stream().wait_stream(stream)
            return self._ratios(E._counts_to_host(dev), xo, zo, mode)
        return done

    @staticmethod
    def _ratios(counts, xo, zo, mode):
        # float64(count) / float64(pairs) per block, as E.ratio: both conversions exact
        # (counts and pairs < 2^53 here) and one IEEE division each — the same bits, vectorised
        pairs = np.diff(xo).astype(np.int64) * np.diff(zo).astype(np.int64)
        if mode == "half":
            pairs = 2 * pairs
        if counts.size and (int(counts.max()) >= 1 << 53 or int(pairs.max()) >= 1 << 53):
            return [E.ratio(c, p) for c, p in zip(counts, pairs)]
        return list(counts.astype(np.float64) / pairs.astype(np.float64))


class CompleteSum(BlockSpec):
    """cs.Un prod/gini (compute_stats.py:15-18) and conv_AUC (compute_stats.py:129-135):
    mean over all pairs of a float kernel."""

    def __init__(self, kern: int, margin: float = 0.0):
        self.kern = kern
        self.margin = margin

    def evaluate(self, X, Z, blocks):
        x = _flat(X).astype(np.float64, copy=False)
        z = _flat(Z).astype(np.float64, copy=False)
        blocks = _elements(_elements(blocks, "x", _row_size(X)), "z", _row_size(Z))
        if M.slots_for(sum(b.nx() * b.nz() for b in blocks), len(blocks)):
            def enqueue(sub):
                xa, xo = _upload_blocks(x, sub, "x")
                za, zo = _upload_blocks(z, sub, "z")
                return E.pair_sum_complete_dev(E.Shards(xa, xo, za, zo, L.TW_F64), self.kern,
                                               self.margin)

            sums = M.gather(M.spread(blocks, lambda b: b.nx() * b.nz(), enqueue))
        else:
            xd, zd = L.to_device(x), L.to_device(z)
            xa, xo = _layout(xd, blocks, "x")
            za, zo = _layout(zd, blocks, "z")
            sums = E.pair_sum_complete(E.Shards(xa, xo, za, zo, L.TW_F64), self.kern,
                                       self.margin)
        # NumPy returns the mean in the operands' float type (float32 stays float32); the
        # device accumulates in float64, so float32 results are the better-rounded value.
        rt = np.result_type(np.asarray(X).dtype, np.asarray(Z).dtype)
        cast = rt.type if rt.kind == "f" else np.float64
        return [cast(s / np.float64(b.nx() * b.nz())) for b, s in zip(blocks, sums)]

    def evaluate_device(self, xd, zd, blocks):
        """evaluate() on float64 device arrays (the device-shuffle path of run_un_repeated)."""
        xa, xo = _layout(xd, blocks, "x")
        za, zo = _layout(zd, blocks, "z")
        sums = E.pair_sum_complete(E.Shards(xa, xo, za, zo, L.TW_F64), self.kern, self.margin)
        return [np.float64(s / np.float64(b.nx() * b.nz())) for b, s in zip(blocks, sums)]


class Incomplete(BlockSpec):
    """cs.UB (compute_stats.py:37-42): B pairs drawn with replacement by two randint calls
    (X indices first, then Z indices), then UB_indices on them."""

    def __init__(self, B: int, kernel: str):
        self.B = int(B)
        self.kernel = kernel

    def draw(self, nx, nz):
        ix = np.random.randint(0, nx, self.B)
        iz = np.random.randint(0, nz, self.B)
        return ix, iz

    def work(self, nx, nz, dtype):
        """B indexed pairs (two random gathers each: ~50 compares of the all-pairs kernel)"""
        return 50 * self.B

    def evaluate(self, X, Z, blocks):
        rs = _row_size(X)
        if _row_size(Z) != rs:
            raise ValueError("UB on rows of different widths cannot broadcast")
        # X[ind] - Z[ind] on rows of rs elements compares element pairs (r*rs + c, r'*rs + c):
        # blocks and draws become element blocks and element-local indices
        eb = _elements(_elements(blocks, "x", rs), "z", rs)
        ix_loc, iz_loc = [], []
        for b in blocks:
            ix, iz = b.aux
            if rs > 1:
                ix = (np.asarray(ix)[:, None] * rs + np.arange(rs)).reshape(-1)
                iz = (np.asarray(iz)[:, None] * rs + np.arange(rs)).reshape(-1)
            ix_loc.append(np.asarray(ix, dtype=np.int64))
            iz_loc.append(np.asarray(iz, dtype=np.int64))
        return block_indexed_values(_flat(X), _flat(Z), eb, ix_loc, iz_loc, self.kernel)

    def evaluate_device(self, xd, zd, blocks):
        """evaluate() on float64 device arrays of 1-D samples (the device-shuffle path of
        run_un_repeated): the blocks laid out as in block_indexed_values, the draws shifted."""
        ix_loc = [np.asarray(b.aux[0], dtype=np.int64) for b in blocks]
        iz_loc = [np.asarray(b.aux[1], dtype=np.int64) for b in blocks]
        offs = np.concatenate([[0], np.cumsum([len(a) for a in ix_loc])]).astype(np.int64)
        npairs = np.diff(offs)
        xa, xo = _layout(xd, blocks, "x")
        za, zo = _layout(zd, blocks, "z")
        ix = np.concatenate([a + o for a, o in zip(ix_loc, xo[:-1])])
        iz = np.concatenate([a + o for a, o in zip(iz_loc, zo[:-1])])
        if self.kernel == "AUC":
            counts = E.count_indexed(xa, za, L.TW_F64, ix, iz, offs, "gt", spans=(xo, zo))
            return [E.ratio(c, p) for c, p in zip(counts, npairs)]
        kern = {"prod": L.TW_KERN_PROD, "gini": L.TW_KERN_GINI}[self.kernel]
        sums = E.pair_sum_indexed(xa, za, ix, iz, offs, kern)
        return [np.float64(s / np.float64(p)) for s, p in zip(sums, npairs)]


def block_indexed_values(x: np.ndarray, z: np.ndarray, blocks: list, ix_loc: list,
                         iz_loc: list, kernel: str) -> list:
    """UB_indices (compute_stats.py:22-30) of every block, block b drawing ix_loc[b] /
    iz_loc[b] (block-local positions).  The blocks are laid out as consecutive spans of one
    device array per sample (slice plans point straight into the shuffled sample, resampled
    prop-SWR blocks are gathered on the device), so every AUC count runs on the LDS rank codes
    (tw_count_pairs_idx32_ws) with int32 absolute indices (8 B per pair)."""
    offs = np.concatenate([[0], np.cumsum([len(a) for a in ix_loc])]).astype(np.int64)
    if kernel == "AUC":
        xx, zz, code, mode = E.subtract_gt_operands(x, z)
    else:
        xx, zz, code, mode = (x.astype(np.float64, copy=False), z.astype(np.float64, copy=False),
                              L.TW_F64, None)
    npairs = np.diff(offs)
    if mode != "ne" and M.slots_for(int(offs[-1]) * 50, len(blocks)):  # ~50 compares a pair
        pos = {id(b): i for i, b in enumerate(blocks)}

        def enqueue(sub):  # this slot's blocks, their draws shifted into the uploaded spans
            i0 = pos[id(sub[0])]
            xa, xo = _upload_blocks(xx, sub, "x")
            za, zo = _upload_blocks(zz, sub, "z")
            ixs = np.concatenate([ix_loc[i0 + k] + xo[k] for k in range(len(sub))])
            izs = np.concatenate([iz_loc[i0 + k] + zo[k] for k in range(len(sub))])
            po = offs[i0:i0 + len(sub) + 1] - offs[i0]
            if kernel == "AUC":
                pred = {"gt": L.TW_PRED_GT, "half": L.TW_PRED_HALF,
                        "subgt": L.TW_PRED_SUBGT}[mode]
                return E.count_indexed_ranked_dev(xa, L.to_device(xo), za, L.to_device(zo),
                                                  int(np.diff(xo).max()), int(np.diff(zo).max()),
                                                  code, ixs, izs, po, pred)
            kern = {"prod": L.TW_KERN_PROD, "gini": L.TW_KERN_GINI}[kernel]
            return E.pair_sum_indexed_dev(xa, za, ixs, izs, po, kern)

        vals = M.gather(M.spread(blocks, lambda b: npairs[pos[id(b)]], enqueue))
        if kernel == "AUC":
            return [E.ratio(c, p) for c, p in zip(vals.astype(np.int64).view(np.uint64), npairs)]
        return [np.float64(v / np.float64(p)) for v, p in zip(vals, npairs)]
    xa, xo = _layout(L.to_device(xx), blocks, "x")
    za, zo = _layout(L.to_device(zz), blocks, "z")
    ix = np.concatenate([a + o for a, o in zip(ix_loc, xo[:-1])]) if ix_loc else np.zeros(0, np.int64)
    iz = np.concatenate([a + o for a, o in zip(iz_loc, zo[:-1])]) if iz_loc else np.zeros(0, np.int64)
    npairs = np.diff(offs)
    if kernel == "AUC":
        counts = E.count_indexed(xa, za, code, ix, iz, offs, mode, spans=(xo, zo))
        return [E.ratio(c, p) for c, p in zip(counts, npairs)]
    kern = {"prod": L.TW_KERN_PROD, "gini": L.TW_KERN_GINI}[kernel]
    sums = E.pair_sum_indexed(xa, za, ix, iz, offs, kern)
    return [np.float64(s / np.float64(p)) for s, p in zip(sums, npairs)]


def indexed_values(x: np.ndarray, z: np.ndarray, ix: np.ndarray, iz: np.ndarray,
                   pair_off: np.ndarray, kernel: str, margin: float = 0.0,
                   spans=None) -> list:
    """Per-shard means of `kernel` over absolute index pairs (UB_indices semantics,
    compute_stats.py:22-30).  spans: the shard spans for the rank-code count (E.count_indexed);
    None = one shard spanning both whole arrays (UB_indices / UB_pairs)."""
    npairs = np.diff(pair_off)
    if spans is None and len(pair_off) == 2:
        spans = ([0, x.shape[0]], [0, z.shape[0]])
    if kernel == "AUC":
        xx, zz, code, mode = E.subtract_gt_operands(x, z)
        counts = E.count_indexed(L.to_device(xx), L.to_device(zz), code, ix, iz, pair_off, mode,
                                 spans=spans)
        return [E.ratio(c, p) for c, p in zip(counts, npairs)]
    kern = {"prod": L.TW_KERN_PROD, "gini": L.TW_KERN_GINI, "hinge": L.TW_KERN_HINGE,
            "logistic": L.TW_KERN_LOGISTIC}[kernel]
    xd = L.to_device(x.astype(np.float64, copy=False))
    zd = L.to_device(z.astype(np.float64, copy=False))
    sums = E.pair_sum_indexed(xd, zd, ix, iz, pair_off, kern, margin)
    return [np.float64(s / np.float64(p)) for s, p in zip(sums, npairs)]


def plan_un(X, Z, N, spec, sampling_type, variant: str, shuffle=shuffle_pair) -> list:
    """The host half of UN (compute_stats.py:56-92 "cs", estimation-experiment/main.py:33-69
    "est"): shuffle X and Z in place, then walk the N blocks making every RNG draw of the
    reference in order.  Returns the plan [("val", Block) | ("zero",)] in append order.
    shuffle(X, Z): the in-place shuffles (or, for the device path, only their draws)."""
    X_rem = X
    Z_rem = Z
    shuffle(X_rem, Z_rem)  # np.random.shuffle(X); np.random.shuffle(Z), bit for bit
    n_X = X_rem.shape[0]
    n_Z = Z_rem.shape[0]
    tau = int((n_X + n_Z) / N)
    plan = []
    x_pos = z_pos = 0
    for _ in range(N):
        if sampling_type != "prop-SWR":
            if sampling_type.startswith("prop"):
                k = int(n_X / N)
            else:
                n_X = X_rem.shape[0] - x_pos
                n_Z = Z_rem.shape[0] - z_pos
                k = np.random.binomial(tau, n_X / (n_X + n_Z))
            if k in (0, tau):
                if variant == "cs":
                    assert sampling_type == "SWOR"
                    plan.append(("zero",))
                elif sampling_type == "SWOR":
                    plan.append(("zero",))
            else:
                xs = (x_pos, min(x_pos + k, X_rem.shape[0]))
                zs = (z_pos, min(z_pos + tau - k, Z_rem.shape[0]))
                blk = Block(xs, zs)
                blk.aux = spec.draw(blk.nx(), blk.nz())
                plan.append(("val", blk))
            x_pos = min(x_pos + k, X_rem.shape[0])
            z_pos = min(z_pos + (tau - k), Z_rem.shape[0])
        elif sampling_type == "prop-SWR":
            ix = np.random.randint(0, n_X, int(n_X / N))
            iz = np.random.randint(0, n_Z, int(n_Z / N))
            blk = Block(ix, iz)
            blk.aux = spec.draw(blk.nx(), blk.nz())
            plan.append(("val", blk))
    return plan


def finish_un(plan, values) -> np.float64:
    """UN's `np.mean(vals)` with the block values in plan order."""
    values = iter(values)
    return np.mean([0 if p[0] == "zero" else next(values) for p in plan])


def run_un(X, Z, N, f_block, sampling_type, variant: str):
    """Shared body of UN (compute_stats.py:56-92, variant "cs"; estimation-experiment/main.py
    :33-69, variant "est").  Keeps the in-place shuffle and every RNG draw in order."""
    spec = getattr(f_block, "_tw_block", None)
    if spec is None:  # user block function: the reference protocol, block by block
        shuffle_pair(X, Z)
        n_X, n_Z = X.shape[0], Z.shape[0]
        return _run_un_python(X, Z, N, f_block, sampling_type, variant, n_X, n_Z,
                              int((n_X + n_Z) / N))
    if (isinstance(X, np.ndarray) and isinstance(Z, np.ndarray)
            and _device_shuffle_ok(X, Z, spec)):
        return _run_un_repeated_device(X, Z, N, spec, sampling_type, variant, 1)
    if (isinstance(X, np.ndarray) and isinstance(Z, np.ndarray) and X.ndim == 1
            and Z.ndim == 1 and sampling_type.startswith("prop") and sampling_type != "prop-SWR"
            and fixed_layout(X.shape[0], Z.shape[0], N, spec, sampling_type) is not None):
        return run_un_repeated(X, Z, N, spec, sampling_type, variant, 1)  # the fixed layout
    plan = plan_un(X, Z, N, spec, sampling_type, variant)
    blocks = [p[1] for p in plan if p[0] == "val"]
    return finish_un(plan, spec.evaluate(X, Z, blocks) if blocks else [])


_LAYOUTS = {}  # (n, m, N, sampling_type) -> fixed_layout (CompleteCount plans draw nothing)


def fixed_layout(n, m, N, spec, sampling_type):
    """The block ranges of a plan that depends on the sizes only — Un's one whole block
    (N None) or prop-SWOR / prop-SWR-free plan_un's N blocks, which draw nothing — as
    (x starts, x end, z starts, z end, pairs per block); None where the spec is not a
    CompleteCount, the plan has an empty block or skips one (the general path's nan / the
    reference's assert), or a block is not a consecutive slice from 0.  Cached per shape."""
    if type(spec) is not CompleteCount:
        return None
    key = (n, m, N, sampling_type)
    if key in _LAYOUTS:
        return _LAYOUTS[key]
    lay = None  # (the plan of a CompleteCount depends on the sizes only)
    if N is None:
        xs, zs = [(0, n)], [(0, m)]
    else:
        plan = plan_un(np.empty(n, np.uint8), np.empty(m, np.uint8), N, spec, sampling_type,
                       "est", shuffle=lambda a, b: None)
        ok = bool(plan) and all(p[0] == "val" for p in plan)
        xs = [p[1].x for p in plan] if ok else []
        zs = [p[1].z for p in plan] if ok else []
    if xs and all(isinstance(a, tuple) for a in xs + zs) and all(
            sel[0][0] == 0 and all(a[1] == b[0] for a, b in zip(sel, sel[1:]))
            for sel in (xs, zs)):
        pairs = np.array([(a[1] - a[0]) * (b[1] - b[0]) for a, b in zip(xs, zs)],
                         dtype=np.int64)
        if np.all(pairs > 0):
            lay = (np.array([a[0] for a in xs], dtype=np.int64), xs[-1][1],
                   np.array([b[0] for b in zs], dtype=np.int64), zs[-1][1], pairs)
    if len(_LAYOUTS) > 256:
        _LAYOUTS.clear()
    _LAYOUTS[key] = lay
    return lay


def fixed_values(spec, bx, bz, lay) -> np.ndarray:
    """Block values (J, blocks) of J snapshot rows bx (J, x end) / bz (J, z end) under one
    fixed layout: one upload, one count launch over all rows' blocks (offsets by
    broadcasting), E.ratio's float64(count) / float64(pairs) as one array division."""
    xs, lx, zs, lz, pairs = lay
    J = bx.shape[0]
    x, z, code, mode = spec.operands(bx.reshape(-1), bz.reshape(-1))
    rows = np.arange(J, dtype=np.int64)[:, None]
    xo = np.append((rows * lx + xs).ravel(), J * lx).astype(np.int64)
    zo = np.append((rows * lz + zs).ravel(), J * lz).astype(np.int64)
    t = L.torch()
    xt, zt = t.from_numpy(x), t.from_numpy(z)
    if x.size > (1 << 16) and xt.is_pinned() and zt.is_pinned():
        # rows staged in page-locked buffers by the caller (replicate): uploaded as they lie,
        # no packing copy on the host; the small offsets in one staged copy
        xa = xt.to(L.device(), non_blocking=True)
        za = zt.to(L.device(), non_blocking=True)
        xod, zod = L.to_device_many([xo, zo])
    else:
        xa, za, xod, zod = L.to_device_many([x, z, xo, zo])
    sh = E.Shards(xa, xo, za, zo, code)
    sh._x_off_dev, sh._z_off_dev = xod, zod
    counts = np.asarray(E.count_complete(sh, mode)).view(np.uint64)
    den = (2 * pairs if mode == "half" else pairs).astype(np.float64)
    return counts.astype(np.float64).reshape(J, len(xs)) / den


def run_un_repeated(X, Z, N, spec, sampling_type, variant: str, T: int):
    """np.mean([UN(X, Z, N, f_block, sampling_type) for _ in range(T)]) (UnNT, UnNBT) with
    the T host halves (in-place shuffles, every RNG draw) in the reference's order and all
    T x N blocks counted in ONE launch on snapshots of the shuffled samples.  Scores must be
    1-D or (n, 1) (evaluate_many); returns None otherwise (the caller loops)."""
    if not (isinstance(X, np.ndarray) and isinstance(Z, np.ndarray)):
        return None  # the in-place shuffles must act on the caller's own objects
    if any(a.ndim > 2 or (a.ndim == 2 and a.shape[1] != 1) for a in (X, Z)):
        return None
    if _device_shuffle_ok(X, Z, spec, N, T):
        return _run_un_repeated_device(X, Z, N, spec, sampling_type, variant, T)
    if (X.ndim == 1 and Z.ndim == 1 and sampling_type.startswith("prop")
            and sampling_type != "prop-SWR" and T >= 1):
        lay = fixed_layout(X.shape[0], Z.shape[0], N, spec, sampling_type)
        if lay is not None:
            # the T snapshots as rows, all blocks in one launch, the plan means and the
            # repetitions' mean as row reductions (the same bits as finish_un / np.mean)
            bx = np.empty((T, lay[1]), dtype=X.dtype)
            bz = np.empty((T, lay[3]), dtype=Z.dtype)
            for t in range(T):
                shuffle_pair(X, Z)  # plan_un's in-place shuffles, bit for bit
                bx[t] = X[:lay[1]]
                bz[t] = Z[:lay[3]]
            return np.mean(fixed_values(spec, bx, bz, lay).mean(axis=-1))
    plans, jobs = [], []
    for t in range(T):
        plan = plan_un(X, Z, N, spec, sampling_type, variant)
        last = t + 1 == T
        jobs.append((X if last else X.copy(), Z if last else Z.copy(),
                     [p[1] for p in plan if p[0] == "val"]))
        plans.append(plan)
    vals = evaluate_many(spec, jobs) if jobs else []
    return np.mean([finish_un(p, v) for p, v in zip(plans, vals)])


# samples of at least this many items (per array) take the device shuffles in UnNT / UnNBT
DEVICE_SHUFFLE_MIN = 1 << 16
# study hook (tools/time_dropin_parts.py): a list receives (label, perf_counter) marks of the
# device-shuffle drop-in call
DROPIN_MARKS = None
# the device-shuffle drop-in's pipelining (round 5): the counts of step k enqueued while the
# host draws step k + 1 (off: measured slower once the launches moved to the launcher thread —
# its enqueue work there competes with the drawing thread; profiles/r05s28_dropin_*.log); the
# call's last shuffle drawn and pushed in this many parts (0: whole)
EARLY_COUNTS = False
STREAM_LAST_SHUFFLE = 4
# ... and the uploads, swap-round launches and count enqueues made on a launcher thread
# (_engine.launcher), off the thread that makes the draws
THREADED_LAUNCHES = True


def _mark(label):
    if DROPIN_MARKS is not None:
        import time
        DROPIN_MARKS.append((label, time.perf_counter()))


def _device_shuffle_ok(X, Z, spec, N: int = 1, T: int = 1) -> bool:
    """The repeated UN's shuffles and blocks can stay on the device: 1-D C-contiguous float64
    samples (8-byte items whose comparison / kernel operands are the scores themselves), a spec
    with a device evaluation, the legacy MT19937 global state, and blocks whose work does not
    call for spreading over several devices (the multi-device split weighs the algorithm that
    will run: the sorted count of est.UnNT's blocks is ~0.1 ms, so a node with 8 GPUs keeps
    the one-device shuffles — DESIGN.md §6)."""
    ok = (X.ndim == 1 and Z.ndim == 1 and X.dtype == np.float64 and Z.dtype == np.float64
          and X.flags.c_contiguous and Z.flags.c_contiguous and X.flags.writeable
          and Z.flags.writeable and max(X.shape[0], Z.shape[0]) >= DEVICE_SHUFFLE_MIN
          and X.shape[0] + Z.shape[0] < 2 ** 31 and hasattr(spec, "evaluate_device")
          and not np.shares_memory(X, Z)  # separate uploads would lose the aliasing
          and np.random.get_state(legacy=True)[0] == "MT19937")
    if not ok or len(M.devices()) < 2:
        return ok
    nb = max(1, int(N)) * max(1, int(T))
    per = spec.work(max(1, X.shape[0] // max(1, N)), max(1, Z.shape[0] // max(1, N)),
                    np.float64)
    return M.slots_for(per * nb, nb) is None


def _run_un_repeated_device(X, Z, N, spec, sampling_type, variant: str, T: int):
    """run_un_repeated with the shuffles' swaps on the device: the host makes every draw in the
    reference's order (the T shuffles' index draws, numpy_rng.shuffle_draws32, interleaved with
    the block draws), the device applies the T shuffles to one upload of X and Z keeping every
    state (_engine.shuffle_snapshots_device: the sequential swaps' permutation, bit for bit),
    the blocks are counted on those states, and the caller's arrays receive the last state (the
    in-place side effect of the T np.random.shuffle calls).  Round 5: every upload and launch
    is made by a launcher thread while this thread draws (THREADED_LAUNCHES), the counts of
    step k are enqueued on their own stream once step k's shuffles are (EARLY_COUNTS: they run
    while the host draws step k + 1), the call's last shuffle is drawn and pushed in parts
    (STREAM_LAST_SHUFFLE, DeviceShuffles.draw_push_z_streamed: its first windows' swaps run
    while the host draws the rest), and Z's write-back runs beside the last step's count."""
    from .numpy_rng import shuffle_draws32
    t = L.torch()
    plans = []
    _mark("start")
    # X and Z go up on a helper thread while the host draws the first shuffle
    ds = E.DeviceShuffles(X, Z, T, reuse=True, threaded=THREADED_LAUNCHES)
    _mark("setup")
    step = [0]

    def draws(a, b):  # each side's draws into pinned memory; the device swaps it meanwhile
        shuffle_draws32(a.shape[0], out=ds.draw_x())
        _mark("x drawn")
        ds.push_x()
        if step[0] == T - 1 and STREAM_LAST_SHUFFLE:
            ds.draw_push_z_streamed(STREAM_LAST_SHUFFLE)
        else:
            shuffle_draws32(b.shape[0], out=ds.draw_z())
            ds.push_z()
        _mark("z drawn")

    early = hasattr(spec, "enqueue_device") and EARLY_COUNTS
    cs = E.side_stream("count") if early else None
    pending = {}
    nx, nz = X.shape[0], Z.shape[0]
    for k in range(T):
        step[0] = k
        plans.append(plan_un(X, Z, N, spec, sampling_type, variant, shuffle=draws))
        if early and k < T - 1:  # step k's counts beside the host's next draws
            def count(k=k):  # after step k's pushes (on the launcher thread when threaded)
                blks = [p[1] for p in plans[k] if p[0] == "val"]
                done = spec.enqueue_device(ds.xs[k], ds.zs[k], blks, stream=cs,
                                           after=(ds.sx, ds.sz)) if blks else None
                if done is not None:
                    pending[k] = done
            ds.submit(count)
            _mark("counts submitted")
    _mark("pushed")
    # the in-place side effect, X first: its last state goes back while Z's last shuffle runs
    # (threaded: on the write-back thread, beside this thread's wait for Z and Z's write-back;
    # not earlier — beside the last draws it slowed them)
    if THREADED_LAUNCHES:
        ds.write_back_x_async(X)
    else:
        t.from_numpy(X).copy_(ds.last_x())
    _mark("x written back")
    xs, zs = ds.finish()  # (drains the launcher: every count task has run)
    _mark("finish")
    if 0 in ds.redone:  # (rare) X's shuffles were resumed: its last state changed
        ds.drain_write_back()
        t.from_numpy(X).copy_(xs[T - 1])
    if ds.redone:  # (rare) later states changed: every step is counted again below
        pending.clear()
    # the steps not counted yet, in one launch (enqueued before Z's write-back runs beside it)
    rest = [k for k in range(T) if k not in pending]
    blocks, counts = [], {}
    for k in rest:
        blks = [p[1] for p in plans[k] if p[0] == "val"]
        for b in blks:
            bx = (b.x[0] + k * nx, b.x[1] + k * nx) if isinstance(b.x, tuple) \
                else np.asarray(b.x) + k * nx
            bz = (b.z[0] + k * nz, b.z[1] + k * nz) if isinstance(b.z, tuple) \
                else np.asarray(b.z) + k * nz
            blocks.append(Block(bx, bz, b.aux))
        counts[k] = len(blks)
    done_rest = None
    if blocks and early:
        done_rest = spec.enqueue_device(xs.reshape(-1), zs.reshape(-1), blocks)
    # the caller's Z ends in the last shuffled state too (X was written above): copied out on
    # a stream of its own, so the copy engine moves it while the last count runs
    wb = E.side_stream("writeback")
    ds.order_after(wb)
    with t.cuda.stream(wb):
        t.from_numpy(Z).copy_(zs[T - 1])
    ds.drain_write_back()  # X's copy (threaded) has landed too
    _mark("z written back")
    if done_rest is not None:
        vals = done_rest()
    else:
        vals = spec.evaluate_device(xs.reshape(-1), zs.reshape(-1), blocks) if blocks else []
    _mark("counted")
    by_step, i = {}, 0
    for k in rest:
        by_step[k] = vals[i:i + counts[k]]
        i += counts[k]
    for k, done in pending.items():
        by_step[k] = done()
    return np.mean([finish_un(plans[k], by_step[k]) for k in range(T)])


def evaluate_many(spec, jobs) -> list:
    """Block values of several independent (X, Z, blocks) jobs of one spec in ONE launch:
    the jobs' score vectors are concatenated and their blocks shifted.  Scores must be 1-D
    (or (n, 1)); returns one list of values per job."""
    xs, zs, blocks, counts = [], [], [], []
    xo = zo = 0
    for X, Z, blks in jobs:
        x, z = _flat(X), _flat(Z)
        for b in blks:
            bx = (b.x[0] + xo, b.x[1] + xo) if isinstance(b.x, tuple) else np.asarray(b.x) + xo
            bz = (b.z[0] + zo, b.z[1] + zo) if isinstance(b.z, tuple) else np.asarray(b.z) + zo
            blocks.append(Block(bx, bz, b.aux))
        xs.append(x)
        zs.append(z)
        counts.append(len(blks))
        xo += x.shape[0]
        zo += z.shape[0]
    if not blocks:
        return [[] for _ in jobs]
    vals = spec.evaluate(np.concatenate(xs), np.concatenate(zs), blocks)
    out, i = [], 0
    for c in counts:
        out.append(vals[i:i + c])
        i += c
    return out


def _run_un_python(X_rem, Z_rem, N, f_block, sampling_type, variant, n_X, n_Z, tau):
    vals = list()
    for _ in range(N):
        if sampling_type != "prop-SWR":
            if sampling_type.startswith("prop"):
                k = int(n_X / N)
            else:
                n_X = X_rem.shape[0]
                n_Z = Z_rem.shape[0]
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
