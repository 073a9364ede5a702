"""Drop-in replacement for the estimator functions of estimation-experiment/main.py.

Un, UN, UnN, UnNT keep the reference's names, signatures, in-place shuffling and RNG order
(estimation-experiment/main.py:29-79); the pair counts run in libtuplewise.so.  The closed-form
moments of the Bernoulli experiment (main.py:10-27, :103-104) are pure formulas and are kept
here verbatim in meaning, since the statistical tests use them as known answers.

Extension (BASELINE.json): ``Un(X, Z, tie_mode="half")`` scores ties 1/2.  The default
"strict" is the reference semantics (ties score 0).
"""
from __future__ import annotations

import numpy as np

from . import _blocks as Bk
from . import _lib as L


def p(e):
    return e


def q(e):
    return 1 - e


def sigma_1(e):
    return (p(e) ** 2) * q(e) * (1 - q(e))


def sigma_2(e):
    return ((1 - q(e)) ** 2) * p(e) * (1 - p(e))


def sigma_0(e):
    return p(e) * q(e) * (1 - p(e)) * (1 - q(e))


def Mean_Un(e):
    return q(e) + (1 - q(e)) * (1 - p(e))


def Var_Un(e, n, m):
    """main.py:103-104 (a closure over n, m there)."""
    return sigma_1(e) / n + sigma_2(e) / m + sigma_0(e) / (n * m)


def _un_block(tie_mode):
    spec = Bk.CompleteCount(literal_sub=False, tie_mode=tie_mode)

    def Un_block(X, Z):
        X = np.asarray(X)
        Z = np.asarray(Z)
        return spec.evaluate(X, Z, [Bk.whole(X, Z)])[0]

    Un_block._tw_block = spec
    return Un_block


_UN_STRICT = _un_block("strict")
_UN_HALF = _un_block("half")


def Un(X, Z, tie_mode="strict"):
    """Computes Un, full two-sample U-statistic.  (main.py:29-31)"""
    return (_UN_HALF if tie_mode == "half" else _UN_STRICT)(X, Z)


# UN(..., f_block=Un) must dispatch in one launch: expose the tagged block function's spec.
Un._tw_block = _UN_STRICT._tw_block


def UN(X, Z, N, f_block, sampling_type="SWOR"):
    """Computes complete or incomplete (depending on f_block) two-sample U-statistic on each
    worker and averages them.  Cuts the dataset X,Z in N splits.  sampling_type can be SWOR,
    prop-SWOR or prop-SWR.  (main.py:33-69)"""
    return Bk.run_un(X, Z, N, f_block, sampling_type, variant="est")


def UnN(X, Z, N, sampling_type, tie_mode="strict"):
    """Computes block-wise complete U-statistic.  (main.py:72-74)"""
    return UN(X, Z, N, _UN_HALF if tie_mode == "half" else Un, sampling_type=sampling_type)


def UnNT(X, Z, N, T, sampling_type, tie_mode="strict"):
    """Computes reshuffled block-wise complete U-statistic.  (main.py:76-79)

    The T repetitions' host halves (in-place shuffles, every RNG draw) run in the reference's
    order; their blocks are counted in ONE device launch (snapshots of the shuffled samples),
    so a small UnNT costs one round trip instead of T."""
    spec = (_UN_HALF if tie_mode == "half" else _UN_STRICT)._tw_block
    v = Bk.run_un_repeated(X, Z, N, spec, sampling_type, "est", T)
    if v is not None:
        return v
    return np.mean([UnN(X, Z, N, sampling_type=sampling_type, tie_mode=tie_mode)
                    for _ in range(T)])


def replicate(estimator, gen_X, gen_Z, n_tries, *args, flush_elems=1 << 24, **kwargs):
    """``[estimator(gen_X(), gen_Z(), *args, **kwargs) for _ in range(n_tries)]`` — the
    Monte-Carlo loops of main.py:106-112 — with identical results and identical NumPy RNG
    consumption, but the pair counts of many tries evaluated in one device launch.

    estimator: Un, UnN or UnNT of this module.  The host side (gen_X/gen_Z, the in-place
    shuffles, every RNG draw) runs in exactly the reference's order; the shuffled samples of
    pending tries are snapshotted and counted in batches of about `flush_elems` scores.
    """
    tie_mode = kwargs.pop("tie_mode", "strict")
    if kwargs:
        raise TypeError(f"unexpected keyword arguments {sorted(kwargs)}")
    spec = (_UN_HALF if tie_mode == "half" else _UN_STRICT)._tw_block
    if estimator is Un:
        reps = 1
        N = sampling_type = None
    elif estimator is UnN:
        N, sampling_type = args
        reps = 1
    elif estimator is UnNT:
        N, T, sampling_type = args
        reps = T
    else:
        raise ValueError("replicate supports estimation.Un, UnN and UnNT")
    if estimator is Un or (sampling_type.startswith("prop") and sampling_type != "prop-SWR"):
        # the fixed-layout plans (Un's one block; prop-SWOR's N blocks of fixed sizes, no RNG
        # draw in the plan): tries batched into preallocated snapshot rows, no per-block Python
        return _replicate_fixed(estimator, gen_X, gen_Z, n_tries, spec, reps, N,
                                sampling_type, flush_elems)
    return _replicate_general(estimator, gen_X, gen_Z, n_tries, spec, reps, N, sampling_type,
                              flush_elems)


def _replicate_general(estimator, gen_X, gen_Z, n_tries, spec, reps, N, sampling_type,
                       flush_elems):
    """replicate() for any plan: per try and repetition, plan_un's shuffles and draws, a
    snapshot and its blocks; the pending tries' blocks counted in one launch per flush."""
    results = []
    pending = []  # (try index, [(plan, job) per repetition])
    jobs = []
    size = 0

    def flush():
        nonlocal jobs, pending, size
        vals = Bk.evaluate_many(spec, jobs)
        j = 0
        for _, plans in pending:
            per_rep = []
            for plan in plans:
                if plan is None:  # Un: one whole block, value as is
                    per_rep.append(vals[j][0])
                else:
                    per_rep.append(Bk.finish_un(plan, vals[j]))
                j += 1
            results.append(per_rep[0] if estimator is not UnNT else np.mean(per_rep))
        jobs, pending, size = [], [], 0

    for t in range(n_tries):
        X = np.asarray(gen_X())
        Z = np.asarray(gen_Z())
        plans = []
        for _ in range(reps):
            if estimator is Un:
                jobs.append((X, Z, [Bk.whole(X, Z)]))
                plans.append(None)
            else:
                plan = Bk.plan_un(X, Z, N, spec, sampling_type, "est")
                blocks = [p[1] for p in plan if p[0] == "val"]
                jobs.append((X.copy(), Z.copy(), blocks))  # later repetitions reshuffle X, Z
                plans.append(plan)
            size += X.size + Z.size
        pending.append((t, plans))
        if size >= flush_elems:
            flush()
    if jobs:
        flush()
    return results


def _replicate_fixed(estimator, gen_X, gen_Z, n_tries, spec, reps, N, sampling_type,
                     flush_elems):
    """replicate() for fixed-layout plans: every try's snapshot (after its in-place shuffles,
    per repetition) is copied into one row of a preallocated host buffer holding only the
    elements the blocks read; a flush counts all rows' blocks in one launch with offsets built
    by broadcasting, and the block values, each try's np.mean over its blocks and UnNT's mean
    over its repetitions are row reductions (np.mean's pairwise sums along the contiguous last
    axis, the same bits as np.mean of each row).  A flush runs on a worker thread (its upload,
    count and read-back release the GIL) while this thread draws and shuffles the next tries
    into the other of two buffer pairs; results are collected in try order.  The same draws,
    shuffles and values as the general path; a try whose shapes or dtypes differ from the last
    one's flushes first and gets its own layout."""
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor
    t = L.torch()
    dev = t.cuda.current_device() if t.cuda.is_available() else None
    results = []
    st = {"key": None}
    pending = deque()  # (future, buffer pair) in flush order
    free = []  # buffer pairs of the current layout not in flight

    def alloc(rows, cols, dtype):
        # page-locked rows on a GPU process (torch's caching host allocator keeps them for
        # the next call): the flush uploads them by DMA without a packing copy
        if dev is None:
            return np.empty((rows, cols), dtype=dtype)
        td = t.from_numpy(np.empty(0, dtype=dtype)).dtype
        return t.empty((rows, cols), dtype=td, pin_memory=True).numpy()

    def work(bx, bz, lay):
        if dev is not None:
            t.cuda.set_device(dev)
        vals = Bk.fixed_values(spec, bx, bz, lay)
        per = vals[:, 0] if N is None else vals.mean(axis=-1)  # finish_un: np.mean per plan
        per = per.reshape(bx.shape[0] // reps, reps)
        return list(per[:, 0] if reps == 1 else per.mean(axis=-1))

    def collect(keep=0):  # results of the oldest flushes, in order, until `keep` remain
        while len(pending) > keep:
            fut, pair = pending.popleft()
            results.extend(fut.result())
            if pair is not None and pair[0].shape == st.get("shape"):
                free.append(pair)

    def new_layout(X, Z):
        collect()
        free.clear()
        lay = Bk.fixed_layout(X.shape[0], Z.shape[0], N, spec, sampling_type)
        st["key"] = (X.shape, Z.shape, X.dtype, Z.dtype)
        st["lay"] = lay
        if lay is None:
            return
        lx, lz = lay[1], lay[3]
        rows = max(reps, (max(1, flush_elems // max(1, lx + lz)) // reps) * reps)
        st["shape"] = (rows, lx)
        st["bufs"] = (alloc(rows, lx, X.dtype), alloc(rows, lz, Z.dtype))
        st["rows"] = 0

    def flush(pool):
        J = st.get("rows", 0)
        if not J:
            return
        bx, bz = st["bufs"]
        pending.append((pool.submit(work, bx[:J], bz[:J], st["lay"]), (bx, bz)))
        st["rows"] = 0
        collect(keep=1)  # at most one flush in flight beside the drawing
        if free:
            st["bufs"] = free.pop()
        else:
            lx, lz = st["lay"][1], st["lay"][3]
            rows = st["shape"][0]
            st["bufs"] = (alloc(rows, lx, bx.dtype), alloc(rows, lz, bz.dtype))

    with ThreadPoolExecutor(max_workers=1) as pool:
        for _ in range(n_tries):
            X = np.asarray(gen_X())
            Z = np.asarray(gen_Z())
            if (X.shape, Z.shape, X.dtype, Z.dtype) != st["key"] or X.ndim != 1 or Z.ndim != 1:
                flush(pool)
                if X.ndim != 1 or Z.ndim != 1:
                    collect()
                    st["key"], st["lay"] = None, None
                else:
                    new_layout(X, Z)
            if st.get("lay") is None:  # this try by the general path (its own launch)
                collect()
                results.extend(_replicate_general(estimator, iter([X]).__next__,
                                                  iter([Z]).__next__, 1, spec, reps, N,
                                                  sampling_type, 0))
                continue
            lx, lz = st["lay"][1], st["lay"][3]
            bx, bz = st["bufs"]
            for _ in range(reps):
                if N is not None:
                    Bk.shuffle_pair(X, Z)  # plan_un's in-place shuffles, bit for bit
                r = st["rows"]
                bx[r] = X[:lx]
                bz[r] = Z[:lz]
                st["rows"] = r + 1
            if st["rows"] == bx.shape[0]:
                flush(pool)
        flush(pool)
        collect()
    return results
