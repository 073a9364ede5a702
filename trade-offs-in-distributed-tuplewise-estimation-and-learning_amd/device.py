"""Device-resident sharded estimation.

The drop-in functions (tuplewise.estimation / tuplewise.compute_stats) keep the reference's
host-side NumPy shuffle so their results are bit-identical to it.  This module is the
production path behind them for data that lives on the GPU(s): the samples stay in HBM, each
repartition is a keyed pseudo-random bijection evaluated on the device (Feistel, csrc/
permute.hip), and all shards are counted in one launch.

Multi-GPU (one process per GPU, torch.distributed over RCCL): rank r holds n_loc X-scores
and m_loc Z-scores and owns shards [r*N, (r+1)*N) of the global prop-SWOR layout.  A
repartition draws ONE global permutation of the G*n_loc X-scores (and of the Z-scores);
every element is sent to the rank owning its new position with a single all-to-all(v) of
{value, position} records, and the receiver scatters them into place.  The resulting global
array — hence every shard's integer count and the final np.mean — is identical for any G.
Per-shard counts are combined with one all-reduce (sum of a zero-padded int64 vector; exact).
UnN_many on rank images (est.UnNT's loop, the bench's problem) walks the call's repartitions as
per-element chains of positions (csrc/chain.hip): each rank walks only its own elements, one
equal-split all-to-all per chunk of <= 32 steps moves {image, position} records to the ranks
that hold those positions, and all steps of a chunk are counted in one launch.
"""
from __future__ import annotations

import contextlib
import ctypes

import numpy as np

from . import _engine as E
from . import _lib as L

# UnN_many's all-pairs steps on rank images (csrc/rankimage.hip; A/B switch: False keeps the
# double-compare kernel of csrc/count.hip)
RANK_IMAGES = True
# UnN_many on rank images as step chains (csrc/chain.hip: every element walks the call's
# repartitions once, the steps' (step, shard) bags are counted in one launch per chunk of
# CHAIN_MAX steps; over ranks one all-to-all per chunk).  False: one launch per step that counts
# and permutes the records for the next step (csrc/rankimage.hip), the A/B baseline.
CHAIN_STEPS = True
CHAIN_MAX = 32
# algo="sorted" on the step chains: bags of at most this many z are counted exactly in
# O(n + m) on their integer rank images (tw_count_pairs_chain_bucket); larger shards keep the
# records path (tw_count_pairs_sorted_steps)
CHAIN_BUCKET_MAX = 16384
# several ranks: 0 (default) — one all-to-all per chunk, its unpack and ONE count launch
# behind it; n > 0 — the chunk's steps in sub-chunks of at most n steps (and at least two),
# each its own async all-to-all with its emission on a side stream, so one sub-chunk's exchange
# runs under the previous sub-chunk's count.  Round 5 (tools/chain_probe.py,
# profiles/r05s36_chain_probe.log): the sub-chunks' extra launches (emission, unpack, count
# tail, cross-stream waits) cost a G = 8 rank 0.05-0.09 ms per call at T = 4 and 0.13-0.15 ms
# at T = 20 — more than the exchange they hide (~0.03 / ~0.08 ms over xGMI)
CHAIN_SUB = 0
# UnN_many on the step chains carries the rank-image records of the final arrays to the next
# call: a repartition permutes the sample and never changes its multiset, so the images (ranks
# against the whole Z) stay valid while the arrays are the ones the chains left — the next call
# skips the ranking (and over ranks the Z all-gather it waits for).  Any assignment of X / Z or
# an in-place change (the tensors' version counters) drops them.
CARRY_IMAGES = True
# over ranks, a chain call's final arrays and carried records by ONE exchange of the walked
# elements to the owners of their final positions (tw_chain_final_pack / _scatter), instead of
# all-gathers of both samples and both record arrays and inverse-chain gathers from them
FINAL_EXCHANGE = True
# ... forked at the call's start on positions walked without emitting (tw_chain_walk) instead
# of after the last emission: off — on one GPU the walk and pack beside the emissions cost more
# than they hide (profiles/r06s22_chain_probe.log), and over RCCL the exchange's all-to-all
# issued first would queue ahead of the chunks' on the communicator
FINAL_EARLY = False
# one process: the call's final scatters (scores and carried records, memory-bound) on a side
# stream beside the last chunk's count (VALU-bound) instead of after it — when that count is
# short (<= FINAL_BESIDE_MAX_STEPS steps): its blocks, starved beside a long count, hold wave
# slots the count needs (K = 4 1.994 -> 1.957 ms per call, K = 20 8.878 -> 8.946,
# profiles/r06s33_ab_final_scatter.log)
FINAL_BESIDE_COUNT = True
FINAL_BESIDE_MAX_STEPS = 8
# UnNB_many over ranks on the step chains (one exchange per chunk of CHAIN_MAX steps, bags at
# exact positions, tw_count_pairs_chain_rng) instead of one repartition exchange per step
CHAIN_RNG = True
# one-shot all-pairs counts (local_counts: est.Un / UnN without a repartition loop) on rank
# images from this many pairs on; below, the double-compare kernel (no ranking to amortise)
ONESHOT_RANK = True
ONESHOT_RANK_MIN_PAIRS = 1 << 32


def prop_swor_layout(n_X: int, n_Z: int, N: int):
    """Block bounds of UN(..., sampling_type="prop-SWOR") on already-shuffled arrays
    (compute_stats.py:70-87 / estimation-experiment/main.py:45-64): k = int(n_X/N) X-scores
    and tau-k Z-scores per block, consumed from the front, clamped at the array ends.
    Returns (x_off, z_off, keep) where keep[s] is False for degenerate blocks (k in (0, tau)),
    which the est variant skips."""
    tau = int((n_X + n_Z) / N)
    k = int(n_X / N)
    x_off = [0]
    z_off = [0]
    keep = []
    for _ in range(N):
        x_off.append(min(x_off[-1] + k, n_X))
        z_off.append(min(z_off[-1] + (tau - k), n_Z))
        keep.append(k not in (0, tau))
    return np.array(x_off, np.int64), np.array(z_off, np.int64), np.array(keep, bool)


class HipOps:
    """The device operations of a repartition step, bound to libtuplewise.so."""

    def __init__(self):
        self.t = L.torch()

    def perm_index(self, n, base, n_total, key):
        out = L.empty((n,), self.t.int64)
        L.call("tw_perm_index", L.ptr(out), int(n), int(base), int(n_total), int(key),
               L.stream_handle())
        return out

    def permute(self, vals, key):
        out = self.t.empty_like(vals)
        L.call("tw_permute_scatter", L.ptr(vals), L.ptr(out), int(vals.numel()), int(key),
               L.stream_handle())
        return out

    def permute_pair(self, X, kx, Z, kz):
        Xo, Zo = self.t.empty_like(X), self.t.empty_like(Z)
        L.call("tw_permute_pair", L.ptr(X), L.ptr(Xo), int(X.numel()), int(kx), L.ptr(Z),
               L.ptr(Zo), int(Z.numel()), int(kz), L.stream_handle())
        return Xo, Zo

    def rank_histogram(self, perm, n_loc, G):
        out = L.empty((G,), self.t.int64)
        L.call("tw_rank_histogram", L.ptr(perm), int(perm.numel()), int(n_loc), int(G),
               L.ptr(out), L.stream_handle())
        return out

    def source_histogram(self, n, base, n_total, key, n_loc, G):
        out = L.empty((G,), self.t.int64)
        L.call("tw_source_histogram", int(n), int(base), int(n_total), int(key), int(n_loc),
               int(G), L.ptr(out), L.stream_handle())
        return out

    def bucket_scatter(self, perm, vals, n_loc, G, start, send, pos_base):
        cursor = L.empty((G,), self.t.int64)
        L.call("tw_bucket_scatter", L.ptr(perm), L.ptr(vals), int(perm.numel()), int(n_loc),
               int(G), L.ptr(start), L.ptr(cursor), int(pos_base), L.ptr(send),
               L.stream_handle())
        return send

    def exchange_counts(self, n_loc, m_loc, rank, G, key_x, key_z):
        """(4G,) counts [send X | receive X | send Z | receive Z] and the pack cursors."""
        counts = L.empty((4 * G,), self.t.int64)
        cursor = L.empty((2 * G,), self.t.int64)
        L.call("tw_exchange_counts", int(n_loc), int(m_loc), int(rank), int(G), int(key_x),
               int(key_z), L.ptr(counts), L.ptr(cursor), L.stream_handle())
        return counts, cursor

    def exchange_pack(self, X, Z, rank, G, key_x, key_z, counts, cursor):
        send = self.t.empty((X.numel() + Z.numel(), 2), dtype=self.t.int64, device=X.device)
        L.call("tw_exchange_pack", L.ptr(X), int(X.numel()), L.ptr(Z), int(Z.numel()),
               int(rank), int(G), int(key_x), int(key_z), L.ptr(counts), L.ptr(cursor),
               L.ptr(send), L.stream_handle())
        return send

    def exchange_pack_fixed(self, X, Z, rank, G, key_x, key_z, cap, cursor, send, flag):
        L.call("tw_exchange_pack_fixed", L.ptr(X), int(X.numel()), L.ptr(Z), int(Z.numel()),
               int(rank), int(G), int(key_x), int(key_z), int(cap), L.ptr(cursor), L.ptr(send),
               L.ptr(flag), L.stream_handle())
        return send

    def scatter_buckets(self, recv, G, cap, out, flag):
        L.call("tw_scatter_buckets", L.ptr(recv), int(G), int(cap), L.ptr(out), int(out.numel()),
               L.ptr(flag), L.stream_handle())
        return out

    def scatter_records(self, rec, out):
        L.call("tw_scatter_records", L.ptr(rec), int(rec.shape[0]), L.ptr(out),
               L.stream_handle())
        return out

    def count(self, x, x_off_dev, z, z_off_dev, n_shards, max_nx, max_nz, dtype, pred,
              algo="pairs"):
        return E.count_launch(x, x_off_dev, z, z_off_dev, int(n_shards), int(max_nx),
                              int(max_nz), int(dtype), int(pred), algo)

    def count_step(self, x, x_off_dev, z, z_off_dev, n_shards, max_nx, max_nz, dtype, pred,
                   out, x_next, key_x, z_next, key_z, out_next):
        """Counts of the current partition into `out` (already zero) and, in the same launch,
        the next repartition into x_next / z_next and zeroing of out_next (tw_count_pairs_step)."""
        L.call("tw_count_pairs_step", L.ptr(x), L.ptr(x_off_dev), L.ptr(z), L.ptr(z_off_dev),
               int(n_shards), int(max_nx), int(max_nz), int(dtype), int(pred), L.ptr(out),
               int(x.numel()), L.ptr(x_next), int(key_x), int(z.numel()), L.ptr(z_next),
               int(key_z), L.ptr(out_next), int(out_next.numel()) if out_next is not None else 0,
               L.stream_handle())
        return out

    def rank_images(self, X, Z, dtype):
        """Rank-image records of both samples (tw_rank_images, csrc/rankimage.hip): int64
        tensors whose low word is the f32 image and high word the score's index; None where
        the path does not apply (n_z >= 2^24)."""
        n, m = int(X.numel()), int(Z.numel())
        wb = int(L.lib().tw_rank_images_work_bytes(n, m))
        if wb < 0:
            return None
        work = L.empty((max(wb, 1),), self.t.uint8)
        xr = L.empty((n,), self.t.int64)
        zr = L.empty((m,), self.t.int64)
        L.call("tw_rank_images", L.ptr(X), n, L.ptr(Z), m, int(dtype), L.ptr(work), wb,
               L.ptr(xr), L.ptr(zr), L.stream_handle())
        return xr, zr

    def count_rank_step(self, xr, x_off_dev, zr, z_off_dev, n_shards, max_nx, max_nz, out,
                        x_next, key_x, z_next, key_z, out_next):
        """tw_count_pairs_step on rank-image records (tw_count_pairs_rank_step): the counts of
        the current partition into `out` (already zero), the next repartition of the records
        into x_next / z_next and the zeroing of out_next in the same launch."""
        L.call("tw_count_pairs_rank_step", L.ptr(xr), L.ptr(x_off_dev), L.ptr(zr),
               L.ptr(z_off_dev), int(n_shards), int(max_nx), int(max_nz), L.ptr(out),
               int(xr.numel()), L.ptr(x_next), int(key_x), int(zr.numel()), L.ptr(z_next),
               int(key_z), L.ptr(out_next), int(out_next.numel()) if out_next is not None else 0,
               L.stream_handle())
        return out

    def gather_records(self, vals, rec):
        """The scores in record order (tw_gather_records): out[p] = vals[rec[p] >> 32]."""
        out = self.t.empty(rec.shape, dtype=vals.dtype, device=rec.device)
        L.call("tw_gather_records", L.ptr(vals), L.ptr(rec), int(rec.numel()), L.ptr(out),
               L.stream_handle())
        return out

    def rank_images_query(self, Z_all, X, Z, dtype, half=False, compact=False):
        """Rank-image records of this rank's X and Z counted against the Z of Z_all
        (tw_rank_images_query); half: the X records' high word is h(x) = #{z <= x}; compact:
        images without indices (x float32, or int64 {g, h} pairs when half; z float32), the bag
        layout of count_chain.  None where the path does not apply (|Z_all| >= 2^24)."""
        n, m, ma = int(X.numel()), int(Z.numel()), int(Z_all.numel())
        wb = int(L.lib().tw_rank_images_work_bytes(n, ma))
        if wb < 0 or n + m >= (1 << 31):
            return None
        t, dev = self.t, X.device
        work = t.empty((max(wb, 1),), dtype=t.uint8, device=dev)
        xr = t.empty((n,), dtype=t.float32 if compact and not half else t.int64, device=dev)
        zr = t.empty((m,), dtype=t.float32 if compact else t.int64, device=dev)
        L.call("tw_rank_images_query", L.ptr(Z_all), ma, L.ptr(X), n, L.ptr(Z), m, int(dtype),
               int(bool(half)) | (int(bool(compact)) << 1), L.ptr(work), wb, L.ptr(xr),
               L.ptr(zr), L.stream_handle())
        return xr, zr

    def chain_emit(self, xr, zr, half, xpos, zpos, first, rank, world, keys_x, keys_z, kx, kz,
                   n_shards, x_bag=None, z_bag=None, cursors=None, send=None, cap=0, flag=None):
        """Walk len(keys_x) repartitions for this rank's elements (tw_chain_emit): into the
        step bags (one process) or the send buckets (several ranks)."""
        kxa = np.ascontiguousarray(keys_x, dtype=np.uint64)
        kza = np.ascontiguousarray(keys_z, dtype=np.uint64)
        L.call("tw_chain_emit", L.ptr(xr), int(xr.numel()), L.ptr(zr), int(zr.numel()),
               int(bool(half)), L.ptr(xpos), L.ptr(zpos), int(bool(first)), int(rank),
               int(world), kxa.ctypes.data, kza.ctypes.data, len(kxa), int(kx), int(kz),
               int(n_shards), L.ptr(x_bag), L.ptr(z_bag), L.ptr(cursors), L.ptr(send),
               int(cap), L.ptr(flag), L.stream_handle())

    def chain_unpack(self, recv, world, steps, cap, half, n, m, x_bag, z_bag, flag, kx, kz,
                     n_shards):
        """The received records appended to their (step, shard) bags (tw_chain_unpack)."""
        cur = self._unpack_cursors(int(steps) * 2 * (int(n_shards) + 1), x_bag.device)
        L.call("tw_chain_unpack", L.ptr(recv), int(world), int(steps), int(cap),
               int(bool(half)), int(n), int(m), int(kx), int(kz), int(n_shards), L.ptr(x_bag),
               L.ptr(z_bag), L.ptr(cur), L.ptr(flag), L.stream_handle())

    def chain_unpack_count(self, recv, world, steps, cap, half, n, m, x_bag, z_bag, flag, kx,
                           kz, n_shards, x_off_dev, z_off_dev, max_nx, max_nz, out):
        """chain_unpack then count_chain in ONE native call (tw_chain_unpack_count): the
        cursors and counts zeroed by one launch, the three launches back to back."""
        cur = self._unpack_cursors(int(steps) * 2 * (int(n_shards) + 1), x_bag.device)
        L.call("tw_chain_unpack_count", L.ptr(recv), int(world), int(steps), int(cap),
               int(bool(half)), int(n), int(m), int(kx), int(kz), int(n_shards), L.ptr(x_bag),
               L.ptr(z_bag), L.ptr(cur), L.ptr(flag), L.ptr(x_off_dev), L.ptr(z_off_dev),
               int(max_nx), int(max_nz), L.ptr(out), L.stream_handle())
        return out

    def chain_final_pack(self, X, xr, xpos, Z, zr, zpos, world, cap, cursor, send, flag):
        """The walked elements into their final positions' buckets (tw_chain_final_pack)."""
        L.call("tw_chain_final_pack", L.ptr(X), L.ptr(xr), L.ptr(xpos), int(X.numel()), L.ptr(Z),
               L.ptr(zr), L.ptr(zpos), int(Z.numel()), int(world), int(cap), L.ptr(cursor),
               L.ptr(send), L.ptr(flag), L.stream_handle())

    def chain_walk(self, x_base, n, NX, z_base, m, NZ, keys_x, keys_z, xpos, zpos):
        """The final positions of the rank's elements after the keys' steps, without emitting
        (tw_chain_walk): the chain state tw_chain_emit leaves after the same steps."""
        kxa = np.ascontiguousarray(keys_x, dtype=np.uint64)
        kza = np.ascontiguousarray(keys_z, dtype=np.uint64)
        L.call("tw_chain_walk", int(x_base), int(n), int(NX), int(z_base), int(m), int(NZ),
               kxa.ctypes.data, kza.ctypes.data, len(kxa), L.ptr(xpos), L.ptr(zpos),
               L.stream_handle())

    def chain_final_scatter(self, recv, world, cap, n, m, Xo, XRo, Zo, ZRo, flag):
        """The received final records at their positions (tw_chain_final_scatter)."""
        L.call("tw_chain_final_scatter", L.ptr(recv), int(world), int(cap), int(n), int(m),
               L.ptr(Xo), L.ptr(XRo), L.ptr(Zo), L.ptr(ZRo), L.ptr(flag), L.stream_handle())

    def chain_unpack_exact(self, recv, world, steps, cap, n, m, x_bag, z_bag, flag):
        """The received records written at their exact positions of the step bags
        (tw_chain_unpack_exact): the bags are the steps' permuted image arrays."""
        L.call("tw_chain_unpack_exact", L.ptr(recv), int(world), int(steps), int(cap), int(n),
               int(m), L.ptr(x_bag), L.ptr(z_bag), L.ptr(flag), L.stream_handle())

    def count_chain_rng(self, x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps, x_stride,
                        z_stride, max_nx, max_nz, B, seed, shard_base, out):
        """B device-drawn pairs per (step, shard) bag of exact-position images
        (tw_count_pairs_chain_rng): step c keyed seed + c, shard streams shard_base + s —
        the draws of count_rng on the same permuted arrays; out (steps, n_shards)."""
        L.call("tw_count_pairs_chain_rng", L.ptr(x_bag), L.ptr(x_off_dev), int(x_stride),
               L.ptr(z_bag), L.ptr(z_off_dev), int(z_stride), int(n_shards), int(steps),
               int(max_nx), int(max_nz), int(B), int(seed) & (2 ** 64 - 1), int(shard_base),
               L.ptr(out), L.stream_handle())
        return out

    def _unpack_cursors(self, words, dev):
        # one buffer per HipOps, grown as needed; unpacks on one stream reuse it in order
        c = getattr(self, "_cursors", None)
        if c is None or c.numel() < words:
            self._cursors = c = self.t.empty((max(words, 1024),), dtype=self.t.int32, device=dev)
        return c

    def count_chain(self, x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps, x_stride,
                    z_stride, max_nx, max_nz, half, out):
        """Counts of steps x n_shards bags in one launch into out (steps, n_shards)."""
        L.call("tw_count_pairs_chain", L.ptr(x_bag), L.ptr(x_off_dev), int(x_stride),
               L.ptr(z_bag), L.ptr(z_off_dev), int(z_stride), int(n_shards), int(steps),
               int(max_nx), int(max_nz), int(bool(half)), L.ptr(out), L.stream_handle())
        return out

    def count_chain_bucket(self, x_bag, x_off_dev, z_bag, z_off_dev, n_shards, steps,
                           x_stride, z_stride, max_nz, z_total, half, out):
        """The exact O(n + m) counts of steps x n_shards bags (tw_count_pairs_chain_bucket,
        bags of <= CHAIN_BUCKET_MAX z) into out (steps, n_shards)."""
        L.call("tw_count_pairs_chain_bucket", L.ptr(x_bag), L.ptr(x_off_dev), int(x_stride),
               L.ptr(z_bag), L.ptr(z_off_dev), int(z_stride), int(n_shards), int(steps),
               int(max_nz), int(z_total), int(bool(half)), L.ptr(out), L.stream_handle())
        return out

    def chain_scatter(self, X, xpos, Z, zpos):
        Xo, Zo = self.t.empty_like(X), self.t.empty_like(Z)
        L.call("tw_chain_scatter", L.ptr(X), L.ptr(xpos), int(X.numel()), L.ptr(Z),
               L.ptr(zpos), int(Z.numel()), L.ptr(Xo), L.ptr(Zo), L.stream_handle())
        return Xo, Zo

    def chain_gather(self, X_all, Z_all, x_base, n, z_base, m, keys_x, keys_z, X2=None,
                     Z2=None):
        """The rank's final arrays: the inverse chains of its own positions, gathered from the
        all-gathered samples (tw_chain_gather); with X2 / Z2 (laid out like X_all / Z_all:
        the carried records) also theirs, from the same walk (tw_chain_gather2)."""
        kxa = np.ascontiguousarray(keys_x, dtype=np.uint64)
        kza = np.ascontiguousarray(keys_z, dtype=np.uint64)
        dev = X_all.device
        Xo = self.t.empty((n,), dtype=X_all.dtype, device=dev)
        Zo = self.t.empty((m,), dtype=Z_all.dtype, device=dev)
        work = self.t.empty((max(1, n + m),), dtype=self.t.int32, device=dev)
        if X2 is None:
            L.call("tw_chain_gather", L.ptr(X_all), L.ptr(Z_all), int(x_base), int(n),
                   int(X_all.numel()), int(z_base), int(m), int(Z_all.numel()), kxa.ctypes.data,
                   kza.ctypes.data, len(kxa), L.ptr(work), L.ptr(Xo), L.ptr(Zo),
                   L.stream_handle())
            return Xo, Zo
        X2o = self.t.empty((n,), dtype=X2.dtype, device=dev)
        Z2o = self.t.empty((m,), dtype=Z2.dtype, device=dev)
        L.call("tw_chain_gather2", L.ptr(X_all), L.ptr(Z_all), L.ptr(X2), L.ptr(Z2), int(x_base),
               int(n), int(X_all.numel()), int(z_base), int(m), int(Z_all.numel()),
               kxa.ctypes.data, kza.ctypes.data, len(kxa), L.ptr(work), L.ptr(Xo), L.ptr(Zo),
               L.ptr(X2o), L.ptr(Z2o), L.stream_handle())
        return Xo, Zo, X2o, Z2o

    def count_rng(self, x, x_off_dev, z, z_off_dev, n_shards, B, seed, shard_base, dtype, pred,
                  max_nx=None, max_nz=None):
        """Device-RNG incomplete counts.  With the shard bounds known, the ranked kernels
        (16-bit rank codes in LDS, csrc/rankcount.hip) run; same draws, same integers."""
        out = L.empty((n_shards,), self.t.int64)
        wb = 0
        if max_nx is not None and max_nz is not None:
            wb = int(L.lib().tw_count_pairs_rng_work_bytes(int(n_shards), int(max_nx),
                                                           int(max_nz), int(dtype), int(pred)))
        if wb > 0:
            work = L.empty((wb,), self.t.uint8)
            L.call("tw_count_pairs_rng_ws", L.ptr(x), L.ptr(x_off_dev), L.ptr(z),
                   L.ptr(z_off_dev), int(n_shards), int(max_nx), int(max_nz), int(B), int(seed),
                   int(shard_base), int(dtype), int(pred), L.ptr(work), wb, L.ptr(out),
                   L.stream_handle())
        else:
            L.call("tw_count_pairs_rng", L.ptr(x), L.ptr(x_off_dev), L.ptr(z), L.ptr(z_off_dev),
                   int(n_shards), int(B), int(seed), int(shard_base), int(dtype), int(pred),
                   L.ptr(out), L.stream_handle())
        return out

    def count_sorted_step(self, x, x_off_dev, z, z_off_dev, n_shards, max_nx, max_nz, dtype,
                          pred, out, x_next, key_x, z_next, key_z, out_next):
        """Exact sorted counts of the current partition into `out` (already zero) and the next
        repartition into x_next / z_next with out_next zeroed, in one launch on the bucket
        path (tw_count_pairs_sorted_step)."""
        work = L.empty((max(1, int(L.lib().tw_count_pairs_sorted_work_bytes(int(n_shards),
                                                                             int(max_nz)))),),
                       self.t.uint8)
        L.call("tw_count_pairs_sorted_step", L.ptr(x), L.ptr(x_off_dev), L.ptr(z),
               L.ptr(z_off_dev), int(n_shards), int(max_nx), int(max_nz), int(dtype), int(pred),
               L.ptr(work), L.ptr(out), int(x.numel()), L.ptr(x_next), int(key_x),
               int(z.numel()), L.ptr(z_next), int(key_z), L.ptr(out_next),
               int(out_next.numel()) if out_next is not None else 0, L.stream_handle())
        return out

    def count_sorted_steps(self, X, Z, x_off_dev, z_off_dev, n_shards, kx, kz, max_nx, max_nz,
                           dtype, pred, keys):
        """T UnN steps with the exact sorted count, the partition kept as destination-bucketed
        records between steps (tw_count_pairs_sorted_steps): returns the (T, N) counts and
        the last partition's arrays, or None where the records path does not apply."""
        t = self.t
        n, m = int(X.numel()), int(Z.numel())
        wb = int(L.lib().tw_count_pairs_sorted_steps_work_bytes(n, m, int(n_shards),
                                                                int(max_nz), int(dtype),
                                                                int(pred)))
        if wb <= 0:
            return None
        work = L.empty((wb,), t.uint8)
        out = L.empty((len(keys), int(n_shards)), t.int64)
        Xo, Zo = t.empty_like(X), t.empty_like(Z)
        kxs = np.array([(2 * k) & (2 ** 64 - 1) for k in keys], dtype=np.uint64)
        kzs = np.array([(2 * k + 1) & (2 ** 64 - 1) for k in keys], dtype=np.uint64)
        L.call("tw_count_pairs_sorted_steps", L.ptr(X), L.ptr(Z), n, m, L.ptr(x_off_dev),
               L.ptr(z_off_dev), int(n_shards), int(kx), int(kz), int(max_nx), int(max_nz),
               int(dtype), int(pred), kxs.ctypes.data, kzs.ctypes.data, len(keys), L.ptr(work),
               wb, L.ptr(out), L.ptr(Xo), L.ptr(Zo), L.stream_handle())
        return out, Xo, Zo

    def count_rng_step(self, x, x_off_dev, z, z_off_dev, n_shards, B, seed, shard_base, dtype,
                       pred, max_nx, max_nz, out, x_next, key_x, z_next, key_z, out_next):
        """Device-RNG incomplete counts of the current partition into `out` (already zero) and
        the next repartition into x_next / z_next with out_next zeroed, in one launch where the
        float32-image kernel applies (tw_count_pairs_rng_step)."""
        wb = int(L.lib().tw_count_pairs_rng_work_bytes(int(n_shards), int(max_nx), int(max_nz),
                                                       int(dtype), int(pred)))
        work = L.empty((max(wb, 1),), self.t.uint8)
        L.call("tw_count_pairs_rng_step", L.ptr(x), L.ptr(x_off_dev), L.ptr(z),
               L.ptr(z_off_dev), int(n_shards), int(max_nx), int(max_nz), int(B), int(seed),
               int(shard_base), int(dtype), int(pred), L.ptr(work), wb, L.ptr(out),
               int(x.numel()), L.ptr(x_next), int(key_x), int(z.numel()), L.ptr(z_next),
               int(key_z), L.ptr(out_next),
               int(out_next.numel()) if out_next is not None else 0, L.stream_handle())
        return out

    def checksum_acc_words(self):
        return int(L.lib().tw_words_checksum_acc_words())

    def words_checksum(self, A, B, acc, expect=None, verdict=None, good=1, bad=0):
        """acc (one int64) = the position-keyed hash of [A | B]'s 8-byte words
        (tw_words_checksum, csrc/guard.hip); with expect / verdict: verdict = good when acc ==
        expect, else bad, in stream order.  verdict may be pinned host memory (written through
        its device mapping, read by the host after the stream's next synchronisation)."""
        vp = None
        if verdict is not None:
            vp = (ctypes.c_void_p(L.host_device_pointer(verdict)) if not verdict.is_cuda
                  else L.ptr(verdict))
            if vp.value is None:
                raise L.TuplewiseError("words_checksum: the verdict word is not mapped memory")
        L.call("tw_words_checksum", L.ptr(A), int(A.numel()), L.ptr(B), int(B.numel()),
               L.ptr(acc), L.ptr(expect), vp, int(good), int(bad), L.stream_handle())
        return acc

    def to_dev(self, arr):
        return L.to_device(arr)


class _StaleImages(RuntimeError):
    """The carried rank images no longer describe the arrays: a write torch's version counter
    did not see (through `.data`, a DLPack alias, a foreign kernel).  UnN_many recounts the call
    from a fresh ranking when it catches this (every rank together over ranks)."""


class ShardedSample:
    """Two-sample scores resident on this rank's GPU, cut into N local prop-SWOR shards.

    X, Z: this rank's 1-D tensors (float64 or int64; all ranks the same sizes and dtype).
    group: a torch.distributed process group (None = single process).
    tie_mode: "strict" (reference) or "half" (ties score 1/2).
    algo: "pairs" (all-pairs compare kernel), "sorted" (sort + binary search, same integers),
    "auto" (sorted for large shards).
    exchange (several ranks): "fixed" (equal-size buckets, one permutation pass, no host round
    trip per repartition) or "exact" (counted buckets: a count pass, the inverse permutation and
    a host copy of the split sizes).  Both give the same arrays.
    collectives: None (default) = the collective branches (exchange, all-gathers, all-reduce of
    the counts) exactly when the group has several ranks; True forces them on a world-size-1
    group too (every RCCL call of the multi-rank path then runs on one GPU; same integers, same
    arrays as the one-process path); False is refused with several ranks."""

    # X / Z: every assignment drops the step chains' carried images (CARRY_IMAGES)
    @property
    def X(self):
        return self._X

    @X.setter
    def X(self, v):
        self._X = v
        self._carry = None

    @property
    def Z(self):
        return self._Z

    @Z.setter
    def Z(self, v):
        self._Z = v
        self._carry = None

    def _carried(self, half):
        """(xr, zr, checksum): the records {image, ...} of the current own elements carried
        from the last chain call and the hash of the arrays they describe, or None.  Valid while
        X / Z are the tensors that call left (same objects, same version counters) with the same
        tie mode; a write the version counters miss is caught by the checksum, verified in the
        stream of the call that reuses them (_unn_many_chain)."""
        c = getattr(self, "_carry", None)
        if not CARRY_IMAGES or c is None:
            return None
        X, Z, vx, vz, h, xr, zr, cs = c
        if (X is self._X and Z is self._Z and X._version == vx and Z._version == vz
                and h == half):
            return xr, zr, cs
        return None

    def _checksum(self, expect=None, verdict=None, good=1, bad=0):
        """A one-word device hash of the current X / Z (None where the ops lack the entry);
        with expect / verdict, also the verdict word (see HipOps.words_checksum)."""
        if not hasattr(self.ops, "words_checksum"):
            return None
        return self._hash_pair(self.X, self.Z, expect, verdict, good, bad)

    def _hash_pair(self, X, Z, expect=None, verdict=None, good=1, bad=0):
        """_checksum of the arrays X / Z (None where the ops lack the entry)."""
        if not hasattr(self.ops, "words_checksum"):
            return None
        accs = getattr(self, "_acc_bufs", None)
        if accs is None or accs[0].device != X.device:
            words = int(getattr(self.ops, "checksum_acc_words", lambda: 1)())
            accs = self._acc_bufs = [self.t.empty((words,), dtype=self.t.int64,
                                                  device=X.device) for _ in range(3)]
            self._acc_next = 0
        if verdict is not None:  # a check: its sums are consumed by the verdict word
            acc = accs[2]
        else:  # a saved hash (the next call's `expect`): two buffers taken in turn
            acc = accs[self._acc_next]
            self._acc_next ^= 1
        return self.ops.words_checksum(X, Z, acc, expect, verdict, good, bad)[:1]

    def _host_verdict(self):
        """The pinned (device-mapped) host word the one-process verdict is written into."""
        v = getattr(self, "_verdict", None)
        if v is None:
            t = self.t
            v = self._verdict = (t.empty((1,), dtype=t.int64, pin_memory=True) if self.X.is_cuda
                                 else t.empty((1,), dtype=t.int64))
            self._verdict_np = v.numpy()  # (a host write through NumPy: no torch dispatch)
        self._verdict_np[0] = -1
        return v

    def __init__(self, X, Z, N: int, group=None, tie_mode: str = "strict", ops=None,
                 algo: str = "auto", exchange: str = "fixed", collectives=None):
        if exchange not in ("fixed", "exact"):
            raise ValueError(f"exchange must be 'fixed' or 'exact', not {exchange!r}")
        self.exchange = exchange
        self._xf = None
        self.ops = ops if ops is not None else HipOps()
        t = L.torch()
        self.t = t
        self.group = group
        if group is not None:
            import torch.distributed as dist
            self.dist = dist
            self.G = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        else:
            self.dist = None
            self.G, self.rank = 1, 0
        self.coll = (L.collectives_default(group, self.G) if collectives is None
                     else bool(collectives))
        if self.coll and group is None:
            raise ValueError("collectives=True needs a process group")
        if self.G > 1 and not self.coll:
            raise ValueError("several ranks always take the collective branches")
        self._flag_all = None  # the ranks' overflow flags, summed by the last counts reduction
        self._carry_all = None  # the ranks' carried-images bits, summed by the same reduction
        if X.dtype == t.float64:
            self.dtype = L.TW_F64
        elif X.dtype == t.int64:
            self.dtype = L.TW_I64
        else:
            raise TypeError("ShardedSample holds float64 or int64 scores")
        if Z.dtype != X.dtype:
            raise TypeError("X and Z must share a dtype")
        self.X, self.Z = X.contiguous(), Z.contiguous()
        self.N = int(N)
        self.n_loc, self.m_loc = self.X.numel(), self.Z.numel()
        self.pred = {"strict": L.TW_PRED_GT, "half": L.TW_PRED_HALF}[tie_mode]
        self.tie_mode = tie_mode
        x_off, z_off, keep = prop_swor_layout(self.n_loc, self.m_loc, self.N)
        self.x_off, self.z_off, self.keep = x_off, z_off, keep
        self.x_off_dev = self.ops.to_dev(x_off)
        self.z_off_dev = self.ops.to_dev(z_off)
        self.max_nx = int(np.diff(x_off).max()) if N else 0
        self.max_nz = int(np.diff(z_off).max()) if N else 0
        self.pairs = np.diff(x_off).astype(object) * np.diff(z_off).astype(object)
        self.algo = E.pick_algo(algo, self.max_nx, self.max_nz, "gt")

    # ------------------------------------------------------------------ repartition
    def _repartition_multi(self, key_x, key_z):
        """Apply the global permutations (over G*n_loc X- and G*m_loc Z-scores) with ONE
        all-to-all of 16-byte records.  Send counts come from the forward permutation, receive
        counts from the inverse one, so the only host round trip of a repartition is the copy
        of the split sizes that all_to_all_single needs.  With the fused device ops
        (tw_exchange_counts / tw_exchange_pack) that is two launches; the primitive path
        (perm_index, rank/source histograms, bucket scatter) does the same in steps."""
        t, dist, G, r, ops = self.t, self.dist, self.G, self.rank, self.ops
        n, m = self.n_loc, self.m_loc
        if self.exchange == "fixed" and hasattr(ops, "exchange_pack_fixed"):
            xf = self._fixed_buffers()
            ops.exchange_pack_fixed(self.X, self.Z, r, G, key_x, key_z, xf["cap"], xf["cursor"],
                                    xf["send"], xf["flag"])
            dist.all_to_all_single(xf["recv"], xf["send"], group=self.group)
            XZ = t.empty((n + m,), dtype=self.X.dtype, device=self.X.device)
            ops.scatter_buckets(xf["recv"], G, xf["cap"], XZ, xf["flag"])
            self.X, self.Z = XZ[:n], XZ[n:]
            return
        if hasattr(ops, "exchange_counts"):  # fused: two launches, no permutation array
            cnt, cursor = ops.exchange_counts(n, m, r, G, key_x, key_z)
            send = ops.exchange_pack(self.X, self.Z, r, G, key_x, key_z, cnt, cursor)
            c = cnt.cpu().numpy().reshape(4, G)
            return self._exchange_records(send, c)
        px = ops.perm_index(n, r * n, G * n, key_x)
        pz = ops.perm_index(m, r * m, G * m, key_z)
        cnt = t.stack([ops.rank_histogram(px, n, G),
                       ops.source_histogram(n, r * n, G * n, key_x, n, G),
                       ops.rank_histogram(pz, m, G),
                       ops.source_histogram(m, r * m, G * m, key_z, m, G)])
        send_tot = cnt[0] + cnt[2]
        start_x = t.cumsum(send_tot, 0) - send_tot  # bucket g = [X records, Z records]
        start_z = start_x + cnt[0]
        send = t.empty((n + m, 2), dtype=t.int64, device=self.X.device)
        ops.bucket_scatter(px, self.X, n, G, start_x, send, 0)
        ops.bucket_scatter(pz, self.Z, m, G, start_z, send, n)  # Z positions follow X's
        c = cnt.cpu().numpy()
        return self._exchange_records(send, c)

    def _fixed_buffers(self):
        """Persistent buffers of the fixed-capacity exchange.  A bucket (records of one source
        rank for one destination) holds (n_loc + m_loc) / G records on average, with a
        hypergeometric spread of about sqrt of that; cap adds 1/8 + 1024 (dozens of standard
        deviations at any size), and an overflow is detected, never silently dropped."""
        if self._xf is None:
            t, G = self.t, self.G
            tot = self.n_loc + self.m_loc
            cap = max(1, min(tot, tot // G + tot // (8 * G) + 1024))
            dev = self.X.device
            self._xf = {"cap": cap,
                        "cursor": t.zeros((G,), dtype=t.int64, device=dev),
                        "flag": t.zeros((1,), dtype=t.int32, device=dev),
                        "send": t.empty((G * (cap + 1), 2), dtype=t.int64, device=dev),
                        "recv": t.empty((G * (cap + 1), 2), dtype=t.int64, device=dev)}
        return self._xf

    def _local_flag(self):
        """This rank's sticky overflow flags (fixed exchange + step chains) as one int64 device
        element, or None before any exchange ran."""
        fl = [f for f in ((self._xf or {}).get("flag"), getattr(self, "_chain_flag", None))
              if f is not None]
        if not fl:
            return None
        return sum(f.to(self.t.int64) for f in fl)

    def _reduce_counts(self, counts, carried=None):
        """(T, N) local counts -> (T, G*N) global counts in shard order on every rank, with the
        ranks' overflow flags summed in the SAME all-reduce (one extra element): a bucket that
        overflowed on any rank is then seen by every rank in values(), so all ranks raise
        together instead of the two involved ones only.  carried (the step
        chains): whether this rank used carried images (1; or a device verdict word: 1 when its
        checksum held, G + 1 when the arrays were written behind the version counter) — summed
        in a second extra element, so a rank whose sample changed alone (its images recomputed,
        or found stale, while the others carried theirs) makes every rank redo the call: any
        sum but 0 (nobody carried) or G (everybody carried valid images) raises _StaleImages
        in values()."""
        t, G, N, r = self.t, self.G, self.N, self.rank
        T = counts.shape[0]
        extra = 1 if carried is None else 2
        flat = t.zeros((T * G * N + extra,), dtype=t.int64, device=counts.device)
        flat[:T * G * N].view(T, G * N)[:, r * N:(r + 1) * N] = counts
        f = self._local_flag()
        if f is not None:
            flat[-1:] = f.reshape(1)
        if isinstance(carried, self.t.Tensor):  # the checksum verdict: 1 good, G + 1 stale
            flat[-2:-1] = carried
        elif carried:
            flat[-2:-1] = 1
        self.dist.all_reduce(flat, group=self.group)
        self._flag_all = flat[-1:]
        self._carry_all = None if carried is None else flat[-2:-1]
        self._flag_tail = flat[-2:]
        return flat[:T * G * N].view(T, G * N)

    def check_exchange(self):
        """Raise if a fixed-capacity repartition overflowed a bucket (host sync).  The flag is
        sticky: records past a bucket's capacity were dropped, so the arrays stay invalid for
        every later step of this sample (a later repartition only permutes them).  Over ranks
        the flag read is the ranks' sum from the last counts all-reduce, so every rank raises."""
        carry_sum = None
        if self._carry_all is not None:  # both extra elements of the reduction in one read
            carry_sum, flag_sum = (int(v) for v in self._flag_tail.cpu().tolist())
            if flag_sum:
                raise RuntimeError("repartition: an exchange bucket on some rank overflowed "
                                   "its capacity; the counts and arrays are invalid")
        elif self._flag_all is not None and int(self._flag_all.item()):
            raise RuntimeError("repartition: an exchange bucket on some rank overflowed its "
                               "capacity; the counts and arrays are invalid")
        if self._xf is not None and int(self._xf["flag"].item()):
            raise RuntimeError("repartition: an exchange bucket overflowed its capacity; the "
                               "arrays are invalid (use ShardedSample(..., exchange='exact'))")
        if getattr(self, "_chain_flag", None) is not None and int(self._chain_flag.item()):
            raise RuntimeError("UnN_many: a step-chain bucket overflowed its capacity; the "
                               "counts and arrays are invalid")
        if carry_sum is not None and carry_sum not in (0, self.G):
            raise _StaleImages("UnN_many: the ranks disagree on the carried rank images (a "
                               "rank's sample was changed on that rank alone, or written behind "
                               "its version counter); the call is recounted")

    def _exchange_records(self, send, c):
        """All-to-all of the packed records (split sizes from the (4, G) host counts) and the
        scatter into one [X | Z] array."""
        t, dist = self.t, self.dist
        n, m = self.n_loc, self.m_loc
        sc = (c[0] + c[2]).tolist()
        rc = (c[1] + c[3]).tolist()
        if sum(rc) != n + m:
            raise RuntimeError(f"repartition: {sum(rc)} records expected for {n + m} positions")
        recv = t.empty_like(send)
        dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc,
                               group=self.group)
        XZ = t.empty((n + m,), dtype=self.X.dtype, device=self.X.device)
        self.ops.scatter_records(recv, XZ)
        self.X, self.Z = XZ[:n], XZ[n:]

    def _multi(self) -> bool:
        """The exchange path: several ranks, or a world-size-1 group with collectives=True."""
        return self.coll

    def repartition(self, key: int, check: bool = True):
        """One repartition: new random shards for both samples (key = any 64-bit integer).
        With several ranks and the fixed-capacity exchange, check=True waits for the exchange
        and raises if a bucket overflowed on any rank (one small all-reduce of the flags, so
        every rank raises together), so X and Z are never read corrupt; the pipelined
        estimators pass check=False (no host sync per step) and check once in values()."""
        self._repartition(key)
        if check and self._multi():
            f = self._local_flag()
            if f is not None:
                f = f.reshape(1).clone()
                self.dist.all_reduce(f, group=self.group)
                self._flag_all = f
                self._carry_all = None  # (this reduction carries no carried-images bit)
            self.check_exchange()

    def _repartition(self, key: int):
        kx, kz = (key * 2) & (2 ** 64 - 1), (key * 2 + 1) & (2 ** 64 - 1)
        if not self._multi():
            self.X, self.Z = self.ops.permute_pair(self.X, kx, self.Z, kz)
        else:
            self._repartition_multi(kx, kz)

    # ------------------------------------------------------------------ estimation
    def local_counts(self):
        """Per-local-shard exact counts (int64 device tensor; uint64 semantics).  Large all-pairs
        counts (est.Un at BASELINE configs[1]: 1e10 pairs in one shard) rank X u Z once and count
        packed f32 images (tw_rank_images_query compact + tw_count_pairs_chain, one step): the
        ranking costs less than the double compares it replaces."""
        if self.algo == "pairs" and self._oneshot_rank_ok():
            half = self.pred == L.TW_PRED_HALF
            xi, zi = self.ops.rank_images_query(self.Z, self.X, self.Z, self.dtype, half,
                                                compact=True)
            out = self.t.empty((1, self.N), dtype=self.t.int64, device=self.X.device)
            self.ops.count_chain(xi, self.x_off_dev, zi, self.z_off_dev, self.N, 1,
                                 self.n_loc, self.m_loc, self.max_nx, self.max_nz, half, out)
            return out[0]
        return self.ops.count(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                              self.max_nx, self.max_nz, self.dtype, self.pred, algo=self.algo)

    def _oneshot_rank_ok(self) -> bool:
        """One-shot counts on rank images: the step-chain predicates, a device sample of fewer
        than 2^24 Z-scores, and at least ONESHOT_RANK_MIN_PAIRS pairs."""
        return (ONESHOT_RANK and RANK_IMAGES and self.X.is_cuda and self.N > 0
                and self.max_nx > 0 and self.max_nz > 0
                and hasattr(self.ops, "rank_images_query") and hasattr(self.ops, "count_chain")
                and (self.pred in (L.TW_PRED_GT, L.TW_PRED_HALF)
                     or (self.pred == L.TW_PRED_SUBGT and self.dtype == L.TW_F64))
                and self.m_loc < (1 << 24) and self.n_loc + self.m_loc < (1 << 31)
                and int(sum(self.pairs)) >= ONESHOT_RANK_MIN_PAIRS)

    def global_counts(self, local):
        """All G*N shard counts, in global shard order, on every rank (one all-reduce, the
        ranks' overflow flags riding along)."""
        if not self.coll:
            return local
        return self._reduce_counts(local.reshape(1, -1))[0]

    def values(self, counts, pairs=None) -> np.ndarray:
        """Block values count / #pairs of the kept shards, in global shard order: each one
        float64(count) / float64(pairs), as the reference's np.mean of a 0/1 array gives.
        counts: (G*N,) or (T, G*N); returns an array of the same rank.  pairs: the pairs per
        shard (default: all pairs of each shard; B for the incomplete statistic)."""
        c = np.asarray(counts.cpu().numpy()).view(np.uint64)
        self.check_exchange()
        # the denominators and kept shards of this layout, built once per (pairs, tie mode):
        # this runs after the call's device work, on its critical path
        ck = (pairs, self.tie_mode, self.G, self.N)
        cache = self.__dict__.setdefault("_den_cache", {})
        ent = cache.get(ck)
        if ent is None:
            keep = np.tile(self.keep, self.G)
            scale = 2 if self.tie_mode == "half" else 1
            per = np.tile(self.pairs, self.G) if pairs is None else [pairs] * (self.G * self.N)
            # uint64 -> float64 and Python int -> float are both correctly rounded, like E.ratio
            den = np.array([float(scale * int(p)) for p in per])
            ent = cache[ck] = (keep, den)
        keep, den = ent
        return (c.astype(np.float64) / den)[..., keep]

    @staticmethod
    def _row_means(vals) -> list:
        """np.mean of each row (the per-step estimates): one reduction over the last,
        contiguous axis — the same pairwise sums as np.mean of each row alone."""
        return list(np.ascontiguousarray(vals).mean(axis=-1))

    def UnN(self, key=None) -> np.float64:
        """Block-wise complete U-statistic over all G*N shards (est.UnN with prop-SWOR,
        estimation-experiment/main.py:72-74); repartitions first when key is given."""
        if key is not None:
            self.repartition(key)
        return np.mean(self.values(self.global_counts(self.local_counts())))

    def _run_steps(self, keys, count_local, fusable, step=None, count_into=None):
        """One repartition + one count of all local shards per key, with no host round trip
        per step; returns the (T, G*N) device counts in global shard order (one all-reduce).
        One GPU and a one-launch step (step(i, out, X_next, key_x, Z_next, key_z, out_next):
        tw_count_pairs_step for the all-pairs count, tw_count_pairs_rng_step for the
        device-RNG incomplete count): each launch counts step i and repartitions both samples
        for step i+1.  Several GPUs: repartition i+1 (pack kernels, the split-size copy, the
        RCCL all-to-all) is issued on a side stream while the counts of step i run.
        count_local(i) enqueues step i's count on the current stream; fusable: the all-pairs
        count (its multi-GPU launches accumulate into one zeroed buffer) — count_into(out) its
        launch into a zeroed row (default: tw_count_pairs_step without a next step)."""
        t = self.t
        local = []
        if not self._multi() and step is not None:
            # each launch counts step i and repartitions for step i+1
            self._repartition(keys[0])
            out = t.zeros((self.N,), dtype=t.int64, device=self.X.device)
            for i in range(len(keys)):
                last = i + 1 == len(keys)
                if last:
                    Xn = Zn = out_n = None
                    kx = kz = 0
                else:
                    Xn, Zn = t.empty_like(self.X), t.empty_like(self.Z)
                    out_n = t.empty((self.N,), dtype=t.int64, device=self.X.device)
                    kx = (keys[i + 1] * 2) & (2 ** 64 - 1)
                    kz = (keys[i + 1] * 2 + 1) & (2 ** 64 - 1)
                step(i, out, Xn, kx, Zn, kz, out_n)
                local.append(out)
                if not last:
                    self.X, self.Z, out = Xn, Zn, out_n
        elif not self._multi():
            for i, k in enumerate(keys):
                self._repartition(k)
                local.append(count_local(i))
        else:
            main = t.cuda.current_stream()
            if getattr(self, "_side", None) is None:
                # high priority: the exchange's small kernels get CU slots as soon as count
                # blocks retire (normal priority: 1.13 ms/step, high: 1.00, one-GPU path 0.88
                # on the world-size-1 probe, tools/multi_path_probe.py)
                self._side = t.cuda.Stream(priority=-1)
            side = self._side

            def repartition_on_side(k):
                self.X.record_stream(side)  # old arrays are read on side before being dropped
                self.Z.record_stream(side)
                with t.cuda.stream(side):
                    self._repartition(k)

            # all-pairs counts go into one buffer zeroed up front: one count launch per step
            # on main, no per-step fill kernel between the counts
            pre = None
            if count_into is None and fusable and hasattr(self.ops, "count_step"):
                def count_into(row):
                    self.ops.count_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                        self.max_nx, self.max_nz, self.dtype, self.pred, row,
                                        None, 0, None, 0, None)
            if count_into is not None:
                pre = t.zeros((len(keys), self.N), dtype=t.int64, device=self.X.device)
            side.wait_stream(main)
            repartition_on_side(keys[0])
            for i in range(len(keys)):
                main.wait_stream(side)  # repartition i (only it is queued on side so far)
                if pre is not None:
                    count_into(pre[i])
                    local.append(pre[i])
                else:
                    local.append(count_local(i))
                self.X.record_stream(main)  # allocated on side, read by this count on main
                self.Z.record_stream(main)
                if i + 1 < len(keys):
                    repartition_on_side(keys[i + 1])
            main.wait_stream(side)
        counts = t.stack(local)  # (T, N)
        if self.coll:
            counts = self._reduce_counts(counts)
        return counts

    def UnN_many(self, keys) -> list:
        """[UnN(k) for k in keys], in order, with identical values (est.UnNT's loop,
        estimation-experiment/main.py:76-79), pipelined as _run_steps describes."""
        keys = list(keys)
        if not keys:
            return []
        if not self.X.is_cuda and not (self.algo == "pairs" and self._chain_ok()):
            # host tensors (CPU rehearsal of the orchestration): the stream-pipelined paths
            # need a device; the step chains (no side stream) run as they are
            return [self.UnN(k) for k in keys]
        if self.algo == "pairs" and self._chain_ok():
            return self._unn_many_chain(keys)
        if (self.algo == "sorted" and self._chain_ok() and self.max_nz <= CHAIN_BUCKET_MAX
                and hasattr(self.ops, "count_chain_bucket")):
            # the step chains with the exact bucket count of each bag (row f4)
            return self._unn_many_chain(keys, bucket=True)
        if (self.algo == "sorted" and not self._multi() and self.N > 0
                and hasattr(self.ops, "count_sorted_steps")):
            # the whole sequence in one call: records between steps (csrc/records.h)
            n, m = self.n_loc, self.m_loc
            kx = int(n / self.N)
            r = self.ops.count_sorted_steps(self.X, self.Z, self.x_off_dev, self.z_off_dev,
                                            self.N, kx, int((n + m) / self.N) - kx,
                                            self.max_nx, self.max_nz, self.dtype, self.pred,
                                            keys)
            if r is not None:
                counts, self.X, self.Z = r
                return self._row_means(self.values(counts))
        fusable = self.algo == "pairs"
        if fusable and self._rank_path_ok():
            r = self._unn_many_rank(keys)
            if r is not None:
                return r
        step = None
        if fusable and hasattr(self.ops, "count_step"):
            def step(i, out, Xn, kx, Zn, kz, out_n):
                self.ops.count_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                    self.max_nx, self.max_nz, self.dtype, self.pred, out, Xn, kx,
                                    Zn, kz, out_n)
        elif (self.algo == "sorted" and self.pred != L.TW_PRED_SUBGT
              and hasattr(self.ops, "count_sorted_step")):
            def step(i, out, Xn, kx, Zn, kz, out_n):
                self.ops.count_sorted_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                           self.max_nx, self.max_nz, self.dtype, self.pred, out,
                                           Xn, kx, Zn, kz, out_n)
        counts = self._run_steps(keys, lambda i: self.local_counts(), fusable, step)
        return self._row_means(self.values(counts))

    def _rank_path_ok(self) -> bool:
        """The all-pairs steps on rank images (csrc/rankimage.hip) apply to the strict
        predicate (SUBGT on doubles is the same predicate; int64 SUBGT wraps and stays on the
        score compare) with fewer than 2^24 Z-scores in all."""
        G = self.G
        return (RANK_IMAGES and self.N > 0 and self.max_nx > 0
                and self.max_nz > 0 and hasattr(self.ops, "rank_images")
                and (self.pred == L.TW_PRED_GT
                     or (self.pred == L.TW_PRED_SUBGT and self.dtype == L.TW_F64))
                and G * self.m_loc < (1 << 24) and G * (self.n_loc + self.m_loc) < (1 << 31))

    def _chain_ok(self) -> bool:
        """The step chains (csrc/chain.hip) take the rank-image predicates and half ties, with
        positions in 32 bits and at most 8191 shards per rank (the emission's LDS buckets)."""
        G = self.G
        return (CHAIN_STEPS and RANK_IMAGES and self.N > 0 and self.max_nx > 0
                and self.max_nz > 0 and hasattr(self.ops, "chain_emit")
                and (self.pred in (L.TW_PRED_GT, L.TW_PRED_HALF)
                     or (self.pred == L.TW_PRED_SUBGT and self.dtype == L.TW_F64))
                and G * self.m_loc < (1 << 24) and G * (self.n_loc + self.m_loc) < (1 << 31)
                and self.N < 8191 and G <= 512)

    def _chain_rng_ok(self) -> bool:
        """UnNB_many on the step chains (several ranks, or forced collectives): CHAIN_RNG, the
        step-chain predicates with the strict predicate (one 4-B image per score at its exact
        position), and a shard's images within a CU's LDS (tw_count_pairs_chain_rng)."""
        al4 = (self.max_nx + 3) & ~3
        return (CHAIN_RNG and self._chain_ok() and hasattr(self.ops, "count_chain_rng")
                and (self.pred == L.TW_PRED_GT
                     or (self.pred == L.TW_PRED_SUBGT and self.dtype == L.TW_F64))
                and (al4 + self.max_nz) * 4 <= 160 * 1024 - 1024)

    def _unn_many_rank(self, keys):
        """UnN_many on rank images, one launch per step (the A/B baseline of the step chains):
        ONE ranking of X u Z per call (the multiset of scores is the same at every step), then
        one launch per step that counts the current partition on packed f32 images and permutes
        the 8-B records {image, index} for the next step (the same keyed permutations as the
        score path); the scores are gathered into the final order once at the end.  Same counts,
        same arrays as the score path."""
        if self.coll:
            # several ranks: every rank ranks the WHOLE sample (one all-gather of both samples
            # per call), keeps its own elements' records (high words: global indices) and the
            # exchanges move 8-B records as they moved scores
            X0, Z0 = self._all_gather(self.X), self._all_gather(self.Z)
            r = self.ops.rank_images(X0, Z0, self.dtype)
            if r is None:
                return None
            a, b = self.rank * self.n_loc, self.rank * self.m_loc
            self.X, self.Z = r[0][a:a + self.n_loc].clone(), r[1][b:b + self.m_loc].clone()
        else:
            r = self.ops.rank_images(self.X, self.Z, self.dtype)
            if r is None:
                return None
            X0, Z0 = self.X, self.Z
            self.X, self.Z = r

        def step(i, out, Xn, kx, Zn, kz, out_n):
            self.ops.count_rank_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                     self.max_nx, self.max_nz, out, Xn, kx, Zn, kz, out_n)

        def count_into(row):
            self.ops.count_rank_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                     self.max_nx, self.max_nz, row, None, 0, None, 0, None)
        try:
            counts = self._run_steps(keys, None, True, step, count_into)
        finally:
            xr, zr = self.X, self.Z
            self.X = self.ops.gather_records(X0, xr)
            self.Z = self.ops.gather_records(Z0, zr)
        return self._row_means(self.values(counts))

    def _unn_many_chain(self, keys, bucket=False, rng=None):
        """_chain_call, recounted once from a fresh ranking when the carried images turn out
        stale (_StaleImages: the arrays were written where torch's version counters do not
        see, or over ranks some rank dropped its images): the call's inputs are still the
        arrays it started from, so the recount gives the call's true estimates and arrays."""
        X_in, Z_in = self._X, self._Z
        try:
            return self._chain_call(keys, bucket, True, rng)
        except _StaleImages:
            self._X, self._Z, self._carry = X_in, Z_in, None
            self.stale_recounts = getattr(self, "stale_recounts", 0) + 1
            return self._chain_call(keys, bucket, False, rng)

    def _chain_call(self, keys, bucket, use_carry, rng=None):
        """UnN_many as step chains (csrc/chain.hip; est.UnNT's loop, estimation-experiment/
        main.py:76-79).  One ranking per call: over ranks the Z structure of the all-gathered Z,
        images written for this rank's own elements only.  Then per chunk of <= CHAIN_MAX steps
        every own element walks the chunk's repartitions (one forward Feistel per step) and its
        image lands in the (step, shard) bag holding its position — directly in one process,
        through ONE equal-split all-to-all of {image, position} records over ranks — and one
        launch counts all bags of the chunk.  The final arrays: a scatter by the chains' last
        positions (one process) or the inverse chains of the rank's own positions gathered from
        the all-gathered sample.  Same permutation chain, counts and final arrays as the
        one-launch-per-step paths, at any G.  bucket: the bags counted exactly in O(n + m) on
        their integer images (algo="sorted") instead of all pairs — the same integers.
        rng = (B, seed): the incomplete statistic (UnNB_many over ranks, cs.UnNBT's loop,
        compute_stats.py:119-123): the received records are written at their EXACT positions
        (tw_chain_unpack_exact) — the device draws address positions — and B pairs per bag are
        drawn and counted on the images (tw_count_pairs_chain_rng, step t keyed seed + t), the
        integers of count_rng on the same permuted arrays."""
        t, ops, G, r = self.t, self.ops, self.G, self.rank
        n, m, N = self.n_loc, self.m_loc, self.N
        dev = self.X.device
        half = self.pred == L.TW_PRED_HALF
        coll = self.coll  # the exchange branch (several ranks, or forced at world size 1)
        works = []  # the asynchronous all-gathers the final arrays wait for
        rec = self._carried(half) if use_carry else None
        carried = rec is not None
        verdict = None
        if carried:
            # the hash of the arrays now against the one saved with the images, verified in
            # stream order: over ranks the verdict rides in the counts' all-reduce, in one
            # process it lands in a pinned host word read after the counts
            xr, zr, cs = rec
            rec = (xr, zr)
            if cs is not None:
                verdict = (self.t.empty((1,), dtype=self.t.int64, device=self.X.device) if coll
                           else self._host_verdict())
                if self.X.is_cuda:
                    # on a side stream beside the emission (both only read): joined before the
                    # counts' reduction / the host's read of the verdict
                    if getattr(self, "_guard_stream", None) is None:
                        self._guard_stream = self.t.cuda.Stream()
                    gs = self._guard_stream
                    gs.wait_stream(self.t.cuda.current_stream())
                    with self.t.cuda.stream(gs):
                        self._checksum(cs, verdict, 1, self.G + 1 if coll else 0)
                    if coll:
                        verdict.record_stream(gs)  # (made on the main stream, written on gs)
                else:
                    self._checksum(cs, verdict, 1, self.G + 1 if coll else 0)
        # over ranks the call's final arrays and carried records come by ONE exchange of the
        # walked elements to the ranks holding their final positions (FINAL_EXCHANGE,
        # tw_chain_final_pack / _scatter) instead of the all-gathers of X and of both record
        # arrays and the inverse-chain gathers from them
        fin_x = coll and FINAL_EXCHANGE and hasattr(ops, "chain_final_pack")
        X0 = Z0 = None
        if coll:
            # the ranking needs the whole Z now (unless the images are carried); without the
            # final exchange the whole X (and Z) only for the final arrays (chain_gather), so
            # those all-gathers run asynchronously under the chunks' counts
            # (every rank gathers Z, carried or not: a rank whose sample changed alone ranks
            # afresh while the others carry, and the ranks' collectives must stay one sequence)
            if not carried:
                Z0 = self._all_gather(self.Z)
            else:
                Z0, w = self._all_gather(self.Z, async_op=True)
                works.append(w)
            if not fin_x:
                X0, w = self._all_gather(self.X, async_op=True)
                works.append(w)
        else:
            X0, Z0 = self.X, self.Z
        if not carried:
            rec = ops.rank_images_query(Z0, self.X, self.Z, self.dtype, half)
        if rec is None:
            for w in works:
                w.wait()
            return [self.UnN(k) for k in keys]
        xr, zr = rec
        RX = RZ = None
        if coll and CARRY_IMAGES and not fin_x:
            # the records follow their elements: gathered by the same inverse chains as the
            # scores, from every rank's records (asynchronous, under the counts)
            RX, w = self._all_gather(xr, async_op=True)
            works.append(w)
            RZ, w = self._all_gather(zr, async_op=True)
            works.append(w)
        T = len(keys)
        C = min(T, CHAIN_MAX)
        M64 = 2 ** 64 - 1
        kxs = [(2 * k) & M64 for k in keys]
        kzs = [(2 * k + 1) & M64 for k in keys]
        final = None
        if coll and self.X.is_cuda and not fin_x:
            # the final arrays depend on the keys and the all-gathered sample only: gathered on
            # a side stream beside the emission, exchanges and counts (not after them)
            main = t.cuda.current_stream()
            if getattr(self, "_final_stream", None) is None:
                self._final_stream = t.cuda.Stream()
            fs = self._final_stream
            fs.wait_stream(main)
            with t.cuda.stream(fs):
                for w in works:
                    if w is not None:
                        w.wait()
                works = []
                final = ops.chain_gather(X0, Z0, r * n, n, r * m, m, kxs, kzs, RX, RZ)
                for a in final:
                    a.record_stream(main)
        early = fin_x and FINAL_EARLY and hasattr(ops, "chain_walk")
        if early:
            # the final positions walked without emitting (tw_chain_walk), so the final
            # exchange forks now, beside the whole call's emissions and counts (its all-to-all
            # is issued before the chunks' on every rank: one collective order)
            final = self._final_exchange(xr, zr, walk=(kxs, kzs))
        kx = int(n / N)
        kz = int((n + m) / N) - kx  # prop_swor_layout's shard sizes
        z_total = G * m  # the Z the images were ranked against: images <= z_total

        def count(xb, zb, steps, out, t0):  # bags of steps t0.. -> out (steps, N)
            if rng is not None:
                ops.count_chain_rng(xb, self.x_off_dev, zb, self.z_off_dev, N, steps, n, m,
                                    self.max_nx, self.max_nz, rng[0], rng[1] + t0, r * N, out)
            elif bucket:
                ops.count_chain_bucket(xb, self.x_off_dev, zb, self.z_off_dev, N, steps, n, m,
                                       self.max_nz, z_total, half, out)
            else:
                ops.count_chain(xb, self.x_off_dev, zb, self.z_off_dev, N, steps, n, m,
                                self.max_nx, self.max_nz, half, out)
        x_bag = self._work("x_bag", (C, n), t.int64 if half else t.float32)
        z_bag = self._work("z_bag", (C, m), t.float32)
        xpos = self._work("xpos", (n,), t.int32)
        zpos = self._work("zpos", (m,), t.int32)
        counts = t.empty((T, N), dtype=t.int64, device=dev)
        if coll:
            # one all-to-all per chunk (CHAIN_SUB = 0), or the chunk's steps in sub-chunks of
            # <= CHAIN_SUB steps, each with its own send / receive buffers and its own async
            # all-to-all: every sub-chunk's emission is enqueued first, then each sub-chunk
            # waits for its records, unpacks and counts
            tot = n + m
            cap = max(1, tot // G + tot // (8 * G) + 1024)
            W = 2 if half else 1
            Sub = max(1, min(CHAIN_SUB, -(-C // 2))) if CHAIN_SUB > 0 else C
            nsub = -(-C // Sub)
            # the send / receive ring persists on the sample across calls (fresh
            # GB-scale allocations per call made the caching allocator flush and re-map)
            rk = (G, Sub, cap, W, nsub)
            ring = getattr(self, "_chain_ring", None)
            if ring is None or ring[0] != rk:
                self._chain_ring = None  # release the old ring first
                sends = [t.empty((G * Sub * (cap + 1) * W,), dtype=t.int64, device=dev)
                         for _ in range(nsub)]
                self._chain_ring = ring = (rk, sends, [t.empty_like(b) for b in sends])
            sends, recvs = ring[1], ring[2]
            if getattr(self, "_chain_flag", None) is None:
                self._chain_flag = t.zeros((1,), dtype=t.int32, device=dev)
        else:
            cursors = self._work("cursors", (C * 2 * (N + 1),), t.int32)
        scattered = None  # one process: the final scatters forked beside the last count
        for i0 in range(0, T, C):
            c = min(C, T - i0)
            if coll:
                # with sub-chunks, the emissions (and the all-to-alls issued behind them) on a
                # side stream, so sub-chunk j+1's emission runs beside sub-chunk j's count; the
                # side stream first waits for the main stream (the previous chunk's unpacks and
                # counts are done with these send / receive buffers)
                es = None
                if self.X.is_cuda and c > Sub:
                    if getattr(self, "_emit_stream", None) is None:
                        self._emit_stream = t.cuda.Stream()
                    es = self._emit_stream
                    es.wait_stream(t.cuda.current_stream())
                xchg = []
                with (t.cuda.stream(es) if es is not None else contextlib.nullcontext()):
                    for j, a in enumerate(range(0, c, Sub)):
                        cs = min(Sub, c - a)
                        ops.chain_emit(xr, zr, half, xpos, zpos, i0 == 0 and a == 0, r, G,
                                       kxs[i0 + a:i0 + a + cs], kzs[i0 + a:i0 + a + cs], kx, kz,
                                       N, send=sends[j], cap=cap, flag=self._chain_flag)
                        sz = G * cs * (cap + 1) * W
                        xchg.append((a, cs, j, self._all_to_all(recvs[j][:sz], sends[j][:sz],
                                                                async_op=True)))
                    emitted = None
                    if fin_x and not early and i0 + c >= T and self.X.is_cuda:
                        # the final exchange (enqueued after the last count) waits for this
                        # event only: the chains' final positions, not the counts
                        emitted = t.cuda.Event()
                        emitted.record()
                for a, cs, j, work in xchg:
                    if work is not None:
                        work.wait()
                    if rng is None and not bucket and hasattr(ops, "chain_unpack_count"):
                        # the receive side in one native call (unpack + count)
                        ops.chain_unpack_count(recvs[j], G, cs, cap, half, n, m, x_bag[a:a + cs],
                                               z_bag[a:a + cs], self._chain_flag, kx, kz, N,
                                               self.x_off_dev, self.z_off_dev, self.max_nx,
                                               self.max_nz, counts[i0 + a:i0 + a + cs])
                        continue
                    if rng is not None:
                        ops.chain_unpack_exact(recvs[j], G, cs, cap, n, m, x_bag[a:a + cs],
                                               z_bag[a:a + cs], self._chain_flag)
                    else:
                        ops.chain_unpack(recvs[j], G, cs, cap, half, n, m, x_bag[a:a + cs],
                                         z_bag[a:a + cs], self._chain_flag, kx, kz, N)
                    count(x_bag[a:a + cs], z_bag[a:a + cs], cs, counts[i0 + a:i0 + a + cs],
                          i0 + a)
                if fin_x and not early and i0 + c >= T:
                    # the walked elements' final positions are known once the call's last
                    # emission ran: their exchange runs on a side stream beside the last
                    # chunk's count — enqueued AFTER that count, so the host's work for it
                    # never delays the count's launch (the collectives keep one order: the
                    # chunk's all-to-all was issued first on every rank)
                    final = self._final_exchange(xr, zr, xpos, zpos, emitted)
                continue
            ops.chain_emit(xr, zr, half, xpos, zpos, i0 == 0, 0, 1, kxs[i0:i0 + c],
                           kzs[i0:i0 + c], kx, kz, N, x_bag=x_bag, z_bag=z_bag,
                           cursors=cursors)
            fork = None
            if (FINAL_BESIDE_COUNT and i0 + c >= T and c <= FINAL_BESIDE_MAX_STEPS
                    and self.X.is_cuda):
                fork = t.cuda.Event()  # the chains' final positions are written
                fork.record()
            count(x_bag, z_bag, c, counts[i0:i0 + c], i0)
            if fork is not None:
                # the final scatters (memory-bound) beside the last count (VALU-bound), on a
                # side stream enqueued after the count's launch
                scattered = self._final_scatter(X0, Z0, xr, zr, xpos, zpos, fork)
        carry = None
        if coll:
            if final is not None:
                if self.X.is_cuda:
                    t.cuda.current_stream().wait_stream(self._final_stream)
                for w in works:  # (fin_x: the Z all-gather of a carried call, unused)
                    if w is not None:
                        w.wait()
                if fin_x and CARRY_IMAGES:
                    RX = xr  # (marks the carry: the records came with the final exchange)
            else:
                for w in works:
                    if w is not None:
                        w.wait()
                final = ops.chain_gather(X0, Z0, r * n, n, r * m, m, kxs, kzs, RX, RZ)
            self.X, self.Z = final[0], final[1]
            if RX is not None:
                carry = (final[2], final[3])
            self._join_guard()
            counts = self._reduce_counts(counts, carried=verdict if verdict is not None
                                         else carried)
        elif scattered is not None:
            t.cuda.current_stream().wait_stream(self._final_stream)
            self.X, self.Z = scattered[0][0], scattered[0][1]
            if CARRY_IMAGES:
                carry = scattered[0][2], scattered[0][3]
        else:
            self.X, self.Z = ops.chain_scatter(X0, xpos, Z0, zpos)
            if CARRY_IMAGES:
                carry = ops.chain_scatter(xr, xpos, zr, zpos)
        if not coll:
            self._join_guard()
        if carry is not None:  # after the assignments above (they drop the old ones)
            # (the hash of the new arrays: made on the final stream beside the count when the
            # scatters ran there)
            h = scattered[1] if scattered is not None else self._checksum()
            self._carry = (self._X, self._Z, self._X._version, self._Z._version, half,
                           carry[0], carry[1], h)
        # (over ranks: raises _StaleImages on a bad verdict sum)
        vals = self.values(counts, pairs=None if rng is None else rng[0])
        if verdict is not None and not coll and int(self._verdict_np[0]) != 1:
            raise _StaleImages("UnN_many: the sample was written behind its version counter; "
                               "the carried rank images are stale")
        return self._row_means(vals)

    def _final_scatter(self, X0, Z0, xr, zr, xpos, zpos, fork):
        """One process: the final arrays and (CARRY_IMAGES) the carried records scattered by
        the chains' last positions (tw_chain_scatter) on the final stream, after `fork` (an
        event behind the last emission): (X, Z[, X records, Z records]), recorded for the main
        stream, which waits for the final stream before using them."""
        t = self.t
        main = t.cuda.current_stream()
        if getattr(self, "_final_stream", None) is None:
            self._final_stream = t.cuda.Stream()
        fs = self._final_stream
        fs.wait_event(fork)
        h = None
        with t.cuda.stream(fs):
            out = self.ops.chain_scatter(X0, xpos, Z0, zpos)
            if CARRY_IMAGES:
                out = out + self.ops.chain_scatter(xr, xpos, zr, zpos)
                h = self._hash_pair(out[0], out[1])  # the carried images' guard hash
            for a in out + ((h,) if h is not None else ()):
                a.record_stream(main)
        return out, h

    def _join_guard(self):
        """The main stream after the guard stream's verdict hash (a no-op without one)."""
        gs = getattr(self, "_guard_stream", None)
        if gs is not None:
            self.t.cuda.current_stream().wait_stream(gs)

    def _final_exchange(self, xr, zr, xpos=None, zpos=None, es=None, walk=None):
        """The call's final arrays over ranks (FINAL_EXCHANGE): on the final stream, this
        rank's walked elements — scores self.X / self.Z, records xr / zr — packed into G
        fixed-capacity buckets of 24-B records by their final positions (tw_chain_final_pack),
        ONE equal-split all-to-all, and every received record written at its position
        (tw_chain_final_scatter): (X, Z, X records, Z records) of the rank's final positions,
        recorded for the main stream.  The final positions: walk = (keys_x, keys_z), the
        call's chains walked here without emitting (tw_chain_walk, at the call's start), or
        xpos / zpos, the chain state after the call's last emission (`es`: the stream it ran
        on, or an event recorded after it)."""
        t, G, n, m = self.t, self.G, self.n_loc, self.m_loc
        main = t.cuda.current_stream() if self.X.is_cuda else None
        tot = n + m
        cap = max(1, tot // G + tot // (8 * G) + 1024)
        send = self._work("fin_send", (G * (cap + 1) * 3,), t.int64)
        recv = self._work("fin_recv", (G * (cap + 1) * 3,), t.int64)
        if getattr(self, "_chain_flag", None) is None:
            self._chain_flag = t.zeros((1,), dtype=t.int32, device=self.X.device)
        if main is None:
            fs = None
        else:
            if getattr(self, "_final_stream", None) is None:
                self._final_stream = t.cuda.Stream()
            fs = self._final_stream
            if isinstance(es, t.cuda.Event):  # the last emission's completion (enqueued later)
                fs.wait_event(es)
            else:
                fs.wait_stream(main)
                if es is not None:
                    fs.wait_stream(es)
        with (t.cuda.stream(fs) if fs is not None else contextlib.nullcontext()):
            # the cursors (zero on entry, left zero by the pack): made on the final stream, so
            # their zeroing is ordered before the pack whatever that stream waits for
            cur = getattr(self, "_fin_cursor", None)
            if cur is None or cur.numel() != G:
                cur = self._fin_cursor = t.zeros((G,), dtype=t.int64, device=self.X.device)
            if walk is not None:
                xpos = self._work("fin_xpos", (n,), t.int32)
                zpos = self._work("fin_zpos", (m,), t.int32)
                self.ops.chain_walk(self.rank * n, n, G * n, self.rank * m, m, G * m, walk[0],
                                    walk[1], xpos, zpos)
            self.ops.chain_final_pack(self.X, xr, xpos, self.Z, zr, zpos, G, cap, cur, send,
                                      self._chain_flag)
            self._all_to_all(recv, send)
            out = (t.empty_like(self.X), t.empty_like(self.Z), t.empty_like(xr),
                   t.empty_like(zr))
            self.ops.chain_final_scatter(recv, G, cap, n, m, out[0], out[2], out[1], out[3],
                                         self._chain_flag)
            if fs is not None:
                for a in out:
                    a.record_stream(main)
        return out

    def _work(self, name, shape, dtype):
        """A work tensor of `shape` kept on the sample across calls (one flat buffer per name,
        grown when a call needs more): the chains' bags, positions and cursors.  Every call
        ends with the counts read back (values()), so the next call finds them free.  Fresh
        per-call bags (80 MB each at K = 20) beside the smaller cached blocks of shorter calls
        made the caching allocator map new memory inside a call: the bench's K = 20 call ran
        0.2-0.3 ms longer than the same call after another K = 20 call (profiles/r05s50_*)."""
        # the view of the last request of each name is kept: a call repeating it (the usual
        # case) costs one dict lookup (host time before a call's first launch is device idle)
        views = self.__dict__.setdefault("_wsv", {})
        v = views.get(name)
        if v is not None and v[0] == shape and v[1] == dtype and v[2] == self.X.device:
            return v[3]
        ws = self.__dict__.setdefault("_ws", {})
        numel = 1
        for d in shape:
            numel *= int(d)
        buf = ws.get(name)
        dev = self.X.device
        if buf is None or buf.numel() < numel or buf.dtype != dtype or buf.device != dev:
            ws[name] = None  # release the old buffer first
            views.pop(name, None)
            buf = ws[name] = self.t.empty((max(numel, 1),), dtype=dtype, device=dev)
        out = buf[:numel].view(shape)
        views[name] = (tuple(shape), dtype, dev, out)
        return out

    def _all_to_all(self, out, inp, async_op=False):
        """Equal-split all-to-all of one flat tensor (RCCL all_to_all_single; gloo on CPU);
        async_op: returns the work handle (its wait() orders the caller's stream after it)."""
        return self.dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)

    def _all_gather(self, A, async_op=False):
        """The G ranks' local arrays concatenated in rank order (one collective); async_op:
        (out, work) — work.wait() orders the caller's stream after it."""
        t, dist = self.t, self.dist
        out = t.empty((self.G * A.numel(),), dtype=A.dtype, device=A.device)
        if dist.get_backend(self.group) == "nccl":
            w = dist.all_gather_into_tensor(out, A.contiguous(), group=self.group,
                                            async_op=async_op)
        else:
            w = dist.all_gather(list(out.chunk(self.G)), A.contiguous(), group=self.group,
                                async_op=async_op)
        return (out, w) if async_op else out

    def UnNT(self, T: int, key0: int = 0) -> np.float64:
        """T repartitions, averaged (est.UnNT, estimation-experiment/main.py:76-79)."""
        return np.mean(self.UnN_many(range(key0, key0 + T)))

    def _count_rng(self, B, seed):
        return self.ops.count_rng(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N, B,
                                  seed, self.rank * self.N, self.dtype, self.pred,
                                  max_nx=self.max_nx, max_nz=self.max_nz)

    def UnNB(self, B: int, seed: int, key=None) -> np.float64:
        """Block-wise incomplete U-statistic with B device-drawn pairs per shard
        (cs.UnNB(kernel="AUC"), compute_stats.py:104-110, device-RNG mode)."""
        if key is not None:
            self.repartition(key)
        counts = self.global_counts(self._count_rng(B, seed))
        return np.mean(self.values(counts, pairs=B))

    def UnNB_many(self, B: int, seed: int, keys) -> list:
        """[UnNB(B, seed + t, key_t) for t, key_t in enumerate(keys)]: T repartitions, each
        with fresh device draws (cs.UnNBT's loop, compute_stats.py:119-123), pipelined like
        UnN_many."""
        keys = list(keys)
        seeds = [(seed + i) & (2 ** 64 - 1) for i in range(len(keys))]
        if not keys:
            return []
        if self.coll and self._chain_rng_ok():
            # over ranks: the step chains, one exchange per chunk (device.py _chain_call)
            return self._unn_many_chain(keys, rng=(int(B), seeds[0]))
        if not self.X.is_cuda:
            return [self.UnNB(B, sd, k) for sd, k in zip(seeds, keys)]
        step = None
        if hasattr(self.ops, "count_rng_step"):
            def step(i, out, Xn, kx, Zn, kz, out_n):
                self.ops.count_rng_step(self.X, self.x_off_dev, self.Z, self.z_off_dev, self.N,
                                        B, seeds[i], self.rank * self.N, self.dtype, self.pred,
                                        self.max_nx, self.max_nz, out, Xn, kx, Zn, kz, out_n)
        counts = self._run_steps(keys, lambda i: self._count_rng(B, seeds[i]), False, step)
        return self._row_means(self.values(counts, pairs=B))
