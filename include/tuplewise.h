/*
 * tuplewise.h — C ABI of libtuplewise.so, the MI355X (gfx950) implementation of the
 * tuplewise hot path of "Trade-offs in Large Scale Distributed Tuplewise Estimation and
 * Learning" (reference: RobinVogel/Trade-offs-in-Distributed-Tuplewise-Estimation-and-Learning).
 *
 * The reference is pure Python/NumPy; its boundary is the `f_block(X_block, Z_block)`
 * protocol consumed by UN / UN_split (learning-experiment/compute_stats.py:44-92) and the
 * estimator functions that produce block values.  Each entry point below replaces the
 * per-shard NumPy body of one of those functions for ALL shards in one launch; the Python
 * package (tuplewise.compute_stats / tuplewise.estimation) keeps the reference names and
 * calls these through ctypes.
 *
 * Conventions
 *   - every pointer argument named d_* is DEVICE memory (hipMalloc / torch.cuda); everything
 *     else is a host scalar.  No entry point allocates, copies to/from the host, or
 *     synchronises: all work is enqueued on `stream` (a hipStream_t, NULL = default stream),
 *     so calls are graph-capturable.
 *   - shards are described by offset arrays: shard s owns elements [off[s], off[s+1]) of the
 *     concatenated input; n_shards+1 int64 entries, device memory.
 *   - dtype codes: TW_F64 (double), TW_I64 (int64).  Both sides of a call share one dtype
 *     (the Python layer applies NumPy's promotion rules first).
 *   - return value: TW_OK (0) or an error code; tw_last_error() gives a thread-local message.
 *     TW_ERR_ARG maps to the reference's AssertionError/ValueError, TW_ERR_HIP to RuntimeError.
 */
#ifndef TUPLEWISE_H
#define TUPLEWISE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TW_OK 0
#define TW_ERR_ARG 1
#define TW_ERR_HIP 2

#define TW_F64 0
#define TW_I64 1

/* Pair predicates.  TW_PRED_GT is the reference AUC kernel 1{x > z}
 * (estimation-experiment/main.py:31; compute_stats.py:19 `X - Z > 0`, identical for IEEE
 * doubles).  TW_PRED_HALF is the opt-in "+0.5 on ties" mode asked for by BASELINE.json: the
 * counter then holds half-units 2*#{x>z} + #{x==z} = #{x>z} + #{x>=z}.
 * TW_PRED_SUBGT is `(x - z) > 0` with int64 wrap-around, the literal cs.Un AUC body for int64
 * inputs (compute_stats.py:19, :30); for doubles it equals TW_PRED_GT. */
#define TW_PRED_GT 0
#define TW_PRED_HALF 1
#define TW_PRED_SUBGT 2

/* Float pair kernels of cs.Un / cs.UB_indices (compute_stats.py:15-18, :27-29) and the
 * hinge surrogate conv_AUC (compute_stats.py:129-135). */
#define TW_KERN_PROD 0  /* x * z                 */
#define TW_KERN_GINI 1  /* |x - z|               */
#define TW_KERN_HINGE 2 /* max(z - x + margin, 0) */
#define TW_KERN_LOGISTIC 3 /* log(1 + exp(z - x + margin)): extension, SURVEY.md §8 row L3 */

/* Pairwise losses of the gradient kernels.  TW_LOSS_HINGE is grad_inc_block's
 * (compute_stats.py:146-162).  TW_LOSS_LOGISTIC is the pairwise-logistic loss BASELINE.json
 * names, absent from the reference (parity pinned against
 * oracle/oracle.py only): softplus(S), S = diff . w + margin, pair weight sigma(S). */
#define TW_LOSS_HINGE 0
#define TW_LOSS_LOGISTIC 1

const char* tw_last_error(void);
int tw_version(void);
/* number of visible HIP devices (0 when no GPU); does not create a context on failure */
int tw_device_count(int* out_count);

/* ---- Row A1/A2/A6/A7: complete two-sample count, all shards in one launch -------------
 * Replaces est.Un (estimation-experiment/main.py:29-31) and cs.Un(kernel="AUC")
 * (compute_stats.py:10-19) as the f_block of UN (main.py:33-69, compute_stats.py:56-92).
 * d_out[s] (uint64) = #{(i,j): pred(x_i, z_j)} over shard s (half-units for TW_PRED_HALF).
 * max_nx / max_nz: the largest shard sizes (host-known; they size the grid). */
int tw_count_pairs(const void* d_x, const int64_t* d_x_off, const void* d_z,
                   const int64_t* d_z_off, int32_t n_shards, int64_t max_nx, int64_t max_nz,
                   int32_t dtype, int32_t pred, uint64_t* d_out, void* stream);

/* One step of est.UnNT's loop (estimation-experiment/main.py:76-79) in ONE launch: the counts
 * of the current partition exactly as tw_count_pairs — except that d_out must already be zero
 * (the kernel accumulates into it) — and, on spare leading blocks of the same grid, the NEXT
 * repartition: d_x_next = the n_x scores of d_x permuted with key_x, d_z_next likewise (as
 * tw_permute_pair), and d_out_next[0 .. n_next_shards) zeroed for the next step.
 * d_x_next == NULL: count only (d_out_next, if given, is zeroed by a memset). */
int tw_count_pairs_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                        const int64_t* d_z_off, int32_t n_shards, int64_t max_nx, int64_t max_nz,
                        int32_t dtype, int32_t pred, uint64_t* d_out, int64_t n_x, void* d_x_next,
                        uint64_t key_x, int64_t n_z, void* d_z_next, uint64_t key_z,
                        uint64_t* d_out_next, int32_t n_next_shards, void* stream);

/* Tuning hook for tw_count_pairs_step: number of spare blocks (0 = automatic), their
 * placement (tail = 1, the default: the last blocks of the grid; tail = 0: one group of 8
 * every `every` blocks, 0 = automatic spacing, 8 = the leading blocks).  Process-global;
 * results do not depend on it. */
int tw_count_step_set_plan(int32_t blocks, int32_t every, int32_t tail);

/* Tuning hook: 1 (default) counts part of each lane's x-values on the scalar unit (double
 * inputs, one-bit predicates; csrc/count.hip), 0 = VALU-only accumulation.  Process-global;
 * results do not depend on it. */
int tw_count_set_scalar_mix(int32_t on);

/* Tuning hook for tw_count_pairs' launch plan: R x-values per lane (1, 2, 4, 8; 0 = automatic)
 * and z-chunk length per block (0 = automatic).  Process-global; results do not depend on it. */
int tw_count_set_plan(int32_t R, int64_t z_chunk);

/* ---- A1/A6/A7 on rank images (round 3, csrc/rankimage.hip): the all-pairs count of
 * est.UnN / UnNT (estimation-experiment/main.py:29-31, :72-79) on packed f32 images.
 * tw_rank_images gives every score an 8-B record {low word: f32 image, high word: its index in
 * d_x / d_z}: image g(v) = #{z in d_z : z < v} (x: g, z: -g; a NaN x: -2^25), so that for any
 * pair x > z <=> x_image + z_image >= 1, NaN and -0 == +0 included (strict predicate, float64
 * or int64 scores; int64 SUBGT / half ties stay on tw_count_pairs).  One bucketed ranking of
 * X u Z per call (sampled splitters, per-bucket LDS sorts of the z keys); needs n_z < 2^24
 * (tw_rank_images_work_bytes returns -1 otherwise).
 * d_work: device scratch of tw_rank_images_work_bytes(n_x, n_z) bytes. */
int64_t tw_rank_images_work_bytes(int64_t n_x, int64_t n_z);
int tw_rank_images(const void* d_x, int64_t n_x, const void* d_z, int64_t n_z, int32_t dtype,
                   void* d_work, int64_t work_bytes, uint64_t* d_x_rec, uint64_t* d_z_rec,
                   void* stream);
/* tw_count_pairs_step on records: counts every shard of the current partition of d_x_rec /
 * d_z_rec into d_out (already zero) — per pair one packed clamp-add and one packed add — and,
 * when d_x_next is given, permutes both record arrays for the next step with the keyed Feistel
 * bijection (as tw_count_pairs_step permutes scores) and zeroes d_out_next, in the same launch.
 * Counts are identical to tw_count_pairs(..., TW_PRED_GT) on the scores the records index. */
int tw_count_pairs_rank_step(const uint64_t* d_x_rec, const int64_t* d_x_off,
                             const uint64_t* d_z_rec, const int64_t* d_z_off, int32_t n_shards,
                             int64_t max_nx, int64_t max_nz, uint64_t* d_out, int64_t n_x,
                             uint64_t* d_x_next, uint64_t key_x, int64_t n_z, uint64_t* d_z_next,
                             uint64_t key_z, uint64_t* d_out_next, int32_t n_next_shards,
                             void* stream);
/* The scores in record order: d_out[p] = d_in[d_rec[p] >> 32] (8-B values; in != out). */
int tw_gather_records(const void* d_in, const uint64_t* d_rec, int64_t n, void* d_out,
                      void* stream);
/* Tuning hook for tw_count_pairs_rank_step: x-images per lane R (8 or 16; 0 = automatic) and
 * z-chunk length (0 = automatic).  Process-global; results do not depend on it. */
int tw_count_rank_set_plan(int32_t R, int64_t z_chunk);
/* Tuning hook for tw_count_pairs_rank_step's fused next repartition: its spare blocks are the
 * last blocks of the grid (front = 0, the default) or the first (front = 1).  Process-global;
 * results do not depend on it. */
int tw_count_rank_set_next(int32_t front);
/* Tuning hook for tw_rank_images / tw_rank_images_query: sampled z keys for the splitters (512,
 * 1024 or 2048) and z per thread in the bucket passes (4, 8 or 16).  Process-global; results
 * do not depend on it (the workspace size does: query it after setting). */
int tw_rank_set_plan(int32_t sample, int32_t per);
/* Tuning hook for small Z (n_z <= 2^18: the one-shot C2 counts): the ranking's sample size
 * (256, 512, 1024 or 2048 keys; default 256), the target z per interval bucket (512, 1024 or
 * 2048; default 2048) and z per thread in the bucket passes (4, 8 or 16; default 4). */
int tw_rank_set_small(int32_t sample, int32_t z_per_interval, int32_t per);
/* tw_rank_images over several ranks (and for half ties): the images are counted against the Z
 * of d_z_all (the all-gathered sample, n_z_all < 2^24) but written only for the n_x + n_z
 * elements of d_x / d_z (this rank's share; d_z may be d_z_all).  half (flags): bit 0 — each X
 * record's high word is h(x) = #{z in d_z_all : z <= x} as f32 bits (NaN x: -2^25) instead of
 * the index; bit 1 — compact images without indices, the bag layout of tw_count_pairs_chain
 * (d_x_rec: n_x f32, or n_x {g, h} f32 pairs with bit 0; d_z_rec: n_z f32).
 * d_work: tw_rank_images_work_bytes(n_x, n_z_all) bytes. */
int tw_rank_images_query(const void* d_z_all, int64_t n_z_all, const void* d_x, int64_t n_x,
                         const void* d_z, int64_t n_z, int32_t dtype, int32_t half,
                         void* d_work, int64_t work_bytes, uint64_t* d_x_rec, uint64_t* d_z_rec,
                         void* stream);

/* ---- A7 / (e) step chains (round 4, csrc/chain.hip): the repartition loop of est.UnNT
 * (estimation-experiment/main.py:76-79; each repartition = the keyed Feistel bijection of
 * tw_permute_pair with keys 2k / 2k+1) walked per element.  A rank holds n_x + n_z elements
 * whose global indices start at rank * n_x / rank * n_z in samples of world * n_x / world * n_z;
 * every rank's local layout is prop-SWOR shards of x_shard / z_shard positions (n_shards of
 * them, clamped at the array ends, then a tail in no shard).
 * tw_chain_emit walks `steps` (<= 32) repartitions (host arrays keys_x / keys_z of the Feistel
 * keys) for every element of d_x_rec / d_z_rec (rank-image records; half = 1: X records carry
 * {g, h}), its global position kept in d_x_pos / d_z_pos (u32; first = 1: start from the
 * element's global index).  d_send == NULL (one process, world == 1): for each step c the
 * images are appended to the bags d_x_bag [steps][n_x] (f32, or {g, h} f32 pairs when half) /
 * d_z_bag [steps][n_z] (f32), each shard's slot range holding exactly its images in an
 * arbitrary order; d_cursors: scratch of steps * 2 * (n_shards + 1) u32.  d_send given (the
 * exchange: world > 1, or a world-size-1 group forced through its collectives): records go to
 * d_send, per destination rank g a
 * chunk of steps buckets of (cap + 1) * W u64 words (W = 1 + half; word 0 of a bucket = its
 * count), each record {image word(s), local position (Z: n_x + position)}; a bucket past cap
 * sets *d_flag (the record is dropped). */
int tw_chain_emit(const uint64_t* d_x_rec, int64_t n_x, const uint64_t* d_z_rec, int64_t n_z,
                  int32_t half, uint32_t* d_x_pos, uint32_t* d_z_pos, int32_t first,
                  int32_t rank, int32_t world, const uint64_t* keys_x, const uint64_t* keys_z,
                  int32_t steps, int64_t x_shard, int64_t z_shard, int32_t n_shards,
                  void* d_x_bag, void* d_z_bag, uint32_t* d_cursors, uint64_t* d_send,
                  int64_t cap, int32_t* d_flag, void* stream);
/* The receiving side of tw_chain_emit's buckets after an equal-split all-to-all (d_recv: world
 * chunks in source order): every record appended to the bag region of its (step, side, shard)
 * — shard b of a side holds positions [min(b k, n), min((b+1) k, n)), k = x_shard / z_shard,
 * b = n_shards the tail — in runs reserved on d_cursors (steps x 2 (n_shards + 1) u32, zeroed
 * here); a bag holds its shard's multiset, in no particular order (what the counts read).  A
 * count past cap sets *d_flag. */
int tw_chain_unpack(const uint64_t* d_recv, int32_t world, int32_t steps, int64_t cap,
                    int32_t half, int64_t n_x, int64_t n_z, int64_t x_shard, int64_t z_shard,
                    int32_t n_shards, void* d_x_bag, void* d_z_bag, uint32_t* d_cursors,
                    int32_t* d_flag, void* stream);
/* The all-pairs counts of `steps` x n_shards bags in ONE launch: bag (c, s) = x images
 * [c * x_stride + d_x_off[s], c * x_stride + d_x_off[s + 1]) against z images likewise;
 * d_out[c * n_shards + s] (zeroed here) = #{x > z} (half = 1: 2 #{x > z} + #{x == z}, the
 * tw_count_pairs TW_PRED_HALF units).  Identical to tw_count_pairs on the scores. */
int tw_count_pairs_chain(const void* d_x_bag, const int64_t* d_x_off, int64_t x_stride,
                         const void* d_z_bag, const int64_t* d_z_off, int64_t z_stride,
                         int32_t n_shards, int32_t steps, int64_t max_nx, int64_t max_nz,
                         int32_t half, uint64_t* d_out, void* stream);
/* The same counts as tw_count_pairs_chain in O(n + m) per bag (algo="sorted", SURVEY row f4;
 * estimation-experiment/main.py:29-31's integer): each bag's z images (integers in
 * [0, z_total], z_total = the Z count the images were ranked against) counting-sorted into
 * <= 16384 LDS buckets, every x's g(x) (and h(x) with half) answered by the bucket prefix and a
 * scan of its own bucket.  Bags of <= 16384 z (max_nz); d_out[c * n_shards + s] written, not
 * accumulated. */
int tw_count_pairs_chain_bucket(const void* d_x_bag, const int64_t* d_x_off, int64_t x_stride,
                                const void* d_z_bag, const int64_t* d_z_off, int64_t z_stride,
                                int32_t n_shards, int32_t steps, int64_t max_nz,
                                int64_t z_total, int32_t half, uint64_t* d_out, void* stream);
/* Tuning hook for tw_chain_emit: elements per thread (2, 4 or 8) and steps per reservation
 * round (1 or 16 / elements per thread); 0 = automatic.  Process-global; results do not depend
 * on it (the order inside a bag does). */
int tw_chain_set_emit(int32_t epr, int32_t steps_per_round);
/* Tuning hook for tw_count_pairs_chain: x-images per lane (8 or 16; 0 = automatic) and z-chunk
 * length (0 = automatic).  Process-global; results do not depend on it. */
int tw_count_chain_set_plan(int32_t R, int64_t z_chunk);
/* The scores in their final order after the chains (one process): d_x_out[d_x_pos[e]] =
 * d_x[e] (8-B values), likewise for Z. */
int tw_chain_scatter(const void* d_x, const uint32_t* d_x_pos, int64_t n_x, const void* d_z,
                     const uint32_t* d_z_pos, int64_t n_z, void* d_x_out, void* d_z_out,
                     void* stream);
/* The same over ranks: this rank's final positions [x_base, x_base + n_x) of the n_x_all-long
 * X (and Z likewise) walked back through all `steps` repartitions (inverse Feistel, last step
 * first) and gathered from the all-gathered samples d_x_all / d_z_all.  d_work: n_x + n_z u32
 * when steps > 32. */
int tw_chain_gather(const void* d_x_all, const void* d_z_all, int64_t x_base, int64_t n_x,
                    int64_t n_x_all, int64_t z_base, int64_t n_z, int64_t n_z_all,
                    const uint64_t* keys_x, const uint64_t* keys_z, int32_t steps,
                    uint32_t* d_work, void* d_x_out, void* d_z_out, void* stream);
/* tw_chain_gather of a second pair of arrays laid out like the first (the carried rank-image
 * records beside the scores) from the same walk of the inverse chains. */
int tw_chain_gather2(const void* d_x_all, const void* d_z_all, const void* d_x_all2,
                     const void* d_z_all2, int64_t x_base, int64_t n_x, int64_t n_x_all,
                     int64_t z_base, int64_t n_z, int64_t n_z_all, const uint64_t* keys_x,
                     const uint64_t* keys_z, int32_t steps, uint32_t* d_work, void* d_x_out,
                     void* d_z_out, void* d_x_out2, void* d_z_out2, void* stream);

/* ---- f4: the same counts in O((n+m) log m): sort each z-chunk (<= 16384 keys) in LDS as
 * order-preserving u64 keys, then binary-search every x (csrc/rankcount.hip).  Bit-identical
 * to tw_count_pairs for TW_PRED_GT and TW_PRED_HALF (not SUBGT).  d_work: device scratch of
 * tw_count_pairs_sorted_work_bytes(n_shards, max_nz) bytes. */
int64_t tw_count_pairs_sorted_work_bytes(int32_t n_shards, int64_t max_nz);
/* Tuning hook: largest sorted chunk (power of two in [1024, 16384]; default 4096).
 * Process-global; results do not depend on it (the workspace size does). */
int tw_count_sorted_set_chunk(int64_t cap);
int tw_count_pairs_sorted(const void* d_x, const int64_t* d_x_off, const void* d_z,
                          const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                          int64_t max_nz, int32_t dtype, int32_t pred, void* d_work,
                          uint64_t* d_out, void* stream);
/* One step of est.UnNT's loop with the exact sorted count: the counts of tw_count_pairs_sorted
 * for the current partition — except that d_out must already be zero (accumulated into) — and
 * the NEXT repartition: d_x_next / d_z_next = the scores permuted with key_x / key_z (as
 * tw_permute_pair), d_out_next[0 .. n_next_shards) zeroed.  On the bucket path (every shard's
 * nz <= 16384) the permutation's gathers ride in the count threads of the same launch;
 * otherwise the count, tw_permute_pair and a memset run in turn.  d_x_next == NULL: count only.
 * Replaces the shuffle + UN loop of estimation-experiment/main.py:43-79 like tw_count_pairs_step. */
int tw_count_pairs_sorted_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                               const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                               int64_t max_nz, int32_t dtype, int32_t pred, void* d_work,
                               uint64_t* d_out, int64_t n_x, void* d_x_next, uint64_t key_x,
                               int64_t n_z, void* d_z_next, uint64_t key_z,
                               uint64_t* d_out_next, int32_t n_next_shards, void* stream);
/* T steps of est.UnNT's loop (estimation-experiment/main.py:76-79) with the exact sorted count
 * in ONE call: step t repartitions both samples with keys_x[t] / keys_z[t] (host arrays; step 0
 * starts from d_x / d_z in position order) and counts every shard into d_out[t * n_shards ..]
 * (zeroed by the call); the last partition is written to d_x_out / d_z_out (distinct from the
 * inputs).  Between steps the partition lives in d_work as records {value, position} grouped by
 * destination shard, so a repartition is a streaming pass (csrc/records.h) instead of one random
 * gather per score.  The layout must be prop-SWOR's: d_x_off[s] = min(s * kx, n_x),
 * d_z_off[s] = min(s * kz, n_z).  tw_count_pairs_sorted_steps_work_bytes() returns 0 where the
 * path does not apply (then use tw_count_pairs_sorted_step per step). */
int64_t tw_count_pairs_sorted_steps_work_bytes(int64_t n_x, int64_t n_z, int32_t n_shards,
                                               int64_t max_nz, int32_t dtype, int32_t pred);
int tw_count_pairs_sorted_steps(const void* d_x, const void* d_z, int64_t n_x, int64_t n_z,
                                const int64_t* d_x_off, const int64_t* d_z_off, int32_t n_shards,
                                int64_t kx, int64_t kz, int64_t max_nx, int64_t max_nz,
                                int32_t dtype, int32_t pred, const uint64_t* keys_x,
                                const uint64_t* keys_z, int32_t T, void* d_work,
                                int64_t work_bytes, uint64_t* d_out, void* d_x_out,
                                void* d_z_out, void* stream);
/* Shards with nz <= 16384 (default 1): the count comes from value buckets of z in LDS (an
 * LDS histogram, prefix and scatter, then one bucket scanned per x) instead of sorted chunks +
 * binary searches; the same integers.  1 = equal-depth buckets (the value-range histogram's
 * CDF refines the map), 2 = value-range buckets only, 0 = always sort + search (A/B, tests). */
int tw_count_sorted_set_bucket(int32_t by_bucket);

/* ---- Row A3/A4/A5/A8: incomplete count on given index pairs (replay mode) -------------
 * Replaces cs.UB_indices / UB_pairs / UB (compute_stats.py:22-42): pair p of shard s
 * compares x[d_ix[p]] with z[d_iz[p]] for p in [d_pair_off[s], d_pair_off[s+1]); indices are
 * absolute positions in d_x / d_z (int64, as NumPy randint returns them). */
int tw_count_pairs_idx(const void* d_x, const void* d_z, const int64_t* d_ix,
                       const int64_t* d_iz, const int64_t* d_pair_off, int32_t n_shards,
                       int64_t max_pairs, int32_t dtype, int32_t pred, uint64_t* d_out,
                       void* stream);
/* The same counts as tw_count_pairs_idx with the compares on the 16-bit rank codes of
 * tw_count_pairs_rng_ws held in LDS (shard s spans d_x_off[s]..d_x_off[s+1] and
 * d_z_off[s]..d_z_off[s+1]; an index outside its shard's span compares the scores), so the
 * kernel streams only the indices.  d_work holds tw_count_pairs_rng_work_bytes(n_shards,
 * max_nx, max_nz, dtype, pred) bytes; when that is 0 (shards of >= 65536 values, int64 SUBGT) or
 * d_work == NULL this call runs tw_count_pairs_idx. */
/* Tuning hook of tw_count_pairs_idx_ws: blocks of 1024 threads per shard (0 = the plan's). */
int tw_count_idx_set_parts(int32_t parts);
/* Tuning hook of the int32-index ranked count: 0 = four 16-B loads of each index stream in
 * flight per thread (default), 1 = the same as nontemporal loads, 2/3 = eight loads (plain /
 * nontemporal), 4/5 = two loads.  Process-global; results do not depend on it. */
int tw_count_idx_set_variant(int32_t v);
int tw_count_pairs_idx_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                          const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                          int64_t max_nz, const int64_t* d_ix, const int64_t* d_iz,
                          const int64_t* d_pair_off, int64_t max_pairs, int32_t dtype,
                          int32_t pred, void* d_work, int64_t work_bytes, uint64_t* d_out,
                          void* stream);
/* int32-index variants — the 8 B/pair replay contract of SURVEY.md §8(d): the same counts as
 * tw_count_pairs_idx / tw_count_pairs_idx_ws with d_ix / d_iz int32 (absolute positions below
 * 2^31).  They replace the same reference lines (compute_stats.py:22-42); the Python layer
 * narrows NumPy's int64 randint output after its bound check (UB_indices' indexing,
 * compute_stats.py:26-30) whenever both samples have fewer than 2^31 elements. */
int tw_count_pairs_idx32(const void* d_x, const void* d_z, const int32_t* d_ix,
                         const int32_t* d_iz, const int64_t* d_pair_off, int32_t n_shards,
                         int64_t max_pairs, int32_t dtype, int32_t pred, uint64_t* d_out,
                         void* stream);
int tw_count_pairs_idx32_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                            const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                            int64_t max_nz, const int32_t* d_ix, const int32_t* d_iz,
                            const int64_t* d_pair_off, int64_t max_pairs, int32_t dtype,
                            int32_t pred, void* d_work, int64_t work_bytes, uint64_t* d_out,
                            void* stream);

/* ---- Row A5/A8, device-RNG mode: B pairs per shard drawn on the device ----------------
 * Philox4x32-10(key = seed, counter = (q lo, q hi, shard_base + s, 0)) gives the 4 words
 * (w0, w1, w2, w3) of pairs 2q (i from w0, j from w1) and 2q+1 (w2, w3) of local shard s; a word
 * w maps to [0, n) by Lemire's multiply-shift (w * n) >> 32 with rejection of (w * n) mod 2^32
 * < 2^32 mod n, a rejected word being replaced by the same word of counter word 3 = 1, 2, ...
 * (exactly uniform; with-replacement sampling like UB's randint, compute_stats.py:40-41).
 * Shards of >= 2^32 values: pair p uses counter (p lo, p hi, shard_base + s, 0) and maps
 * (w1:w0), (w3:w2) by 64-bit multiply-high.
 * shard_base = the global index of local shard 0, so draws do not depend on how shards are
 * spread over ranks.  Not bit-comparable with NumPy's stream; statistically equivalent
 * (tests/test_statistics.py). */
int tw_count_pairs_rng(const void* d_x, const int64_t* d_x_off, const void* d_z,
                       const int64_t* d_z_off, int32_t n_shards, int64_t B, uint64_t seed,
                       uint64_t shard_base, int32_t dtype, int32_t pred, uint64_t* d_out,
                       void* stream);

/* The same draws and counts as tw_count_pairs_rng, with the compares on 16-bit rank codes held
 * in LDS (sorted z per shard; c_i = #{z < x_i}, c'_i = #{z <= x_i}, p_j = #{z < z_j}; x > z iff
 * c_i > p_j, x >= z iff c'_i > p_j) instead of random 8-B gathers of the scores.  Applies when
 * every shard has nx, nz < 65536, the codes fit in LDS and pred is GT or HALF: then
 * tw_count_pairs_rng_work_bytes() > 0 and d_work must hold that many bytes; otherwise (or with
 * d_work == NULL) this call runs tw_count_pairs_rng. */
int64_t tw_count_pairs_rng_work_bytes(int32_t n_shards, int64_t max_nx, int64_t max_nz,
                                      int32_t dtype, int32_t pred);
/* Rank codes of tw_count_pairs_rng_ws / tw_count_pairs_idx(32)_ws: 1 (default) = equal-depth
 * value buckets in LDS when every shard has nz <= 16384, 2 = value-range buckets only, 0 =
 * always sort + binary search (A/B and tests; same codes). */
int tw_count_rng_set_codes(int32_t by_bucket);
/* Default mode 3 of tw_count_rng_set_codes (csrc/imagecount.hip): instead of rank codes, each
 * block stages the float32 images of its shard's scores in LDS (round to nearest: monotone) and
 * decides x > z on them, gathering the scores only for pairs whose images are equal (ties, -0/+0,
 * values within a float ulp): the same counts, no codes kernel, no workspace.  Applies when a
 * shard pair's images fit in LDS (4 * (nx + nz) bytes <= 159 KiB) and pred is GT or HALF (or
 * SUBGT on doubles); otherwise the codes path runs (and past it the plain kernel).  Tuning hook:
 * blocks per shard (0 = plan) and 16-B index vectors per stream and batch (1, 2, 4; + 8 =
 * nontemporal index loads; default 9). */
int tw_count_img_set_plan(int32_t parts, int32_t u);
/* Tuning hook: Philox blocks each thread of the device-RNG image kernel draws per iteration
 * (1, 2 — the default — or 4; independent chains for the scheduler).  No effect on results. */
int tw_count_rng_img_set_unroll(int32_t qu);
int tw_count_pairs_rng_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                          const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                          int64_t max_nz, int64_t B, uint64_t seed, uint64_t shard_base,
                          int32_t dtype, int32_t pred, void* d_work, int64_t work_bytes,
                          uint64_t* d_out, void* stream);
/* One step of cs.UnNBT's loop (compute_stats.py:119-123) in device-RNG mode: the counts of
 * tw_count_pairs_rng_ws for the current partition — except that d_out must already be zero
 * (accumulated into) — and the NEXT repartition: d_x_next = the n_x scores of d_x permuted
 * with key_x, d_z_next likewise (as tw_permute_pair), d_out_next[0 .. n_next_shards) zeroed.
 * On the float32-image path (above) the next repartition's gathers ride in the count threads
 * of the same launch; otherwise the count, tw_permute_pair and a memset run in turn.
 * d_x_next == NULL: count only.  Replaces the repartition + UB loop of compute_stats.py:104-110
 * as tw_count_pairs_step does for est.UnNT. */
int tw_count_pairs_rng_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                            const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                            int64_t max_nz, int64_t B, uint64_t seed, uint64_t shard_base,
                            int32_t dtype, int32_t pred, void* d_work, int64_t work_bytes,
                            uint64_t* d_out, int64_t n_x, void* d_x_next, uint64_t key_x,
                            int64_t n_z, void* d_z_next, uint64_t key_z, uint64_t* d_out_next,
                            int32_t n_next_shards, void* stream);

/* ---- Row A2 (prod/gini) and f1 (conv_AUC): float pair sums, complete -------------------
 * d_out[s] (double) = sum over all pairs of shard s of kern(x_i, z_j).  Deterministic: fixed
 * per-block partial order, then an ordered per-shard reduction.  d_work: n_shards *
 * tw_pair_sum_work_per_shard(max_nx, max_nz) doubles. */
int64_t tw_pair_sum_work_per_shard(int64_t max_nx, int64_t max_nz);
int tw_pair_sum_f64(const double* d_x, const int64_t* d_x_off, const double* d_z,
                    const int64_t* d_z_off, int32_t n_shards, int64_t max_nx, int64_t max_nz,
                    int32_t kern, double margin, double* d_work, double* d_out, void* stream);

/* ---- f1: float pair sums on given index pairs (conv_AUC_deter_pairs, UB_indices prod/gini)
 * d_out[s] = sum_p kern(x[ix_p], z[iz_p]); d_work: n_shards * tw_pair_sum_idx_work_per_shard(max_pairs). */
int64_t tw_pair_sum_idx_work_per_shard(int64_t max_pairs);
int tw_pair_sum_idx_f64(const double* d_x, const double* d_z, const int64_t* d_ix,
                        const int64_t* d_iz, const int64_t* d_pair_off, int32_t n_shards,
                        int64_t max_pairs, int32_t kern, double margin, double* d_work,
                        double* d_out, void* stream);
/* int32 indices; d_count (nullable, uint64 per shard): the same pass also counts x > z — the
 * fixed-pair br_AUC of evaluation_step (UB_pairs(kernel="AUC"), make_exps.py:162-168) beside
 * its hinge mean bc_AUC (conv_AUC_deter_pairs, compute_stats.py:137-144), one read of the
 * monitor pairs for both. */
int tw_pair_sum_idx32_f64(const double* d_x, const double* d_z, const int32_t* d_ix,
                          const int32_t* d_iz, const int64_t* d_pair_off, int32_t n_shards,
                          int64_t max_pairs, int32_t kern, double margin, double* d_work,
                          double* d_out, uint64_t* d_count, void* stream);

/* ---- Row L1: pairwise hinge gradient, all shards in one launch ------------------------
 * Replaces grad_inc_block(w, B, margin)(X_s, Z_s) (compute_stats.py:146-162) for every shard
 * of UN_split (compute_stats.py:44-46).  X: (n_X, d) row-major doubles, Z: (n_Z, d).
 * Shard s, pair b: rx = d_rows_x[s*kx + d_ix[s*B+b]], rz = d_rows_z[s*kz + d_iz[s*B+b]]
 * (SWR_divide row draws composed with the per-block randint draws, compute_stats.py:48-54,
 * :155-156); d_rows_x / d_rows_z may be NULL meaning identity (shard = whole array).
 * diff = Z[rz] - X[rx]; S = diff . w + margin; d_out[s*d + j] = (sum_{b: S_b > 0} diff_bj) / B,
 * summed over b in order (as NumPy's axis-0 reduce does). */
int tw_hinge_grad(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                  int64_t kx, const int64_t* d_rows_z, int64_t kz, const int64_t* d_ix,
                  const int64_t* d_iz, int32_t n_shards, int64_t B, const double* d_w,
                  double margin, double* d_out, void* stream);

/* Same for either loss: d_out[s*d + j] = (sum_b weight_b * diff_bj) / B in row order, with
 * weight 1{S_b > 0} (hinge: filtered rows only, exactly as above) or sigma(S_b) (logistic). */
int tw_pair_grad(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                 int64_t kx, const int64_t* d_rows_z, int64_t kz, const int64_t* d_ix,
                 const int64_t* d_iz, int32_t n_shards, int64_t B, const double* d_w,
                 double margin, int32_t loss, double* d_out, void* stream);

/* Sign audit (SURVEY.md §7 "count and report" the hinge-filter flips): tw_pair_grad plus
 * d_scores[s*B + b] = S_b = diff_b . w + margin exactly as the kernel computed it (the generic
 * kernel; its narrow and wide paths sum the dot product in the orders of the streaming and fused
 * kernels).  The reference decides the filter on BLAS's S (compute_stats.py:158-159); the
 * caller compares the signs (tuplewise.learning.learning_process(..., sign_audit=[])). */
int tw_pair_grad_audit(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                       int64_t kx, const int64_t* d_rows_z, int64_t kz, const int64_t* d_ix,
                       const int64_t* d_iz, int32_t n_shards, int64_t B, const double* d_w,
                       double margin, int32_t loss, double* d_out, double* d_scores,
                       void* stream);

/* ---- Complete-block gradient (extension; BASELINE.json north_star item (2)) -------------
 * The same surrogate's gradient over ALL kx*kz pairs of each shard, computed as per-point
 * pair-coefficient reductions followed by X^T c (csrc/complete_grad.hip):
 *   sx_i = X[rx_i].w, sz_j = Z[rz_j].w, S_ij = sz_j - sx_i + margin,
 *   a_j = sum_i phi'(S_ij), b_i = sum_j phi'(S_ij)  (phi' = 1{S>0} hinge, sigma(S) logistic),
 *   d_out[s*d + c] = (sum_j a_j Z[rz_j][c] - sum_i b_i X[rx_i][c]) / (kx*kz).
 * Rows as tw_hinge_grad (d_rows_* NULL = shard s owns rows [s*k, (s+1)*k)).  d_work: device
 * scratch of tw_pair_grad_complete_work_bytes(n_shards, kx, kz, d) bytes.  Deterministic
 * (fixed summation orders); not in the reference (its learner samples B pairs). */
int64_t tw_pair_grad_complete_work_bytes(int32_t n_shards, int64_t kx, int64_t kz, int64_t d);
int tw_pair_grad_complete(const double* d_X, const double* d_Z, int64_t d,
                          const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                          int64_t kz, int32_t n_shards, const double* d_w, double margin,
                          int32_t loss, void* d_work, double* d_out, void* stream);
/* Hinge coefficients are counts; by default they come from binary searches with the exact
 * floating-point predicate over each shard's sorted scores (S is monotone in each score), the
 * same integers as the pair-by-pair sums in O(k log k); logistic coefficients come from one
 * pass over the pairs (each sigma(S_ij) feeds a_j and b_i).  on = 0 selects the two-pass
 * pair-by-pair kernels (kept for A/B checks). */
int tw_pair_grad_complete_set_search(int32_t on);

/* ---- Row L1/A9, device-RNG mode (no host RNG in the loop; graph-capturable) -----------
 * Draws are Philox4x32-10(key = seed, counter = (index, shard, step lo, tag | step hi)) with
 * step = *d_step (device memory, advanced by tw_sgd_update), mapped by 64-bit multiply-high;
 * the shard word is shard_base + local shard, so draws follow GLOBAL shard indices and a
 * run spread over ranks draws exactly what a single GPU draws:
 * tw_hinge_grad_rng: pair b of shard s -> (ix, iz) in [0,kx) x [0,kz) (tag 0x80000000);
 * tw_swr_rows_rng:   d_rows[s*k + t] in [0, n), side 0 = X rows (tag 0x40000000), 1 = Z rows
 *                    (tag 0x20000000) — SWR_divide (compute_stats.py:48-54) on the device.
 * Statistically equivalent to the reference's NumPy draws, not bit-comparable; exactly
 * reproducible from (seed, step) and checked against oracle/oracle.py's restatement. */
int tw_hinge_grad_rng(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                      int64_t kx, const int64_t* d_rows_z, int64_t kz, int32_t n_shards,
                      int64_t B, const double* d_w, double margin, uint64_t seed,
                      const uint64_t* d_step, int32_t shard_base, double* d_out, void* stream);
/* Tuning hook for 32 < d <= 512 rows: 0 = the streaming kernel (default: two register stages,
 * 16-pair chunks), 1 = the unpipelined kernel, 2 = the burst-pipelined kernel (32-pair chunks).
 * Process-global; all give identical bits. */
int tw_hinge_set_variant(int32_t legacy_wide);
int tw_pair_grad_rng(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                     int64_t kx, const int64_t* d_rows_z, int64_t kz, int32_t n_shards, int64_t B,
                     const double* d_w, double margin, int32_t loss, uint64_t seed,
                     const uint64_t* d_step, int32_t shard_base, double* d_out, void* stream);
int tw_swr_rows_rng(int64_t* d_rows, int32_t n_shards, int64_t k, int64_t n, uint64_t seed,
                    const uint64_t* d_step, int32_t side, int32_t shard_base, void* stream);

/* ---- Row L2: update of learning_process (make_exps.py:130-141) ------------------------
 * g = mean_s(d_grads[s]) + reg * w  (shards summed in order, then / n_shards — np.mean axis 0)
 * momentum: dw = momentum * dw + lr * g;  SGD (momentum < 0): dw = lr * g;   w = w - dw.
 * d_step (nullable): device-RNG step counter, incremented once. */
int tw_sgd_update(double* d_w, double* d_dw, const double* d_grads, int32_t n_shards, int64_t d,
                  double reg, double lr, double momentum, uint64_t* d_step, void* stream);
/* Same update from (d_w_in, d_dw_in) into (d_w, d_dw) (may be the same buffers); the step
 * counter (nullable) advances by step_inc.  Ends a segment of tw_sgd_step launches. */
int tw_sgd_update_to(const double* d_w_in, const double* d_dw_in, double* d_w, double* d_dw,
                     const double* d_grads, int32_t n_shards, int64_t d, double reg, double lr,
                     double momentum, uint64_t* d_step, int32_t step_inc, void* stream);

/* ---- Rows L1 + L2 fused: one launch per SGD step (narrow rows, d <= 32, n_shards*d <= 4096;
 * tw_sgd_step_fusable says whether a shape qualifies).  The launch first applies the update of
 * the PREVIOUS step (d_grads_in, d_w_in, d_dw_in -> w, written by block 0 to d_w_out/d_dw_out;
 * every block computes it, so no grid synchronisation), then computes this step's per-shard
 * gradients with it into d_grads_out.  d_grads_in == NULL: no pending update (w = d_w_in).
 * Draws: replay (d_ix, d_iz) or device RNG at step *d_step + step_off (the counter itself is
 * advanced by the tw_sgd_update_to that ends the segment).  A segment of k steps is
 *   step 0: in (w0, -, -) -> grads G0;   step j>0: in (W[j-1&1], DW[j-1&1], G[j-1&1]) ->
 *   out (W[j&1], DW[j&1], G[j&1]);  then tw_sgd_update_to(W[k-1&1], DW[k-1&1] -> w0, dw0,
 *   G[k-1&1], step_inc = k)
 * (ping-pong slots, slot 0 = w0/dw0): the same bits as k tw_pair_grad(_rng) + tw_sgd_update
 * pairs, with k + 1 launches instead of 2k. */
int tw_sgd_step_fusable(int64_t d, int32_t n_shards);
int tw_sgd_step(const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x,
                int64_t kx, const int64_t* d_rows_z, int64_t kz, const int64_t* d_ix,
                const int64_t* d_iz, int32_t n_shards, int64_t B, double margin, int32_t loss,
                uint64_t seed, const uint64_t* d_step, int32_t step_off, int32_t shard_base,
                const double* d_w_in, const double* d_dw_in, const double* d_grads_in, double reg,
                double lr, double momentum, double* d_w_out, double* d_dw_out,
                double* d_grads_out, void* stream);

/* A segment of nsteps narrow-row SGD steps (d <= 32; the steps tw_sgd_step launches one by
 * one) in ONE persistent launch (csrc/sgdseg.hip k_sgd_segment_narrow): one block per shard,
 * all co-resident, one grid barrier per step, the update recomputed in every block from the
 * published shard gradients (slots d_grads0 / d_grads1 by step parity).  On return d_w_out /
 * d_dw_out hold the state after the segment's last update and the last step's gradients are
 * in slot (nsteps-1) & 1: apply them with tw_sgd_update_to(d_w_out, d_dw_out -> w, dw,
 * step_inc = nsteps).  Draws: d_ix/d_iz + step k * draw_stride (replay) or device RNG at
 * *d_step + k.  d_ctl: 2 words, zeroed once by the caller — the arrival counter (the kernel
 * leaves it at zero again) and a sticky abort word (set when a bounded barrier wait expired).
 * The residency check (tw_sgd_segment_narrow_ok) is the caller's, once, outside any stream
 * capture: this entry only checks shapes.  Same bits as tw_sgd_step per step.
 * make_exps.py:122-141 with compute_stats.py:146-162. */
int tw_sgd_segment_narrow_ok(int64_t d, int32_t n_shards, int64_t B);
int tw_sgd_segment_narrow(const double* d_X, const double* d_Z, int64_t d,
                          const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z, int64_t kz,
                          const int64_t* d_ix, const int64_t* d_iz, int64_t draw_stride,
                          int32_t n_shards, int64_t B, double margin, int32_t loss, uint64_t seed,
                          const uint64_t* d_step, int32_t shard_base, int32_t nsteps,
                          const double* d_w_in, const double* d_dw_in, double reg, double lr,
                          double momentum, double* d_grads0, double* d_grads1, double* d_w_out,
                          double* d_dw_out, uint32_t* d_ctl, void* stream);
/* tw_sgd_segment_narrow replaying through reshuffles: d_rows_x / d_rows_z are stacks of SWR
 * row tables tab_x / tab_z words apart (>= n_shards * kx / kz), and step k of the segment
 * reads table (tab_phase + k) / tab_mod — the segment starts at step tab_phase of a reshuffle
 * period of tab_mod steps (0 <= tab_phase < tab_mod), table 0 being the tables in force at its
 * start (learning_process's SWR_divide every `mod` steps, make_exps.py:123-125, without
 * ending the segment there). */
int tw_sgd_segment_narrow_tables(
    const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x, int64_t kx,
    const int64_t* d_rows_z, int64_t kz, int64_t tab_x, int64_t tab_z, int64_t tab_phase,
    int64_t tab_mod, const int64_t* d_ix, const int64_t* d_iz, int64_t draw_stride,
    int32_t n_shards, int64_t B, double margin, int32_t loss, uint64_t seed,
    const uint64_t* d_step, int32_t shard_base, int32_t nsteps, const double* d_w_in,
    const double* d_dw_in, double reg, double lr, double momentum, double* d_grads0,
    double* d_grads1, double* d_w_out, double* d_dw_out, uint32_t* d_ctl, void* stream);
/* tw_sgd_segment_narrow in device-RNG mode with the SWR row tables drawn IN the kernel: the
 * row of draw position a of shard s at step counter c is the one tw_swr_rows_rng drew at the
 * last reshuffle, counter rc = c - (c - swr_base) % swr_mod (reshuffles every swr_mod steps
 * from swr_base: make_exps.py:123-125), so one launch runs through any number of reshuffles.
 * Same bits as tw_swr_rows_rng at every reshuffle + tw_sgd_segment_narrow between them. */
int tw_sgd_segment_narrow_swr(const double* d_X, const double* d_Z, int64_t d, int64_t n_X,
                              int64_t n_Z, int64_t kx, int64_t kz, int32_t n_shards, int64_t B,
                              double margin, int32_t loss, uint64_t seed, const uint64_t* d_step,
                              int32_t shard_base, int32_t nsteps, int64_t swr_mod,
                              uint64_t swr_base, const double* d_w_in, const double* d_dw_in,
                              double reg, double lr, double momentum, double* d_grads0,
                              double* d_grads1, double* d_w_out, double* d_dw_out,
                              uint32_t* d_ctl, void* stream);
/* evaluation_step's FIXED_PAIRS statistics (make_exps.py:143-190) for small problems in two
 * launches: the scores A @ w of train X (n_trX x d), train Z, test X, test Z into d_scores
 * (concatenated, k_gemv's arithmetic), then the monitor pairs' surrogate sum and AUC count
 * (d_ix/d_iz: n_pairs int32 row indices; d_offs = {0, n_pairs, 0, n_teX, 0, n_teZ} on the
 * device) and all test pairs' surrogate sum and AUC count, reduced in one launch: d_out =
 * {monitor sum, monitor count (uint64 bits), test sum, test count (uint64 bits)} — the same
 * values as tw_gemv_f64 + tw_pair_sum_idx32_f64 + tw_pair_sum_f64 + tw_count_pairs.  d_work /
 * d_cwork: tw_eval_small_work(...) entries each; d_ticket: one zeroed word (left zero). */
int64_t tw_eval_small_work(int64_t n_pairs, int64_t n_test_x, int64_t n_test_z);
int tw_eval_small(const double* d_trX, int64_t n_trX, const double* d_trZ, int64_t n_trZ,
                  const double* d_teX, int64_t n_teX, const double* d_teZ, int64_t n_teZ,
                  int64_t d, const double* d_w, const int32_t* d_ix, const int32_t* d_iz,
                  int64_t n_pairs, const int64_t* d_offs, int32_t kern, double margin,
                  double* d_scores, double* d_work, uint64_t* d_cwork, uint32_t* d_ticket,
                  double* d_out, void* stream);
/* tw_pair_grad_rng with the SWR rows drawn in the kernel (reshuffles every swr_mod steps from
 * counter swr_base; the rows of tw_swr_rows_rng at the last reshuffle): the per-step gradient
 * of wide rows (C5) needs no row tables and no table-drawing launch per reshuffle. */
int tw_pair_grad_rng_swr(const double* d_X, const double* d_Z, int64_t d, int64_t n_X,
                         int64_t n_Z, int64_t kx, int64_t kz, int32_t n_shards, int64_t B,
                         const double* d_w, double margin, int32_t loss, uint64_t seed,
                         const uint64_t* d_step, int32_t shard_base, int64_t swr_mod,
                         uint64_t swr_base, double* d_out, void* stream);
/* ---- The hinge surrogate over ALL pairs of each shard in O((n + m) log m) (f64 scores):
 * d_out[s] = sum_{i,j} max(fl(fl(z_j - x_i) + margin), 0) — cs.conv_AUC's sum
 * (compute_stats.py:129-135) as evaluation_step's tc_AUC (make_exps.py:167-168) and
 * SAME_AS_BATCH's bc_AUC (:154-157) need it.  For each x the positive terms are the top c of
 * the shard's sorted z (a binary search with the exact predicate), summed from double-double
 * prefix sums: the exact sum of the terms rounded once (vs NumPy's pairwise sum of rounded
 * terms: ~1e-15 relative).  NaN / +-inf follow NumPy's elementwise semantics (NaN or +inf
 * results).  Empty shards give 0.  d_work: tw_pair_hinge_sum_sorted_work_bytes bytes. */
int64_t tw_pair_hinge_sum_sorted_work_bytes(int32_t n_shards, int64_t max_nx, int64_t max_nz);
int tw_pair_hinge_sum_sorted(const double* d_x, const int64_t* d_x_off, const double* d_z,
                             const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                             int64_t max_nz, double margin, void* d_work, double* d_out,
                             void* stream);

/* ---- f1: scores = A @ w for a row-major (n, d) matrix (evaluation_step, make_exps.py:163,
 * :170-171).  d <= 32: row dot products in index order; d > 32: see tw_gemv_set_variant. */
int tw_gemv_f64(const double* d_A, int64_t n, int64_t d, const double* d_w, double* d_out,
                void* stream);
/* Tuning hook: 1 (default) computes rows of d > 32 one wave per row (lane-strided partial dots
 * + a fixed butterfly, coalesced 16-B loads; 16-B aligned A and w), 0 = a thread per row in
 * index order.  Scores may differ in the last ulp between the two (BLAS's order differs too). */
int tw_gemv_set_variant(int32_t rows);

/* ---- Row A6/A9/(e): repartition on the device ----------------------------------------
 * Keyed pseudo-random permutation of [0, n): a 6-round Feistel network over the smallest
 * even-bit power-of-two domain >= n, with cycle walking (a bijection on [0, n)).
 * tw_permute_scatter: d_out[perm(i)] = d_in[i] for i in [0, n) (8-byte elements).
 * tw_perm_index: d_perm[i] = perm(i). */
int tw_permute_scatter(const void* d_in, void* d_out, int64_t n, uint64_t key, void* stream);
/* Both samples of one repartition in one launch: X (n elements, key_x) and Z (m, key_z),
 * each exactly as tw_permute_scatter. */
int tw_permute_pair(const void* d_x_in, void* d_x_out, int64_t n, uint64_t key_x,
                    const void* d_z_in, void* d_z_out, int64_t m, uint64_t key_z, void* stream);
int tw_perm_index(int64_t* d_perm, int64_t n, int64_t base, int64_t n_total, uint64_t key,
                  void* stream);

/* ---- (e) multi-rank repartition: counting sort of this rank's elements by destination rank
 * (dest = perm / n_loc, G <= 64 ranks), packed as 16-byte records {value bits, dest-local
 * position + pos_base} for an all-to-all(v); the receiver scatters the records into its local
 * array.  tw_rank_histogram: d_counts[g] = #elements bound for rank g.  tw_source_histogram:
 * d_counts[q] = #positions in [base, base+n) whose source perm^-1(p) (the permutation of
 * [0, n_total) keyed by `key`, as tw_perm_index) lies on rank q = source / n_loc — what this
 * rank receives from q, known without a message.  tw_bucket_scatter: record of element i goes
 * to d_send[2*(d_start[dst] + k)], k a per-destination slot reserved per block (d_cursor: G
 * uint64 of scratch); pos_base lets two arrays share one record buffer (e.g. Z positions
 * offset by n_loc of X).  tw_scatter_records: d_out[rec.pos] = rec.value for m records. */
int tw_rank_histogram(const int64_t* d_perm, int64_t n, int64_t n_loc, int32_t G,
                      uint64_t* d_counts, void* stream);
int tw_source_histogram(int64_t n, int64_t base, int64_t n_total, uint64_t key, int64_t n_loc,
                        int32_t G, uint64_t* d_counts, void* stream);
int tw_bucket_scatter(const int64_t* d_perm, const void* d_vals, int64_t n, int64_t n_loc,
                      int32_t G, const int64_t* d_start, uint64_t* d_cursor, int64_t pos_base,
                      void* d_send, void* stream);
int tw_scatter_records(const void* d_rec, int64_t m, void* d_out, void* stream);
/* The same exchange for BOTH samples of one repartition in two launches and without a
 * permutation array (what ShardedSample runs).  Rank `rank` owns global X positions
 * [rank*n_loc, (rank+1)*n_loc) of G*n_loc (key_x) and Z positions likewise (m_loc, key_z).
 * tw_exchange_counts: d_counts (4G uint64) = [send X | receive X | send Z | receive Z] per
 *   rank; zeroes d_cursor (2G uint64 of scratch).
 * tw_exchange_pack: d_send ((n_loc+m_loc) records of 16 bytes) grouped by destination rank g,
 *   each group [X records | Z records] in the order of the send counts; a record is {value
 *   bits, destination-local position}, Z positions offset by n_loc, so the receiver scatters
 *   everything into one [X | Z] array with tw_scatter_records. */
/* Tuning hook: grid cap (blocks) of tw_exchange_counts / tw_exchange_pack /
 * tw_scatter_records, which run beside a count kernel (0 = default).  Results do not
 * depend on it. */
int tw_exchange_set_grid(int32_t blocks);
int tw_exchange_counts(int64_t n_loc, int64_t m_loc, int32_t rank, int32_t G, uint64_t key_x,
                       uint64_t key_z, uint64_t* d_counts, uint64_t* d_cursor, void* stream);
int tw_exchange_pack(const void* d_x, int64_t n_loc, const void* d_z, int64_t m_loc, int32_t rank,
                     int32_t G, uint64_t key_x, uint64_t key_z, const uint64_t* d_counts,
                     uint64_t* d_cursor, void* d_send, void* stream);
/* Fixed-capacity variant (the default exchange of ShardedSample): ONE forward-permutation pass,
 * no count pass and no host round trip.  d_send holds G buckets of (1 + cap) records: bucket g =
 * [header {count, 0} | records {value bits, position at rank g (Z offset by n_loc)}], so the
 * all-to-all is an equal-split one (G*(1+cap) records each way).  d_cursor (G uint64) must be
 * zero on the first call; it is left zero for the next.  A bucket over cap sets *d_flag (the
 * records past cap are dropped): the caller must check the flag before using the result.
 * tw_scatter_buckets: for every received bucket, d_out[pos] = value for its first
 * min(header, cap) records; a header over cap or a position outside [0, n_out) sets *d_flag.
 * Replaces the same reference loop as tw_exchange_pack (compute_stats.py:64-67 per rank). */
int tw_exchange_pack_fixed(const void* d_x, int64_t n_loc, const void* d_z, int64_t m_loc,
                           int32_t rank, int32_t G, uint64_t key_x, uint64_t key_z, int64_t cap,
                           uint64_t* d_cursor, void* d_send, int32_t* d_flag, void* stream);
int tw_scatter_buckets(const void* d_recv, int32_t G, int64_t cap, void* d_out, int64_t n_out,
                       int32_t* d_flag, void* stream);

/* ---- (e): row exchange for the row-partitioned learning layout ------------------------
 * Replaces the row copies of SWR_divide (compute_stats.py:48-54) when X is split by rows over
 * G ranks.  d_rows: the M = N*k global row indices of all N shards (shard-major; identical on
 * every rank).  Requester q owns positions [q*M_q, (q+1)*M_q).  This rank owns matrix rows
 * [lo, hi), stored row-major as d_part ((hi-lo) x d).
 * tw_row_route_counts: d_counts[q] = #positions of q whose row lies in [lo, hi).
 * tw_row_pack: one record of d+1 doubles per such position into d_send — the row, then the
 *   requester-local position bit-cast to a double — requester q's records occupying
 *   [d_start[q], d_start[q] + d_counts[q]) (order inside a bucket unspecified); d_cursor: G
 *   int64 of scratch.  G <= 1024.
 * tw_row_unpack: d_out[pos*d + c] = record[c] for m received records. */
int tw_row_route_counts(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi,
                        int32_t G, int64_t* d_counts, void* stream);
int tw_row_pack(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi, int32_t G,
                const double* d_part, int64_t d, const int64_t* d_start, int64_t* d_cursor,
                double* d_send, void* stream);
int tw_row_unpack(const double* d_rec, int64_t m, int64_t d, double* d_out, void* stream);
/* Remote rows only (the learning layout's default): this rank's matrix is [partition |
 * receive area], and its row tables point into it — owned draws at their partition row, the
 * others where the exchange lands them.  Nothing owned is copied; at G = 1 nothing moves.
 * tw_row_route_remote_counts: tw_row_route_counts with d_counts[me] = 0 (me: this rank).
 * tw_row_pack_remote: requester q's bucket starts at word d_start[q] of d_send and holds
 *   d_count[q] rows (d doubles each; order unspecified) followed by their requester-local
 *   positions (bit-cast int64), padded by the caller to whole rows: ceil(d_count[q] / d) * d
 *   words.  d_cursor: G int64 of scratch.
 * tw_row_table_local: d_table[i] = d_rows[i] - lo for this rank's M_q positions whose row it
 *   owns (d_rows: its own slice of the draws), -1 for the others.
 * tw_row_table_remote: for the `total` records received (source g's bucket at word
 *   d_rstart[g] of d_recv, d_rcount[g] records, d_rprefix[g] = sum of the counts before g):
 *   d_table[position] = base + d_rstart[g] / d + j for record j — d_recv being the receive
 *   area of the matrix at row `base` (the partition's row count); a position outside
 *   [0, table_len), or a record past recv_len words, is not used and raises *d_bad (position
 *   + 1, or 2^62: a protocol error the caller reports; d_bad may be NULL). */
int tw_row_route_remote_counts(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo,
                               int64_t hi, int32_t G, int32_t me, int64_t* d_counts,
                               void* stream);
int tw_row_pack_remote(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi,
                       int32_t G, int32_t me, const double* d_part, int64_t d,
                       const int64_t* d_start, const int64_t* d_count, int64_t* d_cursor,
                       double* d_send, void* stream);
int tw_row_table_local(const int64_t* d_rows, int64_t M_q, int64_t lo, int64_t hi,
                       int64_t* d_table, void* stream);
int tw_row_table_remote(const double* d_recv, int32_t G, const int64_t* d_rstart,
                        const int64_t* d_rcount, const int64_t* d_rprefix, int64_t total,
                        int64_t d, int64_t base, int64_t* d_table, int64_t table_len,
                        int64_t recv_len, int64_t* d_bad, void* stream);

/* ---- (e) single-process multi-device communicator (RCCL over xGMI) --------------------
 * The reference's workers are one serial in-process loop (compute_stats.py:71-91,
 * estimation-experiment/main.py:48-68), so the drop-in API drives all of the node's GPUs
 * from ONE process: a call's blocks are spread over the devices and their
 * per-block integers combined by an all-gather.  RCCL is bound at run time (the copy already
 * in the process, else the system librccl.so.1); without it tw_comm_init returns TW_ERR_HIP
 * and the caller gathers on the host (same integers).
 * tw_comm_init: one communicator over ndev distinct devices (ncclCommInitAll) -> *out_comm.
 * tw_allgather_u64 / _f64: for every k, device devs[k] sends count words from d_send[k] and
 *   receives ndev*count words (rank order) into d_recv[k], on streams[k] (hipStream_t of
 *   device k); pointer arrays are host arrays of ndev device pointers. */
int tw_comm_init(int32_t ndev, const int32_t* devs, int32_t* out_comm);
int tw_comm_destroy(int32_t comm);
int tw_allgather_u64(int32_t comm, const uint64_t* const* d_send, uint64_t* const* d_recv,
                     int64_t count, void* const* streams);
int tw_allgather_f64(int32_t comm, const double* const* d_send, double* const* d_recv,
                     int64_t count, void* const* streams);
/* Failure detection (the one entry point here that waits): block until the
 * collectives enqueued on streams[k] (one per device of the communicator) complete, polling
 * ncclCommGetAsyncError on every device's communicator; an RCCL error, a failed stream or
 * timeout_ms (<= 0: the tw_comm_set_timeout default, 60 s) aborts the communicator
 * (ncclCommAbort) and returns TW_ERR_HIP — later calls on the handle fail at once, and the
 * caller gathers on the host instead.  Replaces the wait the reference never needed: its
 * workers are a serial loop (compute_stats.py:71-92). */
int tw_comm_wait(int32_t comm, void* const* streams, int64_t timeout_ms);
int tw_comm_set_timeout(int64_t ms);
/* The deadline of the work queued on the streams BEFORE the last collective (default 600 s):
 * tw_comm_wait waits for it first, outside the collective's own deadline, and aborts the
 * communicator if it has not drained by then (a wedged stream ends in an error, not a hang). */
int tw_comm_set_prior_timeout(int64_t ms);

/* ---- (e) learning over ranks: device-resident gradient exchange (round 5, csrc/peer.hip,
 * csrc/peer.h).  Replaces the per-step all-gather of the shard partials between the gradient
 * and the update launches (the shard mean of make_exps.py:126-141 / compute_stats.py:44-46,
 * split over ranks) by GPU-to-GPU stores into one peer buffer per rank, IPC-mapped into the
 * others.  tw_peer_buffer_bytes: the buffer size for n_total shards of d columns (-1: bad
 * sizes).  tw_peer_alloc: a zeroed UNCACHED device buffer (*out_uncached = 1); fails with
 * TW_ERR_HIP when the driver cannot give uncached memory (no cached fallback: stale lines).  tw_peer_handle / tw_peer_open / tw_peer_close: the 64-byte
 * IPC handle of a buffer, mapped into another process (hipIpcMemLazyEnablePeerAccess).
 * d_peer_bases below: G device addresses in rank order (this rank's own buffer at `rank`). */
int64_t tw_peer_buffer_bytes(int32_t n_total, int64_t d);
int tw_peer_alloc(int64_t bytes, void** d_out, int32_t* out_uncached);
int tw_peer_free(void* d_ptr);
int tw_peer_handle(void* d_ptr, uint8_t* out_handle);
int tw_peer_open(const uint8_t* handle, void** d_out);
int tw_peer_close(void* d_ptr);
/* Setup handshake: tw_peer_hello stores `token` into this rank's hello word of every rank's
 * buffer (and waits for it); after a host barrier over the ranks, tw_peer_check sets *out_ok
 * = 1 when its own buffer's G hello words all hold `token`. */
int tw_peer_hello(void* const* d_peer_bases, int32_t G, int32_t rank, uint64_t token,
                  void* stream);
int tw_peer_check(void* d_my_base, int32_t G, uint64_t token, int32_t* out_ok);
/* Per-step form, ONE launch after the gradient launch, parity par = step & 1: this rank's
 * `words` partial words (its shards' rows, global offset offset_words = shard_base * d) stored
 * into every rank's slot and the launch's arrivals added to every rank's counter; then the
 * launch waits (bounded: 20 s, *d_abort raised on timeout) until all G ranks' arrivals are in
 * and applies tw_sgd_update's arithmetic to the n_total x d slot (same bits), d_step advanced
 * by one when given.  Uneven shard splits need nothing more: the arrivals per rank depend on
 * d only. */
int tw_peer_step(const double* d_grads_loc, int64_t words, int64_t offset_words,
                 void* const* d_peer_bases, int32_t G, int32_t rank, int32_t n_total, int64_t d,
                 int32_t par, double* d_w, double* d_dw, double reg, double lr, double momentum,
                 uint64_t* d_step, uint32_t* d_abort, void* stream);
/* Column-owned per-step form (round 6): tw_peer_step's arguments and the same w / dw bits on
 * every rank; rank p sums and updates only columns [p d / G, (p+1) d / G) (each rank pushes
 * each partial column to its owner only, owners publish their updated columns to every rank).
 * words and offset_words are whole rows (multiples of d). */
int tw_peer_step_cols(const double* d_grads_loc, int64_t words, int64_t offset_words,
                      void* const* d_peer_bases, int32_t G, int32_t rank, int32_t n_total,
                      int64_t d, int32_t par, double* d_w, double* d_dw, double reg, double lr,
                      double momentum, uint64_t* d_step, uint32_t* d_abort, void* stream);
/* The narrow persistent segment (tw_sgd_segment_narrow) over ranks: this rank's n_shards
 * blocks (global shards shard_base..) push every step's gradients into every rank's peer
 * buffer and wait for all n_total shards on their own; the last update is applied in the
 * launch (d_w / d_dw in place; d_step += nsteps when given).  Replay draws d_ix / d_iz: this
 * rank's first shard's rows (draw_stride per step); device RNG: d_ix = d_iz = NULL, and
 * swr_mod > 0 draws the SWR rows in the kernel (else the row tables d_rows_x / d_rows_z).
 * d_ctl[1]: the abort word. */
int tw_sgd_segment_narrow_peer(const double* d_X, const double* d_Z, int64_t d,
                               const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                               int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                               int64_t draw_stride, int32_t n_shards, int64_t B, double margin,
                               int32_t loss, uint64_t seed, uint64_t* d_step,
                               int32_t shard_base, int32_t nsteps, int64_t n_X, int64_t n_Z,
                               int64_t swr_mod, double* d_w, double* d_dw, double reg,
                               double lr, double momentum, uint32_t* d_ctl,
                               void* const* d_peer_bases, int32_t G, int32_t rank,
                               int32_t n_total, void* stream);

/* ---- f2: bulk draws of NumPy's legacy global RNG (host code, no GPU) ------------------
 * key (624 words) / pos: the MT19937 state of np.random.get_state(), advanced in place.
 * tw_np_randint_batch: n_calls consecutive RandomState.randint(low[c], high[c], cnt[c]) calls
 * (int64 output, NumPy's masked-rejection algorithm), values concatenated into out; returns
 * 0, or 1 when a range is empty (high <= low).  Replaces the per-shard randint calls of
 * grad_inc_block (compute_stats.py:155-156) and SWR_divide (:52-53) in replay mode.
 * tw_np_mt_next32: the raw genrand_int32 stream. */
int tw_np_randint_batch(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                        const int64_t* high, const int64_t* cnt, int64_t* out);
/* tw_np_randint_batch narrowed to uint16, for calls on [0, high) with high <= 65536 (SWR_divide's
 * rows for the replay loop's narrowed row tables); 1 for any other call (state untouched). */
int tw_np_randint_batch_u16(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                            const int64_t* high, const int64_t* cnt, uint16_t* out);
int tw_np_mt_next32(uint32_t* key, int32_t* pos, int64_t cnt, uint32_t* out);
/* grad_inc_block's draws for every shard of one UN_split call: for s < N, randint(0,kx,B)
 * into ix[s*B..] then randint(0,kz,B) into iz[s*B..].  Returns 1 if kx or kz <= 0. */
int tw_np_randint_pairs(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz,
                        int64_t B, int64_t* ix, int64_t* iz);
/* S consecutive steps of those draws (the replay loop's segment between two reshuffles):
 * out is (S, 2, N, B) int64 — out[s][0] the step's X indices, out[s][1] its Z indices. */
int tw_np_randint_pairs_steps(uint32_t* key, int32_t* pos, int32_t S, int32_t N, int64_t kx,
                              int64_t kz, int64_t B, int64_t* out);
/* The same draws narrowed to uint16 (needs kx, kz <= 65536): a quarter of the bytes for the
 * replay loop's host-to-device copy; tw_widen_u16 restores the int64 indices on the device. */
int tw_np_randint_pairs_steps_u16(uint32_t* key, int32_t* pos, int32_t S, int32_t N,
                                  int64_t kx, int64_t kz, int64_t B, uint16_t* out);
/* The same draws narrowed to uint8 (needs kx, kz <= 256): half the bytes of the uint16 form. */
int tw_np_randint_pairs_steps_u8(uint32_t* key, int32_t* pos, int32_t S, int32_t N,
                                 int64_t kx, int64_t kz, int64_t B, uint8_t* out);
/* d_out[i] = d_in[i] (uint16 -> int64) for i < n, on `stream`; d_in may be the device address
 * of pinned host memory (tw_host_device_pointer): the kernel then reads it over PCIe, 16 B per
 * lane when d_in is 16-B aligned. */
int tw_widen_u16(const uint16_t* d_in, int64_t n, int64_t* d_out, void* stream);
/* The same for uint8 indices. */
int tw_widen_u8(const uint8_t* d_in, int64_t n, int64_t* d_out, void* stream);
/* The replay loop's segment upload in one launch: widen n narrowed draws (width 1 = uint8,
 * 2 = uint16) d_in -> d_out as above, and copy nx + nz 8-byte row indices d_rows ->
 * d_rows_x[0:nx], d_rows_z[0:nz] (a reshuffle's SWR tables; nx = nz = 0: none).  Either
 * source may be mapped host memory.  Replaces learning-experiment/make_exps.py:123-125's
 * SWR_divide hand-off + compute_stats.py:155-156's draws for one segment of steps. */
int tw_ship_draws(const void* d_in, int32_t width, int64_t n, int64_t* d_out,
                  const void* d_rows, int64_t nx, int64_t* d_rows_x, int64_t nz,
                  int64_t* d_rows_z, void* stream);
/* tw_ship_draws for a segment running through reshuffles: d_rows holds ntab tables, each
 * [nx x values | nz z values] of row_width bytes (8: int64, 2: uint16, widened), copied into
 * ntab consecutive tables of the stacks d_rows_x
 * (nx words apart) and d_rows_z (nz apart) — the input of tw_sgd_segment_narrow_tables. */
int tw_ship_draws_tables(const void* d_in, int32_t width, int64_t n, int64_t* d_out,
                         const void* d_rows, int32_t row_width, int32_t ntab, int64_t nx,
                         int64_t* d_rows_x, int64_t nz, int64_t* d_rows_z, void* stream);
/* The replay loop's draws made ahead on a native thread (csrc/drawpipe.hip): segment j of
 * n_seg (seg_steps[j] steps, its first step being step seg_phase[j] of a reshuffle period of
 * `mod` steps: a reshuffle before each of its steps k with (seg_phase[j] + k) % mod == 0) is
 * drawn from NumPy's MT19937 state (key/pos, advanced in place) into ring buffer j % nbuf, in
 * the reference's order: each reshuffle's SWR rows (make_exps.py:123-125,
 * compute_stats.py:48-54: N randint calls on [0, n_X) of n_X / N values, then N on [0, n_Z))
 * into the next of row_tabs tables of row_bufs[k] (N * (n_X/N + n_Z/N) values each, of
 * row_width bytes: 8 = int64, 2 = uint16 when n_X, n_Z <= 65536),
 * then the pairs (compute_stats.py:155-156) of the steps up to the next reshuffle into
 * seg_bufs[k] as (S, 2, N, B) values of `width` bytes (1, 2 or 8).  A segment with more
 * reshuffles than row_tabs fails the worker.  tw_draw_pipe_wait blocks until segment j is drawn; tw_draw_pipe_shipped records
 * that the uploads reading its buffers are enqueued on `stream` (the worker refills them only
 * after they have run); tw_draw_pipe_stop cancels what is not drawn, joins and frees.
 * Nothing else may use NumPy's global RNG between start and stop. */
int tw_draw_pipe_start(uint32_t* key, int32_t* pos, int32_t n_seg, const int32_t* seg_steps,
                       const int32_t* seg_phase, int64_t mod, int32_t N, int64_t kx, int64_t kz,
                       int64_t B, int64_t n_X, int64_t n_Z, int32_t width, int32_t nbuf,
                       void* const* seg_bufs, void* const* row_bufs, int32_t row_tabs,
                       int32_t row_width, void** out_handle);
int tw_draw_pipe_wait(void* handle, int32_t j);
int tw_draw_pipe_shipped(void* handle, int32_t j, void* stream);
int tw_draw_pipe_stop(void* handle);
/* n 8-byte words d_in -> d_out on `stream` (d_in may be mapped host memory, as above). */
int tw_copy_words(const void* d_in, int64_t n, void* d_out, void* stream);
/* learning_process's deferred evaluations (make_exps.py:143-190): one evaluation's nres
 * statistics, the nw words of w and (d_ctl not null) the SGD engine's abort word, written in one
 * launch into h_out, pinned host memory of nres + nw + 1 8-byte words. */
int tw_stage_eval(const void* d_res, int32_t nres, const void* d_w, int32_t nw,
                  const uint32_t* d_ctl, void* h_out, void* stream);
/* The call's final arrays over ranks by ONE exchange (round 6): tw_chain_final_pack packs this
 * rank's walked elements — scores d_x / d_z, rank-image records d_x_rec / d_z_rec, final global
 * positions d_x_pos / d_z_pos (the chains' state after the call's last emission), n_x / n_z a
 * rank — into world buckets of 1 + cap 24-B records {score, record, local position; z: n_x +
 * position} (d_send: world * (cap + 1) * 3 u64; d_cursor: world u64, zero on entry, left
 * zero); after an equal-split all-to-all tw_chain_final_scatter writes every received record
 * at its position of d_x_out / d_x_rec_out / d_z_out / d_z_rec_out (n_x / n_z 8-B words).
 * Replaces est.UnNT's final in-place arrays (main.py:46-47) gathered by inverse chains from
 * all-gathered samples.  Overflows raise *d_flag. */
int tw_chain_final_pack(const void* d_x, const uint64_t* d_x_rec, const uint32_t* d_x_pos,
                        int64_t n_x, const void* d_z, const uint64_t* d_z_rec,
                        const uint32_t* d_z_pos, int64_t n_z, int32_t world, int64_t cap,
                        uint64_t* d_cursor, void* d_send, int32_t* d_flag, void* stream);
int tw_chain_final_scatter(const void* d_recv, int32_t world, int64_t cap, int64_t n_x,
                           int64_t n_z, void* d_x_out, void* d_x_rec_out, void* d_z_out,
                           void* d_z_rec_out, int32_t* d_flag, void* stream);
/* The final global positions of this rank's elements (x: x_base + e, z: z_base + e) after
 * `steps` chained permutations of the n_x_all / n_z_all domains (keys as tw_chain_emit's): the
 * chain state tw_chain_emit leaves after the same steps, computed without emitting, so that
 * tw_chain_final_pack can run at a call's start beside its emissions and counts (main.py:46-47's
 * final arrays, est.UnNT). */
int tw_chain_walk(int64_t x_base, int64_t n_x, int64_t n_x_all, int64_t z_base, int64_t n_z,
                  int64_t n_z_all, const uint64_t* keys_x, const uint64_t* keys_z, int32_t steps,
                  uint32_t* d_x_pos, uint32_t* d_z_pos, void* stream);
/* A chunk's receive side over ranks in ONE call (round 6): tw_chain_unpack (its arguments, in
 * order) then tw_count_pairs_chain on the filled bags (shard offsets d_x_off / d_z_off, largest
 * shards max_nx / max_nz, bag strides n_x / n_z, out [steps][n_shards]), the cursors and the
 * counts zeroed by one launch — est.UnNT's per-step counts (main.py:72-79) of a chunk. */
int tw_chain_unpack_count(const uint64_t* d_recv, int32_t world, int32_t steps, int64_t cap,
                          int32_t half, int64_t n_x, int64_t n_z, int64_t x_shard,
                          int64_t z_shard, int32_t n_shards, void* d_x_bag, void* d_z_bag,
                          uint32_t* d_cursors, int32_t* d_flag, const int64_t* d_x_off,
                          const int64_t* d_z_off, int64_t max_nx, int64_t max_nz,
                          uint64_t* d_out, void* stream);
/* The incomplete statistic on the step chains over ranks (cs.UnNBT, compute_stats.py:119-123,
 * with device-RNG draws): tw_chain_unpack_exact writes every received record {image, local
 * position} of a chunk's (source, step) buckets (tw_chain_emit's exchange layout, strict
 * images) at its exact position of the step's bags [steps][n_x] / [steps][n_z];
 * tw_count_pairs_chain_rng counts B device-drawn pairs (tw_count_pairs_rng's Philox/Lemire
 * draws, step c keyed seed + c, shard streams stream_id + s) of every (step, shard) bag on
 * those images, out [steps][n_shards] (zeroed here). */
int tw_chain_unpack_exact(const uint64_t* d_recv, int32_t world, int32_t steps, int64_t cap,
                          int64_t n_x, int64_t n_z, void* d_x_bag, void* d_z_bag,
                          int32_t* d_flag, void* stream);
int tw_count_pairs_chain_rng(const float* d_x_bag, const int64_t* d_x_off, int64_t x_stride,
                             const float* d_z_bag, const int64_t* d_z_off, int64_t z_stride,
                             int32_t n_shards, int32_t steps, int64_t max_nx, int64_t max_nz,
                             int64_t B, uint64_t seed, uint64_t stream_id, uint64_t* d_out,
                             void* stream);
/* The carried rank images' validity check (ShardedSample.UnN_many, device.py CARRY_IMAGES;
 * the arrays only ever permute between calls, estimation-experiment/main.py:43-44): *d_acc =
 * sum over the na + nb 8-byte words of [d_a | d_b] of a position-keyed 64-bit hash (d_acc:
 * tw_words_checksum_acc_words() u64 words, the rest scratch for the blocks' partials).  With
 * d_expect (one device word) and d_verdict (one int64; device or mapped host memory) both set,
 * also *d_verdict = (*d_acc == *d_expect) ? good : bad, in stream order. */
int tw_words_checksum(const void* d_a, int64_t na, const void* d_b, int64_t nb, void* d_acc,
                      const void* d_expect, void* d_verdict, int64_t good, int64_t bad,
                      void* stream);
int64_t tw_words_checksum_acc_words(void);
/* The device address of pinned, mapped host memory (hipHostGetDevicePointer); TW_ERR_ARG when
 * `host` is not such memory. */
int tw_host_device_pointer(void* host, void** out_dev);
/* np.random.shuffle(x); np.random.shuffle(z) — the in-place shuffles of UN
 * (compute_stats.py:66-67, estimation-experiment/main.py:46-47) — on C-contiguous arrays of
 * nx / nz items of isx / isz bytes (rows of a 2-D array are items): legacy RandomState's
 * _shuffle_raw restated (i = n-1 down to 1: j = masked-rejection draw on [0, i], swap), the same
 * draws from the same stream and the same final arrays; x's swaps run on a second thread while
 * z's draws and swaps run.  jbuf: nx + nz int64 of scratch.  Returns 2 on bad arguments. */
int tw_np_shuffle_pair(uint32_t* key, int32_t* pos, void* x, int64_t nx, int64_t isx, void* z,
                       int64_t nz, int64_t isz, int64_t* jbuf);
/* The index draws of np.random.shuffle on n <= 2^31 items WITHOUT the swaps (j[i] for
 * i = n-1 down to 1; j[0] untouched), advancing the state as the shuffle would: the host half
 * of the device shuffle below.  Returns 2 on bad arguments. */
int tw_np_shuffle_draws32(uint32_t* key, int32_t* pos, int64_t n, uint32_t* j);
/* The same draws for i = hi down to lo only (1 <= lo <= hi < n; j is the shuffle's n-entry
 * array, other entries untouched), the state advanced past them: consecutive ranges from
 * hi = n - 1 down to lo = 1 make exactly tw_np_shuffle_draws32's draws (the streamed last
 * shuffle of the drop-in).  Returns 2 on bad arguments. */
int tw_np_shuffle_draws32_range(uint32_t* key, int32_t* pos, int64_t n, int64_t hi, int64_t lo,
                                uint32_t* j);

/* ---- Device shuffle swaps (csrc/devshuffle.hip): the swaps of np.random.shuffle(x) and
 * np.random.shuffle(z) (UN's in-place shuffles, compute_stats.py:66-67,
 * estimation-experiment/main.py:46-47) on 8-byte items in HBM, from the host's draws
 * (tw_np_shuffle_draws32): for i = n-1 down to 1, swap a[i] and a[j[i]] — run as parallel
 * rounds with deterministic reservations, giving the sequential loop's permutation bit for bit.
 * One call enqueues tw_shuffle_swaps_rounds(nx, nz) rounds (first = 1, round0 = 0 on the first
 * call; later calls: first = 0, round0 += rounds) and writes the number of iterations still
 * pending to *d_pending (device u32); the caller repeats while it is non-zero (one call
 * suffices w.h.p.).  nx + nz < 2^31.  d_work: tw_shuffle_swaps_work_bytes bytes. */
int64_t tw_shuffle_swaps_work_bytes(int64_t nx, int64_t nz);
int32_t tw_shuffle_swaps_rounds(int64_t nx, int64_t nz);
/* rounds per batch (0 = the default 4.5 ln n + 24; at least 17): a test hook that forces resumed batches */
int tw_shuffle_swaps_set_rounds(int32_t rounds);
/* 1 (default): the tail rounds of a batch (every chunk entered, a short pending list) run in
 * one workgroup launch; 0: one launch per round.  Process-global; results do not depend on it. */
int tw_shuffle_swaps_set_tail(int32_t on);
int tw_shuffle_swaps(uint64_t* d_x, int64_t nx, uint64_t* d_z, int64_t nz, const uint32_t* d_jx,
                     const uint32_t* d_jz, int32_t first, int32_t round0, void* d_work,
                     uint32_t* d_pending, void* stream);
/* The draw windows of the rounds: iterations enter in W = tw_shuffle_swaps_windows() chunks of
 * p = ceil((n - 1) / W) draws, window c holding i in [max(1, n - (c + 1) p), n - c p). */
int32_t tw_shuffle_swaps_windows(void);
/* The first batch (first = 1, round0 = 0) of tw_shuffle_swaps enqueued in parts as the draws
 * arrive: rounds [r_begin, r_end) — round r reads windows 0 .. r + 1, so with windows [0, c)
 * on the device r_end = c - 1 (< W); r_begin = 0 also clears the workspace and reserves round
 * 0; last != 0 enqueues the remaining rounds, the tail and *d_pending (r_end ignored).  The
 * parts in sequence (each r_begin = the previous r_end) equal one tw_shuffle_swaps call. */
int tw_shuffle_swaps_part(uint64_t* d_x, int64_t nx, uint64_t* d_z, int64_t nz,
                          const uint32_t* d_jx, const uint32_t* d_jz, int32_t r_begin,
                          int32_t r_end, int32_t last, void* d_work, uint32_t* d_pending,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TUPLEWISE_H */
