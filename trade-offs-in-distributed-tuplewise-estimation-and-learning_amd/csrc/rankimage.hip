// rankimage.hip — the all-pairs count of est.UnN on packed-f32 RANK IMAGES (SURVEY.md §8 rows
// A1/A6/A7; round 3).
//
// Reference: est.Un   estimation-experiment/main.py:29-31   mean(X[:,None] > Z[None,:])
//            est.UnN / UnNT   estimation-experiment/main.py:72-79 (the repartition loop)
//
// Why images.  csrc/count.hip compares the doubles themselves: one v_cmp_f64 per 64 pairs plus
// the count of its 64 result bits (a carry-add on the VALU or s_bcnt1 + s_add on the scalar
// unit) — an instruction mix whose issue ceiling is ~0.63 of the lane-op peak (DESIGN.md
// §4.1).  Packed f32 VALU ops (v_pk_*_f32, full rate on gfx950) process TWO lanes' worth per
// instruction, and with integer-valued operands a compare-and-count is two of them:
//     t   = clamp(gx + nz)           v_pk_add_f32 ... clamp   (nz = -gz from an SGPR)
//     acc = acc + t                  v_pk_add_f32
// where clamp(gx - gz) is exactly 1 when gx - gz >= 1 and 0 when gx - gz <= 0.  That is 1 VALU
// wave-instruction per 64 pairs and nothing on the scalar unit (tools/mb_pk.hip: 0.88 of the
// lane-op peak on the bench shape, profiles/r03_mb_pk.log).
//
// The images.  Over ONE call (est.UnNT's T repartitions) the multiset of scores does not change,
// only which shard holds which score.  So the images are computed once per call from the whole
// sample: every element v (of X or of Z) gets
//     g(v) = #{z in Z : key(z) < key(v)}      (order keys: NaN last, -0 == +0)
// Then for any x, z:  x > z  <=>  g(x) > g(z)  <=>  g(x) - g(z) >= 1.  (x > z: every z' <= z
// is < x, z itself included, so g(x) >= g(z) + 1.  x <= z: every z' < x is < z, so
// g(x) <= g(z).)  NaN x get -2^25 (never greater); a NaN z has g = #non-NaN z >= every g(x)
// (never less).  Images are integers <= m < 2^24, so every f32 sum g(x) - g(z) is exact;
// the sentinel is an exact power of two and keeps its sign.  Per pair the count is the
// reference's integer, bit for bit.
//
// State between steps.  An element is an 8-B record: low word = its f32 image (negated for z),
// high word = its index in the call's input array.  The repartition permutes records exactly as
// it permuted doubles (nextstep.h: the next step's gather rides on the tail blocks of the count
// launch, the same 8 B per element), and at the end of the call one gather writes the doubles in
// the final order (tw_gather_records).
//
// The ranking (once per call) is a bucket count, not a sort of all n + m elements: a sorted
// sample of Z gives B - 1 splitters; every element goes to the interval bucket between two
// splitters or to the EQUALITY bucket of a splitter (heavy ties land there, where g is the same
// for every element); per bucket the z keys are sorted in LDS and every element's g is the z
// count of the lower buckets plus a binary search in its own.  See tw_rank_images below.
#include "nextstep.h"
#include "pkcount.h"
#include "sortkeys.h"

namespace tw {

// ----------------------------------------------------------------------------- images
// g(v) = #{z : key(z) < key(v)} for all n + m elements, from a structure over Z alone:
//  1. a sample of Z at hashed positions, sorted (by counting, over C / 64 blocks from C = 1024
//     keys): B - 1 splitter keys;
//  2. z -> bucket: 2j for the keys strictly between splitters j-1 and j, 2j + 1 for keys EQUAL
//     to splitter j (heavy ties land there: no z of such a bucket is below any of its values);
//     per-block histograms (each z's bucket kept), their prefix per bucket, and the z keys
//     scattered bucket by bucket (the bucket starts scanned in the scatter blocks);
//  3. per interval bucket, a counting sort of its z keys over 2048 sub-buckets by a monotone map
//     (linear in the value or in the order key, whichever spreads the bucket's z better; so
//     sub(z) < sub(v) => z < v), into a second key array, with the sub-bucket prefix table;
//  4. every element, in input order (coalesced record stores): bucket by splitter search, then
//     g = z count below the bucket + below its sub-bucket + a scan of its own sub-bucket (about
//     one key for smooth data; ties or clusters only lengthen the scan, never change g).
constexpr int kRkThreads = 256;
constexpr int kRkSample = 2048;                    // largest sample (one k_sort_chunks block)
// tuning hooks (tw_rank_set_plan): sample size, z per thread in the bucket passes (1024 / 8:
// 145 us per 1e6 + 1e6 ranking against 169-172 us for 2048 / 16; profiles/r04_chain_parts.log)
static int g_rank_cs = 1024;
static int g_rank_per = 8;
// small Z (m <= kRkSmallM, the one-shot C2 counts): a shorter sample (its one-block sort is a
// serial latency chain: 15 us for 1024 keys) and shorter interval buckets (more sub-sort
// blocks); tw_rank_set_small
constexpr int64_t kRkSmallM = 1 << 18;
static int g_rank_cs_small = 256;
static int g_rank_zint_small = 2048;
static int g_rank_per_small = 4;  // 43 vs 47 us at 1e5 + 1e5 (profiles/r04s7_rank_small_per*.log)
constexpr int kRkMaxB = 256;                       // splitter intervals (511 buckets max)
constexpr int kRkSub = 2048;                       // sub-buckets per interval bucket
// sub-buckets of more than kRkSortedMin keys (ties, skew) are sorted in place by the sub-sort
// (up to kRkSortedMax keys) and binary-searched by the record pass, whose scan of a sub-bucket
// was otherwise unbounded (1000 copies of each of 1000 values took 3.6 ms)
constexpr uint32_t kRkSortedMin = 32;
constexpr uint32_t kRkSortedMax = 4096;
constexpr uint32_t kRkWaveSortMax = 1024;  // sorted by one wave (16 keys per lane)

// position of sample i in [0, m): a hashed, not an index-strided, sample (Z with periodic
// structure would give an evenly spaced sample of repeated values)
__device__ __forceinline__ int64_t sample_index(int i, int64_t m) {
  return (int64_t)(((uint64_t)mix32((uint32_t)i * 0x9E3779B1u + 0x7F4A7C15u) * (uint64_t)m) >> 32);
}

// the sample of C >= 1024 keys (Z beyond kRkSmallM), sorted by counting over C / 64 blocks
// (one block's bitonic network was a serial chain of ~50 shuffle levels: 16 us at C = 1024,
// the longest of the ranking's structure launches; 8 blocks placing 128 keys each: 10 us):
// every block draws the whole sample into LDS (cs hashed positions of z, padded with ~0) and
// places 64 of its keys — key i goes to #{j : k_j < k_i} + #{j < i : k_j == k_i}, sixteen
// threads per key each counting a C / 16 share (a wave's lanes hold different keys and read
// the same k_j: LDS broadcasts), the shares added with LDS atomics.  The sorted array is the
// bitonic one's, key for key.
constexpr int kRkSampPlace = 64;  // keys placed per block
template <typename T>
__global__ __launch_bounds__(1024) void k_rank_sample_count(const T* __restrict__ z, int64_t m,
                                                            int cs, int C,
                                                            uint64_t* __restrict__ ss) {
  __shared__ uint64_t keys[kRkSample];
  __shared__ uint32_t cnt[kRkSampPlace];
  const int tid = threadIdx.x;
  for (int i = tid; i < C; i += 1024) keys[i] = i < cs ? order_key<T>(z[sample_index(i, m)]) : ~0ull;
  if (tid < kRkSampPlace) cnt[tid] = 0;
  __syncthreads();
  constexpr int kParts = 1024 / kRkSampPlace;
  const int q = tid % kRkSampPlace, part = tid / kRkSampPlace;
  const int i = (int)blockIdx.x * kRkSampPlace + q;
  const uint64_t ki = keys[i];
  const int span = C / kParts, j0 = part * span;  // a multiple of 4 (C >= 1024)
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  for (int j = j0; j < j0 + span; j += 4) {
    const uint64_t a = keys[j], b = keys[j + 1], c = keys[j + 2], d = keys[j + 3];
    c0 += (a < ki || (a == ki && j < i)) ? 1u : 0u;
    c1 += (b < ki || (b == ki && j + 1 < i)) ? 1u : 0u;
    c2 += (c < ki || (c == ki && j + 2 < i)) ? 1u : 0u;
    c3 += (d < ki || (d == ki && j + 3 < i)) ? 1u : 0u;
  }
  atomicAdd(&cnt[q], c0 + c1 + c2 + c3);
  __syncthreads();
  if (tid < kRkSampPlace) ss[cnt[tid]] = keys[(int)blockIdx.x * kRkSampPlace + tid];
}

// the sample drawn and sorted in one block: keys of z at cs hashed positions, padded with ~0
// to C (a power of two >= 256), sorted by counting — key i goes to #{j : k_j < k_i} + #{j < i :
// k_j == k_i}: 1024 threads, each counting one key against a 1 / (1024 / C) share of the keys
// (LDS broadcasts, four independent partial counts), the shares added with LDS atomics; for
// C <= 512 (the bitonic network on one block is a serial chain of ~40 shuffle levels: 8.8 us
// at C = 256 against 5.6)
template <typename T>
__global__ __launch_bounds__(1024) void k_rank_sample_sort(const T* __restrict__ z, int64_t m,
                                                           int cs, int C,
                                                           uint64_t* __restrict__ ss) {
  __shared__ uint64_t keys[kRkSample];
  __shared__ uint32_t cnt[kRkSample];
  constexpr int kMaxPer = kRkSample / 1024;
  const int tid = threadIdx.x;
  const int per = C > 1024 ? C / 1024 : 1;     // keys per thread
  const int parts = C >= 1024 ? 1 : 1024 / C;  // threads per key
  for (int u = 0; u < per; ++u) {  // load and zero (every slot written once)
    const int i = tid + u * 1024;
    if (i < C) {
      keys[i] = i < cs ? order_key<T>(z[sample_index(i, m)]) : ~0ull;
      cnt[i] = 0;
    }
  }
  __syncthreads();
  const int part = tid / (C < 1024 ? C : 1024);
  const int j0 = part * (C / parts), j1 = j0 + C / parts;
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    if (u >= per) break;
    const int i = (C < 1024 ? tid % C : tid) + u * 1024;
    const uint64_t ki = keys[i];
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int j = j0; j < j1; j += 4) {  // C / parts is a multiple of 4
      const uint64_t a = keys[j], b = keys[j + 1], c = keys[j + 2], d = keys[j + 3];
      c0 += (a < ki || (a == ki && j < i)) ? 1u : 0u;
      c1 += (b < ki || (b == ki && j + 1 < i)) ? 1u : 0u;
      c2 += (c < ki || (c == ki && j + 2 < i)) ? 1u : 0u;
      c3 += (d < ki || (d == ki && j + 3 < i)) ? 1u : 0u;
    }
    atomicAdd(&cnt[i], c0 + c1 + c2 + c3);
  }
  __syncthreads();
  for (int u = 0; u < per; ++u) {
    const int i = tid + u * 1024;
    if (i < C) ss[cnt[i]] = keys[i];
  }
}

// bucket of a key: 2j for the interval below splitter j (j = #splitters < key), 2j + 1 for a key
// equal to splitter j; bucket order is key order
__device__ __forceinline__ int rank_bucket(const uint64_t* sp, int nsp, uint64_t k) {
  int lo = 0, n = nsp;  // lower_bound over sp[0..nsp)
  while (n > 0) {
    const int h = n >> 1;
    if (sp[lo + h] < k) {
      lo += h + 1;
      n -= h + 1;
    } else {
      n = h;
    }
  }
  return 2 * lo + ((lo < nsp && sp[lo] == k) ? 1 : 0);
}

// m: the Z of the STRUCTURE (every z counted by g); n / mq: the X / Z elements whose images the
// record pass writes (the same Z as the structure in one process; a rank's own share of X and Z
// against the all-gathered Z over several ranks, tw_rank_images_query); tot = n + mq.
// half: the X record's high word holds h(x) = #{z : key(z) <= key(x)} instead of the index.
// compact: images without indices (x: f32, or the {g, h} f32 pair when half; z: f32), the
// layout of tw_count_pairs_chain's bags
struct RankGeo {
  int64_t n, m, tot, mq;
  int B, NB, nblk, cs, half, per, C;  // C: the sorted sample's padded length (power of two)
  int compact;
};

// splitter j = the sample's ((j + 1) * cs / B)-th key; loaded into LDS by every pass
__device__ __forceinline__ int load_splitters(const uint64_t* __restrict__ ss, const RankGeo& g,
                                              uint64_t* sp) {
  const int nsp = g.B - 1;
  for (int j = threadIdx.x; j < nsp; j += blockDim.x)
    sp[j] = ss[(int)(((int64_t)(j + 1) * g.cs) / g.B)];
  __syncthreads();
  return nsp;
}

// pass 1: per-block bucket histogram of Z (row blk of rel[blk][b]: each block's NB counters
// stored contiguously, and read back the same way by the scatter pass); PER z per thread
template <typename T, int PER>
__global__ __launch_bounds__(kRkThreads) void k_rank_hist(const T* __restrict__ z, RankGeo g,
                                                          const uint64_t* __restrict__ ss,
                                                          uint32_t* __restrict__ rel,
                                                          uint16_t* __restrict__ bid) {
  __shared__ uint64_t sp[kRkMaxB];
  __shared__ uint32_t h[2 * kRkMaxB];
  for (int b = threadIdx.x; b < g.NB; b += kRkThreads) h[b] = 0;
  const int64_t e0 = (int64_t)blockIdx.x * kRkThreads * PER + threadIdx.x;
  T zv[PER];  // all of the thread's loads in flight at once (few waves per CU)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int64_t e = e0 + k * kRkThreads;
    zv[k] = e < g.m ? z[e] : (T)0;
  }
  const int nsp = load_splitters(ss, g, sp);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int64_t e = e0 + k * kRkThreads;
    if (e < g.m) {
      const int b = rank_bucket(sp, nsp, order_key<T>(zv[k]));
      atomicAdd(&h[b], 1u);
      bid[e] = (uint16_t)b;  // the scatter pass reads it instead of searching again
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < g.NB; b += kRkThreads)
    rel[(int64_t)blockIdx.x * g.NB + b] = h[b];
}

// pass 2a: exclusive prefix of every bucket's column of rel[blk][NB] over the blocks (in
// place) and the bucket totals.  A block takes 64 consecutive buckets (one per lane: every
// wave-load is a 256-B run of one rel row) and splits the rows among its 16 waves: each wave
// sums its rows, the waves' sums are scanned in LDS, then each wave walks its rows again writing
// the running prefix — two coalesced passes instead of one strided wave per bucket.
constexpr int kRowsWaves = 16;
__global__ __launch_bounds__(kRowsWaves * kWave) void k_rank_rows(RankGeo g,
                                                                  uint32_t* __restrict__ rel,
                                                                  uint32_t* __restrict__ total) {
  __shared__ uint32_t part[kRowsWaves][kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int b = blockIdx.x * kWave + lane;
  const bool live = b < g.NB;
  const int per = (g.nblk + kRowsWaves - 1) / kRowsWaves;
  const int c0 = wid * per, c1 = min(g.nblk, c0 + per);
  uint32_t sum = 0;
  int c = c0;
  for (; c + 4 <= c1; c += 4) {  // four rows' loads in flight
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = live ? rel[(int64_t)(c + u) * g.NB + b] : 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) sum += v[u];
  }
  for (; c < c1; ++c) sum += live ? rel[(int64_t)c * g.NB + b] : 0u;
  part[wid][lane] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (int w = 0; w < wid; ++w) run += part[w][lane];
  if (wid == kRowsWaves - 1 && live) total[b] = run + sum;
  if (!live) return;
  for (c = c0; c < c1; c += 8) {  // eight rows' loads issued before their stores
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = c + u < c1 ? rel[(int64_t)(c + u) * g.NB + b] : 0u;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (c + u < c1) rel[(int64_t)(c + u) * g.NB + b] = run;
      run += v[u];
    }
  }
}

// passes 2a + 2b in one 1024-thread block when every bucket row fits two wave loads (nblk <= 128: the
// C2-size ranking, where two launches of ~2 us of work each took ~8 us): each wave scans the
// rows of buckets wid, wid + 16, ..., then the block scans the totals
__global__ __launch_bounds__(1024) void k_rank_rows_starts(RankGeo g, uint32_t* __restrict__ rel,
                                                           uint32_t* __restrict__ total,
                                                           uint32_t* __restrict__ start) {
  __shared__ uint32_t a[1024];
  constexpr int kPerWave = 2 * kRkMaxB / (1024 / kWave);  // NB <= 512 rows over 16 waves
  const int t = threadIdx.x, wid = t / kWave, lane = t & (kWave - 1);
  a[t] = 0u;
  // nblk <= 2 kWave here: two values per lane and row, every row's loads issued before the
  // first scan
  uint32_t v[kPerWave][2];
#pragma unroll
  for (int r = 0; r < kPerWave; ++r) {
    const int b = wid + r * (1024 / kWave);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = h * kWave + lane;
      v[r][h] = (b < g.NB && c < g.nblk) ? rel[(int64_t)c * g.NB + b] : 0u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPerWave; ++r) {
    const int b = wid + r * (1024 / kWave);
    if (b >= g.NB) break;
    uint32_t carry = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = h * kWave + lane;
      uint32_t inc = v[r][h];
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += u;
      }
      if (c < g.nblk) rel[(int64_t)c * g.NB + b] = carry + inc - v[r][h];
      carry += __shfl(inc, kWave - 1, kWave);
    }
    if (lane == 0) {
      total[b] = carry;
      a[b] = carry;
    }
  }
  __syncthreads();
  // exclusive scan of the NB <= 512 totals: a wave scan per 64, then the wave totals (two
  // barriers; a Hillis-Steele scan over the block took twenty)
  __shared__ uint32_t wsum[1024 / kWave];
  const uint32_t own = a[t];
  uint32_t inc = own;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wsum[wid] = inc;
  __syncthreads();
  uint32_t before = 0;
  for (int w = 0; w < wid; ++w) before += wsum[w];
  if (t < g.NB) start[t] = before + inc - own;
}

// pass 3: the z keys into their buckets' slots (order inside a bucket is free), by the bucket
// ids the histogram pass kept (no second splitter search).  The bucket starts — the z count
// below every bucket, an exclusive scan of the NB <= 512 totals — are made by every block in
// LDS (two per thread, wave scans) and stored by block 0 for the sub-sort and record passes:
// one launch fewer than a separate scan kernel.
template <typename T, int PER>
__global__ __launch_bounds__(kRkThreads) void k_rank_scatter(const T* __restrict__ z, RankGeo g,
                                                             const uint16_t* __restrict__ bid,
                                                             const uint32_t* __restrict__ rel,
                                                             const uint32_t* __restrict__ total,
                                                             uint32_t* __restrict__ start,
                                                             uint64_t* __restrict__ bkeys) {
  static_assert(2 * kRkMaxB <= 2 * kRkThreads, "two bucket totals per thread");
  __shared__ uint32_t cur[2 * kRkMaxB];
  __shared__ uint32_t wsum[kRkThreads / kWave];
  const int64_t e0 = (int64_t)blockIdx.x * kRkThreads * PER + threadIdx.x;
  T zv[PER];
  uint32_t bv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int64_t e = e0 + k * kRkThreads;
    zv[k] = e < g.m ? z[e] : (T)0;
    bv[k] = e < g.m ? bid[e] : 0u;
  }
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const uint32_t a0 = 2 * t < g.NB ? total[2 * t] : 0u;
  const uint32_t a1 = 2 * t + 1 < g.NB ? total[2 * t + 1] : 0u;
  uint32_t inc = a0 + a1;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wsum[wid] = inc;
  __syncthreads();
  uint32_t ex = inc - (a0 + a1);
  for (int w = 0; w < wid; ++w) ex += wsum[w];
  if (2 * t < g.NB) {
    cur[2 * t] = ex + rel[(int64_t)blockIdx.x * g.NB + 2 * t];
    if (blockIdx.x == 0) start[2 * t] = ex;
  }
  if (2 * t + 1 < g.NB) {
    cur[2 * t + 1] = ex + a0 + rel[(int64_t)blockIdx.x * g.NB + 2 * t + 1];
    if (blockIdx.x == 0) start[2 * t + 1] = ex + a0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (e0 + k * kRkThreads < g.m) bkeys[atomicAdd(&cur[bv[k]], 1u)] = order_key<T>(zv[k]);
}

// The sub-bucket map of an interval bucket, one of two monotone maps (sub(z) < sub(v) => z < v),
// whichever spreads the bucket's z better (the smaller sum of squared sub-bucket counts, i.e.
// the shorter expected scan):
//  * linear in the VALUE between the bucket's smallest and largest finite z:
//    fl(fl(v - lo) * scale) never decreases as v grows; right for bulk buckets, and for the
//    bucket that straddles 0, where every tiny magnitude lies between the two signs' keys;
//  * linear in the ORDER KEY between the bucket's smallest and largest non-NaN z key (a log
//    scale in the magnitude): right for heavy tails (Cauchy-like scores), where a value-linear
//    map crowds the bucket's inner edge into one sub-bucket.
// Both clamp; NaN goes last.
struct SubMap {
  double lo, scale;
  uint64_t klo;
  int kshift, bykey;
  __device__ __forceinline__ uint32_t operator()(double v, uint64_t k) const {
    if (bykey) {
      if (k <= klo) return 0;
      const uint64_t d = (k - klo) >> kshift;
      return d >= (uint64_t)(kRkSub - 1) ? (uint32_t)(kRkSub - 1) : (uint32_t)d;
    }
    if (v != v) return kRkSub - 1;
    const double d = (v - lo) * scale;
    if (!(d > 0.0)) return 0;
    return d >= (double)(kRkSub - 1) ? (uint32_t)(kRkSub - 1) : (uint32_t)d;
  }
};

template <typename T>
__device__ __forceinline__ double key_value(uint64_t k);
template <>
__device__ __forceinline__ double key_value<double>(uint64_t k) {
  return key_to_double(k);
}
template <>
__device__ __forceinline__ double key_value<long long>(uint64_t k) {
  return (double)(long long)(k ^ 0x8000000000000000ull);
}

// block-wide min / max over NT threads (all threads get the result)
template <int NT>
__device__ __forceinline__ void block_minmax(double& lo, double& hi, uint64_t& klo,
                                             uint64_t& khi, double* sd, uint64_t* sk) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, kWave));
    hi = fmax(hi, __shfl_xor(hi, o, kWave));
    const uint64_t a = __shfl_xor(klo, o, kWave), b = __shfl_xor(khi, o, kWave);
    klo = a < klo ? a : klo;
    khi = b > khi ? b : khi;
  }
  const int wid = threadIdx.x / kWave;
  constexpr int W = NT / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    sd[wid] = lo;
    sd[W + wid] = hi;
    sk[wid] = klo;
    sk[W + wid] = khi;
  }
  __syncthreads();
  lo = sd[0];
  hi = sd[W];
  klo = sk[0];
  khi = sk[W];
#pragma unroll
  for (int w = 1; w < W; ++w) {
    lo = fmin(lo, sd[w]);
    hi = fmax(hi, sd[W + w]);
    klo = sk[w] < klo ? sk[w] : klo;
    khi = sk[W + w] > khi ? sk[W + w] : khi;
  }
}

// exclusive prefix of h[0 .. kRkSub) by wave 0 (32 entries per lane), total in h[kRkSub]
__device__ __forceinline__ void sub_prefix(uint32_t* h) {
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    constexpr int per = kRkSub / kWave;
    uint32_t loc[per], sum = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
      loc[k] = h[lane * per + k];
      sum += loc[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += t;
    }
    uint32_t run = inc - sum;
#pragma unroll
    for (int k = 0; k < per; ++k) {
      h[lane * per + k] = run;
      run += loc[k];
    }
    if (lane == kWave - 1) h[kRkSub] = run;
  }
}

// pass 4: one block per interval bucket: the two candidate maps, their histograms, the better
// one's prefix table subp[b][0 .. kRkSub] and the z keys sorted by it into skeys
constexpr int kSubThreads = 1024;  // ~4000 z per bucket: four per thread and pass
template <typename T>
__global__ __launch_bounds__(kSubThreads) void k_rank_subsort(
    RankGeo g, const uint32_t* __restrict__ start, const uint32_t* __restrict__ total,
    const uint64_t* __restrict__ bkeys, uint64_t* __restrict__ skeys,
    uint32_t* __restrict__ subp, SubMap* __restrict__ maps) {
  __shared__ uint32_t hv[kRkSub + 1], hk[kRkSub + 1];
  __shared__ double sd[2 * kSubThreads / kWave];
  __shared__ uint64_t sk[2 * kSubThreads / kWave];
  __shared__ unsigned long long cost[2];
  const int b = 2 * blockIdx.x;  // interval buckets only
  const uint32_t s0 = start[b], c = total[b];
  // a bucket of <= kSubK * kSubThreads keys is read once into registers and every pass reuses
  // them (three dependent global passes were most of this kernel's time at C2 size)
  constexpr int kSubK = 4;
  const bool inreg = c <= (uint32_t)(kSubK * kSubThreads);  // block-uniform
  uint64_t kr[kSubK];
  if (inreg) {
#pragma unroll
    for (int u = 0; u < kSubK; ++u) {
      const uint32_t i = threadIdx.x + u * kSubThreads;
      kr[u] = i < c ? bkeys[s0 + i] : 0ull;
    }
  }
  auto each = [&](auto&& fn) {
    if (inreg) {
#pragma unroll
      for (int u = 0; u < kSubK; ++u)
        if (threadIdx.x + u * kSubThreads < c) fn(kr[u]);
    } else {
      for (uint32_t i = threadIdx.x; i < c; i += kSubThreads) fn(bkeys[s0 + i]);
    }
  };
  double lo = __builtin_inf(), hi = -__builtin_inf();
  uint64_t klo = ~0ull, khi = 0;
  each([&](uint64_t k) {
    const double v = key_value<T>(k);
    if (v - v == 0.0) {  // finite
      lo = fmin(lo, v);
      hi = fmax(hi, v);
    }
    if (k != ~0ull) {  // not NaN
      klo = k < klo ? k : klo;
      khi = k > khi ? k : khi;
    }
  });
  for (int i = threadIdx.x; i <= kRkSub; i += kSubThreads) hv[i] = hk[i] = 0;
  if (threadIdx.x < 2) cost[threadIdx.x] = 0;
  block_minmax<kSubThreads>(lo, hi, klo, khi, sd, sk);
  SubMap fv{0.0, 0.0, 0, 0, 0}, fk{0.0, 0.0, 0, 0, 1};
  if (hi > lo) {
    const double scale = (double)kRkSub / (hi - lo);
    if (scale - scale == 0.0) fv.lo = lo, fv.scale = scale;  // a finite span
  }
  if (khi > klo) {
    const uint64_t r = khi - klo;
    const int bits = 64 - __builtin_clzll(r);  // r < 2^bits
    fk.klo = klo;
    fk.kshift = bits > 11 ? bits - 11 : 0;
  }
  each([&](uint64_t k) {
    const double v = key_value<T>(k);
    atomicAdd(&hv[fv(v, k)], 1u);
    atomicAdd(&hk[fk(v, k)], 1u);
  });
  __syncthreads();
  unsigned long long cv = 0, ck = 0;
  for (int i = threadIdx.x; i < kRkSub; i += kSubThreads) {
    cv += (unsigned long long)hv[i] * hv[i];
    ck += (unsigned long long)hk[i] * hk[i];
  }
  // wave sums first: 1024 LDS atomics on one address serialise (most of this kernel's 18 us)
  cv = wave_sum_u64(cv);
  ck = wave_sum_u64(ck);
  if ((threadIdx.x & (kWave - 1)) == 0) {
    atomicAdd(&cost[0], cv);
    atomicAdd(&cost[1], ck);
  }
  __syncthreads();
  const bool bykey = cost[1] < cost[0];
  const SubMap f = bykey ? fk : fv;
  uint32_t* h = bykey ? hk : hv;
  if (threadIdx.x == 0) maps[blockIdx.x] = f;
  sub_prefix(h);
  __syncthreads();
  uint32_t* sp_out = subp + (int64_t)blockIdx.x * (kRkSub + 1);
  for (int i = threadIdx.x; i <= kRkSub; i += kSubThreads) sp_out[i] = h[i];
  __syncthreads();
  each([&](uint64_t k) { skeys[s0 + atomicAdd(&h[f(key_value<T>(k), k)], 1u)] = k; });
  // long sub-buckets sorted in place: h[i] is now the END of sub-bucket i
  __shared__ uint16_t longs[kRkSub];
  __shared__ int nlong;
  if (threadIdx.x == 0) nlong = 0;
  __syncthreads();  // also: the scatter's skeys stores are visible to the whole block
  for (int i = threadIdx.x; i < kRkSub; i += kSubThreads) {
    const uint32_t L = h[i] - (i ? h[i - 1] : 0u);
    if (L > kRkSortedMin && L <= kRkSortedMax) longs[atomicAdd(&nlong, 1)] = (uint16_t)i;
  }
  __syncthreads();
  const int nl = nlong;
  if (nl == 0) return;
  // up to kRkWaveSortMax keys: one wave per sub-bucket, the block's waves on different ones at
  // once (ties: ~200 copies of each value made every interval bucket ~20 sequential 4096-key
  // block sorts, 1.9 ms for 1e6 + 1e6 keys of 5000 values; profiles/r04s12_rank_plan_ties.log)
  {
    const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    auto wave_sort = [&](auto e_const, uint64_t* q, uint32_t L) {
      constexpr int E = decltype(e_const)::value;
      uint64_t v[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint32_t t = (uint32_t)(lane * E + e);
        v[e] = t < L ? q[t] : ~0ull;
      }
      wave_sort_keys<E>(v, lane);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const uint32_t t = (uint32_t)(lane * E + e);
        if (t < L) q[t] = v[e];
      }
    };
    for (int li = wid; li < nl; li += kSubThreads / kWave) {
      const int i = __builtin_amdgcn_readfirstlane(longs[li]);
      const uint32_t a = i ? h[i - 1] : 0u, L = h[i] - a;
      uint64_t* q = skeys + s0 + a;
      if (L <= 4 * kWave)
        wave_sort(std::integral_constant<int, 4>(), q, L);
      else if (L <= kRkWaveSortMax)
        wave_sort(std::integral_constant<int, kRkWaveSortMax / kWave>(), q, L);
    }
  }
  __shared__ uint64_t sbuf[kRkSortedMax];
  for (int li = 0; li < nl; ++li) {
    const int i = longs[li];
    const uint32_t a = i ? h[i - 1] : 0u, L = h[i] - a;
    if (L <= kRkWaveSortMax) continue;  // sorted by a wave above
    for (uint32_t t = threadIdx.x; t < kRkSortedMax; t += kSubThreads)
      sbuf[t] = t < L ? skeys[s0 + a + t] : ~0ull;
    __syncthreads();
    sort_keys_block<kRkSortedMax / kSubThreads>(sbuf, (int)kRkSortedMax, skeys + s0 + a, (int)L);
    __syncthreads();
  }
}

// pass 5: every element in input order, one per thread (the chain splitters -> bucket map ->
// sub-bucket prefix -> keys is three dependent loads; many waves hide them): its image and its
// record (coalesced stores)
template <typename T>
__global__ __launch_bounds__(kRkThreads) void k_rank_records(
    const T* __restrict__ x, const T* __restrict__ z, RankGeo g, const uint64_t* __restrict__ ss,
    const uint32_t* __restrict__ start, const uint32_t* __restrict__ total,
    const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ subp,
    const SubMap* __restrict__ maps, uint64_t* __restrict__ x_rec,
    uint64_t* __restrict__ z_rec) {
  __shared__ uint64_t sp[kRkMaxB];
  const int64_t e = (int64_t)blockIdx.x * kRkThreads + threadIdx.x;
  const bool isx = e < g.n;
  T v = 0;
  if (e < g.tot) v = isx ? x[e] : z[e - g.n];  // issued before the barrier
  const uint64_t key = order_key<T>(v);
  const int nsp = load_splitters(ss, g, sp);
  if (e >= g.tot) return;
  const int b = rank_bucket(sp, nsp, key);
  uint32_t gv = start[b];  // every z of the lower buckets is below key
  const uint32_t tb = total[b];
  uint32_t hv = gv + tb;   // h(v) for an equality bucket: every z of it equals v
  // issued with start / total (in bounds for every bucket; used for interval buckets only), so
  // the chain is splitters -> {start, total, map} -> sub-bucket prefix -> keys
  const SubMap f = maps[b >> 1];
  if ((b & 1) == 0) {  // interval bucket: sub-buckets below + a scan (equal keys share one)
    hv = gv;
    if (tb != 0) {
      const uint32_t sb = f((double)v, key);
      const uint32_t* pt = subp + (int64_t)(b >> 1) * (kRkSub + 1);
      const uint32_t lo = pt[sb], hi = pt[sb + 1];
      const uint64_t* q = skeys + gv;
      uint32_t below = lo, eq = 0;
      if (hi - lo > kRkSortedMin && hi - lo <= kRkSortedMax) {  // sorted by the sub-sort
        uint32_t a = lo, n = hi - lo;  // lower_bound(key)
        while (n > 0) {
          const uint32_t h2 = n >> 1;
          if (q[a + h2] < key) {
            a += h2 + 1;
            n -= h2 + 1;
          } else {
            n = h2;
          }
        }
        uint32_t b2 = a, m2 = hi - a;  // upper_bound(key)
        while (m2 > 0) {
          const uint32_t h2 = m2 >> 1;
          if (q[b2 + h2] <= key) {
            b2 += h2 + 1;
            m2 -= h2 + 1;
          } else {
            m2 = h2;
          }
        }
        below = a;
        eq = b2 - a;
      } else {
        for (uint32_t i = lo; i < hi; ++i) {
          const uint64_t k = q[i];
          below += k < key ? 1u : 0u;
          eq += k == key ? 1u : 0u;
        }
      }
      gv += below;
      hv = gv + eq;
    }
  }
  if (isx) {
    const bool nan = std::is_floating_point<T>::value && key == ~0ull;
    const float img = nan ? kImgNever : (float)gv;
    const uint64_t hi = g.half ? (uint64_t)__float_as_uint(nan ? kImgNever : (float)hv)
                               : (uint64_t)e;
    if (g.compact && !g.half)
      ((uint32_t*)x_rec)[e] = __float_as_uint(img);  // the image alone, 4 B
    else
      x_rec[e] = (uint64_t)__float_as_uint(img) | (hi << 32);
  } else {
    const int64_t j = e - g.n;
    if (g.compact)
      ((uint32_t*)z_rec)[j] = __float_as_uint(-(float)gv);
    else
      z_rec[j] = (uint64_t)__float_as_uint(-(float)gv) | ((uint64_t)j << 32);
  }
}

struct RankWork {
  void* samp;
  uint64_t *ss, *bkeys, *skeys;
  uint32_t *rel, *total, *start, *subp;
  uint16_t* bid;  // each z's bucket (the histogram pass -> the scatter pass)
  SubMap* maps;
  size_t total_bytes;
};

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

static RankGeo rank_geo(int64_t n, int64_t m, int64_t mq = -1, int half = 0, int compact = 0) {
  RankGeo g{};
  g.n = n;
  g.m = m;
  g.mq = mq < 0 ? m : mq;
  g.tot = n + g.mq;
  g.half = half;
  g.compact = compact;
  const bool small = m <= kRkSmallM;
  const int64_t zint = small ? g_rank_zint_small : 2048;  // >= ~zint z per interval
  g.cs = (int)std::min<int64_t>(m, small ? g_rank_cs_small : g_rank_cs);
  int B = 1;
  while (B < kRkMaxB && 2 * B <= std::max(g.cs, 1) && (int64_t)B * zint < m) B <<= 1;
  g.B = B;
  g.NB = 2 * B;
  g.per = small ? g_rank_per_small : g_rank_per;
  g.nblk = (int)std::max<int64_t>(1, ceil_div(m, (int64_t)kRkThreads * g.per));
  g.C = 256;
  while (g.C < g.cs) g.C <<= 1;
  return g;
}

static RankWork rank_work(const RankGeo& g, char* base) {
  RankWork w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align256(bytes);
    return base ? (void*)(base + o) : nullptr;
  };
  w.samp = take(8 * (size_t)kRkSample);
  w.ss = (uint64_t*)take(8 * (size_t)kRkSample);
  w.rel = (uint32_t*)take(4 * (size_t)g.NB * g.nblk);
  w.total = (uint32_t*)take(4 * (size_t)g.NB);
  w.start = (uint32_t*)take(4 * (size_t)g.NB);
  w.subp = (uint32_t*)take(4 * (size_t)g.B * (kRkSub + 1));
  w.maps = (SubMap*)take(sizeof(SubMap) * (size_t)g.B);
  w.bkeys = (uint64_t*)take(8 * (size_t)std::max<int64_t>(g.m, 1));
  w.skeys = (uint64_t*)take(8 * (size_t)std::max<int64_t>(g.m, 1));
  w.bid = (uint16_t*)take(2 * (size_t)std::max<int64_t>(g.m, 1));
  w.total_bytes = off;
  return w;
}

static bool rank_sizes_ok(int64_t n, int64_t m) {
  // images are exact integers while m < 2^24; ids fit 32 bits
  return n >= 0 && m >= 0 && m < (1ll << 24) && n + m < (1ll << 31);
}

// ----------------------------------------------------------------------------- the count
// (gt_clamp / acc_add: pkcount.h; a z record's LOW word is its negated image)
__device__ __forceinline__ float rec_image(uint64_t r) { return __uint_as_float((uint32_t)r); }

// One wave item: 64*R x-images (R per lane as R/2 packed pairs) against z records [z0, z1).
template <int R>
__device__ __forceinline__ unsigned long long count_rank_item(const uint64_t* __restrict__ xr,
                                                              int64_t x0, int64_t xe,
                                                              const uint64_t* __restrict__ zr,
                                                              int64_t z0, int64_t z1, int lane) {
  constexpr int P = R / 2;
  f2 xv[P], acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t i0 = x0 + (2 * p) * kWave + lane, i1 = i0 + kWave;
    xv[p].x = i0 < xe ? rec_image(xr[i0]) : kImgNever;  // padded lanes: never greater
    xv[p].y = i1 < xe ? rec_image(xr[i1]) : kImgNever;
    acc[p] = f2{0.f, 0.f};
  }
  // all compares of one z first, then the accumulations: no adjacent dependent pair
  auto one_z = [&](uint64_t zu) {
    f2 t[P];
#pragma unroll
    for (int p = 0; p < P; ++p) t[p] = gt_clamp(xv[p], zu);
#pragma unroll
    for (int p = 0; p < P; ++p) acc_add(acc[p], t[p]);
  };
  const uint64_t* __restrict__ zp = zr + z0;
  const int nz = (int)(z1 - z0);
  int j = 0;
  // 8 records per s_load_dwordx16; the next group's loads are in flight while one is compared
  // (two register buffers, loads past the chunk clamped to its last full group)
  if (nz >= 16) {
    uint64_t za[8], zb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) za[u] = zp[u];
    const int last = nz - 8;
    for (; j + 16 <= nz; j += 16) {
      const uint64_t* qb = zp + j + 8;
#pragma unroll
      for (int u = 0; u < 8; ++u) zb[u] = qb[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) one_z(za[u]);
      const uint64_t* qa = zp + (j + 16 <= last ? j + 16 : last);
#pragma unroll
      for (int u = 0; u < 8; ++u) za[u] = qa[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) one_z(zb[u]);
    }
  }
  for (; j + 8 <= nz; j += 8) {
    uint64_t zv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) zv[u] = zp[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) one_z(zv[u]);
  }
  for (; j < nz; ++j) one_z(zp[j]);
  unsigned long long tot = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) tot += (unsigned)acc[p].x + (unsigned)acc[p].y;  // exact < 2^24
  return wave_sum_u64(tot);
}

// Same work decomposition and epilogue as k_count_complete (csrc/count.hip): per-wave items
// (shard, x tile, z chunk), XCD-aware block order, one u64 atomic per block and shard; the
// last nxt.blocks blocks carry the next repartition (nextstep.h) on the records.
template <int R>
__global__ __launch_bounds__(kBlock) void k_count_rank(
    const uint64_t* __restrict__ xr, const int64_t* __restrict__ x_off,
    const uint64_t* __restrict__ zr, const int64_t* __restrict__ z_off, int n_shards,
    int tiles_x, int zchunks, int64_t z_chunk, unsigned long long* __restrict__ out,
    NextStep nxt) {
  // spare blocks: the last nxt.blocks of the grid (tail = 1) or the first (tail = 0: dispatched
  // beside the count blocks from the start, for count grids of a few waves per SIMD)
  const int nb = nxt.blocks;
  const int sb = nxt.tail ? (int)blockIdx.x - ((int)gridDim.x - nb) : (int)blockIdx.x;
  if (nb && sb >= 0 && sb < nb) {
    next_step_part<kBlock>(nxt, sb);
    return;
  }
  const int per_shard = tiles_x * zchunks;
  // whole shards per XCD (nb is a multiple of kXcds, so front spares keep the XCD order)
  const int lb = xcd_block(nxt.tail ? blockIdx.x : blockIdx.x - nb, gridDim.x - nb);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int item = lb * (kBlock / kWave) + wid;
  const int s = item / per_shard;
  bool active = s < n_shards;
  int64_t x0 = 0, xe = 0, z0 = 0, z1 = 0;
  if (active) {
    const int rem = item - s * per_shard;
    const int cz = rem / tiles_x;
    const int tx = rem - cz * tiles_x;
    const int64_t xb = x_off[s], zb = z_off[s], ze = z_off[s + 1];
    xe = x_off[s + 1];
    x0 = xb + (int64_t)tx * (kWave * R);
    z0 = zb + (int64_t)cz * z_chunk;
    z1 = (z0 + z_chunk < ze) ? z0 + z_chunk : ze;
    active = x0 < xe && z0 < ze;
  }
  unsigned long long tot = 0;
  if (active) tot = count_rank_item<R>(xr, x0, xe, zr, z0, z1, lane);
  __shared__ unsigned long long part[kBlock / kWave];
  __shared__ int part_s[kBlock / kWave];
  if (lane == 0) {
    part[wid] = tot;
    part_s[wid] = active ? s : -1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int cur = part_s[0];
    unsigned long long sum = part[0];
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) {
      if (part_s[w] != cur) {
        if (cur >= 0 && sum) atomicAdd(out + cur, sum);
        cur = part_s[w];
        sum = 0;
      }
      sum += part[w];
    }
    if (cur >= 0 && sum) atomicAdd(out + cur, sum);
  }
}

// Final order of the doubles: out[p] = in[rec[p] >> 32]
__global__ __launch_bounds__(kBlock) void k_gather_records(const uint64_t* __restrict__ in,
                                                           const uint64_t* __restrict__ rec,
                                                           int64_t n, uint64_t* __restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * kBlock)
    out[p] = in[rec[p] >> 32];
}

// ----------------------------------------------------------------------------- plan
struct RankPlan {
  int R, tiles_x, zchunks;
  int64_t z_chunk, blocks;
};
static int g_rank_R = 0;          // tuning hooks (tw_count_rank_set_plan); 0 = automatic
static int g_rank_next_front = 0;  // tw_count_rank_set_next: spare blocks first (1) or last (0)
static int64_t g_rank_zchunk = 0;

// R in {16, 8}: least padded x-slots (ties to 16: half the z loads per compare); z chunks of
// ~1024 records (tools/mb_pk.hip: 528 is too short for R = 8, >= 2048 leaves the tail ragged).
static RankPlan plan_rank(int64_t max_nx, int64_t max_nz, int32_t n_shards, bool fused) {
  RankPlan p{16, 1, 1, max_nz, 0};
  int64_t best = -1;
  for (int R : {16, 8}) {
    if (g_rank_R && R != g_rank_R) continue;
    const int64_t slots = ceil_div(max_nx, (int64_t)kWave * R) * kWave * R;
    if (best < 0 || slots < best) {
      best = slots;
      p.R = R;
    }
  }
  p.tiles_x = (int)ceil_div(max_nx, (int64_t)kWave * p.R);
  int64_t zc = g_rank_zchunk > 0 ? g_rank_zchunk : 1024;
  // enough work items to fill the chip when shards are few / short: 16 per SIMD; but a count
  // with a fused next repartition and under 4 items per SIMD at 1024-long chunks (8 shards of
  // 15625 + 15625, the strong-scaling shape at G = 8) aims at 4, so the whole count grid is
  // resident at once and the spare blocks behind it start at once (tools/replicated_probe.py:
  // 80.4 -> 72.5 us per step there)
  const int64_t base = (int64_t)p.tiles_x * n_shards;
  const int64_t few = 256 * 4 * (kBlock / kWave);
  const int64_t target =
      fused && base * ceil_div(max_nz, (int64_t)1024) < few ? few : 256 * 16 * (kBlock / kWave);
  if (g_rank_zchunk <= 0 && base * ceil_div(max_nz, zc) < target)
    zc = std::max<int64_t>(256, ceil_div(max_nz, std::max<int64_t>(1, target / base)));
  zc = std::min<int64_t>(zc, (int64_t)1 << 24);  // f32 lane counters stay exact
  p.z_chunk = ceil_div(std::min<int64_t>(zc, max_nz), 8) * 8;
  p.zchunks = (int)ceil_div(max_nz, p.z_chunk);
  p.blocks = ceil_div((int64_t)p.tiles_x * p.zchunks * n_shards, kBlock / kWave);
  return p;
}

static int next_rank_blocks(int64_t elems) {
  int64_t b = ceil_div(elems, (int64_t)kBlock * 8);
  b = std::min<int64_t>(std::max<int64_t>(b, 8), 512);
  return (int)(ceil_div(b, kXcds) * kXcds);
}

}  // namespace tw

using namespace tw;

extern "C" int64_t tw_rank_images_work_bytes(int64_t n_x, int64_t n_z) {
  if (!rank_sizes_ok(n_x, n_z)) return -1;
  return (int64_t)rank_work(rank_geo(n_x, n_z), nullptr).total_bytes;
}

namespace tw {
// z / m: the structure's Z; xq / zq: the elements imaged (g.n and g.mq of them)
template <typename T>
static int rank_images_t(const T* xq, const T* zq, const T* z, int64_t m, const RankWork& w,
                         const RankGeo& g, uint64_t* x_rec, uint64_t* z_rec, hipStream_t st) {
  if (m > 0) {  // the sample: hashed positions of z, sorted (k_sort_chunks pads with ~0 past cs)
    if (g.C <= 512)
      hipLaunchKernelGGL((k_rank_sample_sort<T>), dim3(1), dim3(1024), 0, st, z, m, g.cs, g.C,
                         w.ss);
    else
      hipLaunchKernelGGL((k_rank_sample_count<T>), dim3(g.C / kRkSampPlace), dim3(1024), 0, st,
                         z, m, g.cs, g.C, w.ss);
    TW_LAUNCH_CHECK();
    auto passes = [&](auto per) {
      constexpr int PER = decltype(per)::value;
      hipLaunchKernelGGL((k_rank_hist<T, PER>), dim3(g.nblk), dim3(kRkThreads), 0, st, z, g,
                         w.ss, w.rel, w.bid);
      if (g.nblk <= 2 * kWave)  // small Z: rows (and starts) in one block
        hipLaunchKernelGGL(k_rank_rows_starts, dim3(1), dim3(1024), 0, st, g, w.rel, w.total,
                           w.start);
      else
        hipLaunchKernelGGL(k_rank_rows, dim3((unsigned)ceil_div(g.NB, kWave)),
                           dim3(kRowsWaves * kWave), 0, st, g, w.rel, w.total);
      // the starts: made (again, for the small path) by the scatter blocks
      hipLaunchKernelGGL((k_rank_scatter<T, PER>), dim3(g.nblk), dim3(kRkThreads), 0, st, z, g,
                         w.bid, w.rel, w.total, w.start, w.bkeys);
    };
    if (g.per == 4)
      passes(std::integral_constant<int, 4>());
    else if (g.per == 8)
      passes(std::integral_constant<int, 8>());
    else
      passes(std::integral_constant<int, 16>());
    hipLaunchKernelGGL((k_rank_subsort<T>), dim3(g.B), dim3(kSubThreads), 0, st, g, w.start,
                       w.total, w.bkeys, w.skeys, w.subp, w.maps);
    TW_LAUNCH_CHECK();
  } else {  // no z: every image is 0
    TW_HIP_CHECK(tw_zero_async(w.start, 0, 4 * (size_t)g.NB, st));
    TW_HIP_CHECK(tw_zero_async(w.total, 0, 4 * (size_t)g.NB, st));
    TW_HIP_CHECK(tw_zero_async(w.ss, 0, 8 * (size_t)kRkSample, st));
  }
  // (one element per thread: 128 .. 1024 threads per block and four elements per thread
  // measured the same or slower, profiles/r03s53_time_ranking.log)
  if (g.tot == 0) return TW_OK;
  hipLaunchKernelGGL((k_rank_records<T>), dim3((unsigned)ceil_div(g.tot, kRkThreads)),
                     dim3(kRkThreads), 0, st, xq, zq, g, w.ss, w.start, w.total, w.skeys, w.subp,
                     w.maps, x_rec, z_rec);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

static int rank_images_any(const void* d_zs, int64_t m, const void* d_xq, int64_t nq_x,
                           const void* d_zq, int64_t nq_z, int32_t dtype, int32_t half,
                           void* d_work, int64_t work_bytes, uint64_t* d_x_rec,
                           uint64_t* d_z_rec, hipStream_t st) {
  const RankGeo g = rank_geo(nq_x, m, nq_z, half & 1, (half >> 1) & 1);
  const RankWork w = rank_work(g, (char*)d_work);
  TW_ARG_CHECK(d_work != nullptr && work_bytes >= (int64_t)w.total_bytes,
               "tw_rank_images: work buffer of %lld bytes, %lld needed", (long long)work_bytes,
               (long long)w.total_bytes);
  if (dtype == TW_F64)
    return rank_images_t<double>((const double*)d_xq, (const double*)d_zq, (const double*)d_zs,
                                 m, w, g, d_x_rec, d_z_rec, st);
  return rank_images_t<long long>((const long long*)d_xq, (const long long*)d_zq,
                                  (const long long*)d_zs, m, w, g, d_x_rec, d_z_rec, st);
}
}  // namespace tw

extern "C" int tw_rank_images(const void* d_x, int64_t n_x, const void* d_z, int64_t n_z,
                              int32_t dtype, void* d_work, int64_t work_bytes, uint64_t* d_x_rec,
                              uint64_t* d_z_rec, void* stream) {
  TW_ARG_CHECK(rank_sizes_ok(n_x, n_z),
               "tw_rank_images: needs n_z < 2^24 and n_x + n_z < 2^31 (got %lld, %lld)",
               (long long)n_x, (long long)n_z);
  TW_ARG_CHECK(dtype == TW_F64 || dtype == TW_I64, "tw_rank_images: unknown dtype %d", dtype);
  if (n_x + n_z == 0) return TW_OK;
  return rank_images_any(d_z, n_z, d_x, n_x, d_z, n_z, dtype, 0, d_work, work_bytes, d_x_rec,
                         d_z_rec, (hipStream_t)stream);
}

extern "C" int tw_rank_images_query(const void* d_z_all, int64_t n_z_all, const void* d_x,
                                    int64_t n_x, const void* d_z, int64_t n_z, int32_t dtype,
                                    int32_t half, void* d_work, int64_t work_bytes,
                                    uint64_t* d_x_rec, uint64_t* d_z_rec, void* stream) {
  TW_ARG_CHECK(rank_sizes_ok(n_x, n_z_all) && n_z >= 0 && n_x + n_z < (1ll << 31),
               "tw_rank_images_query: needs n_z_all < 2^24 and n_x + n_z < 2^31 (got %lld, "
               "%lld, %lld)", (long long)n_z_all, (long long)n_x, (long long)n_z);
  TW_ARG_CHECK(dtype == TW_F64 || dtype == TW_I64, "tw_rank_images_query: unknown dtype %d",
               dtype);
  TW_ARG_CHECK(half >= 0 && half <= 3, "tw_rank_images_query: flags in [0, 3]");
  if (n_x + n_z == 0) return TW_OK;
  return rank_images_any(d_z_all, n_z_all, d_x, n_x, d_z, n_z, dtype, half, d_work, work_bytes,
                         d_x_rec, d_z_rec, (hipStream_t)stream);
}

extern "C" int tw_rank_set_plan(int32_t sample, int32_t per) {
  TW_ARG_CHECK(sample == 512 || sample == 1024 || sample == 2048,
               "tw_rank_set_plan: sample of 512, 1024 or 2048 keys");
  TW_ARG_CHECK(per == 4 || per == 8 || per == 16, "tw_rank_set_plan: 4, 8 or 16 z per thread");
  g_rank_cs = sample;
  g_rank_per = per;
  return TW_OK;
}

extern "C" int tw_rank_set_small(int32_t sample, int32_t z_per_interval, int32_t per) {
  TW_ARG_CHECK(sample == 256 || sample == 512 || sample == 1024 || sample == 2048,
               "tw_rank_set_small: sample of 256, 512, 1024 or 2048 keys");
  TW_ARG_CHECK(z_per_interval == 512 || z_per_interval == 1024 || z_per_interval == 2048,
               "tw_rank_set_small: 512, 1024 or 2048 z per interval bucket");
  TW_ARG_CHECK(per == 4 || per == 8 || per == 16, "tw_rank_set_small: 4, 8 or 16 z per thread");
  g_rank_cs_small = sample;
  g_rank_zint_small = z_per_interval;
  g_rank_per_small = per;
  return TW_OK;
}

extern "C" int tw_count_rank_set_next(int32_t front) {
  TW_ARG_CHECK(front == 0 || front == 1, "tw_count_rank_set_next: front in {0, 1}");
  g_rank_next_front = front;
  return TW_OK;
}

extern "C" int tw_count_rank_set_plan(int32_t R, int64_t z_chunk) {
  TW_ARG_CHECK(R == 0 || R == 8 || R == 16, "tw_count_rank_set_plan: R in {0, 8, 16}");
  TW_ARG_CHECK(z_chunk >= 0 && z_chunk <= (1ll << 24), "tw_count_rank_set_plan: bad z_chunk");
  g_rank_R = R;
  g_rank_zchunk = z_chunk;
  return TW_OK;
}

extern "C" int tw_count_pairs_rank_step(const uint64_t* d_x_rec, const int64_t* d_x_off,
                                        const uint64_t* d_z_rec, const int64_t* d_z_off,
                                        int32_t n_shards, int64_t max_nx, int64_t max_nz,
                                        uint64_t* d_out, int64_t n_x, uint64_t* d_x_next,
                                        uint64_t key_x, int64_t n_z, uint64_t* d_z_next,
                                        uint64_t key_z, uint64_t* d_out_next,
                                        int32_t n_next_shards, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && n_x >= 0 && n_z >= 0 &&
                   n_x < (1ll << 60) && n_z < (1ll << 60) && n_next_shards >= 0,
               "tw_count_pairs_rank_step: bad sizes");
  TW_ARG_CHECK(max_nz < (1ll << 24), "tw_count_pairs_rank_step: shards of < 2^24 z-values");
  TW_ARG_CHECK(d_x_next == nullptr || ((n_x == 0 || d_x_next != d_x_rec) &&
                                       (n_z == 0 || (d_z_next != nullptr && d_z_next != d_z_rec))),
               "tw_count_pairs_rank_step: next arrays must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  NextStep nxt{};
  if (d_x_next != nullptr) {
    nxt = NextStep{d_x_rec, d_x_next, n_x, d_z_rec, d_z_next, n_z,
                   (unsigned long long*)d_out_next, d_out_next ? (int64_t)n_next_shards : 0,
                   make_feistel(std::max<int64_t>(n_x, 1), key_x),
                   make_feistel(std::max<int64_t>(n_z, 1), key_z), next_rank_blocks(n_x + n_z),
                   0, g_rank_next_front ? 0 : 1};
  } else if (d_out_next != nullptr && n_next_shards > 0) {
    TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
  }
  const bool counts = n_shards > 0 && max_nx > 0 && max_nz > 0;
  if (!counts) {
    if (nxt.blocks == 0) return TW_OK;
    hipLaunchKernelGGL((k_count_rank<16>), dim3(nxt.blocks), dim3(kBlock), 0, st, nullptr,
                       nullptr, nullptr, nullptr, 0, 1, 1, (int64_t)1, nullptr, nxt);
    TW_LAUNCH_CHECK();
    return TW_OK;
  }
  const RankPlan p = plan_rank(max_nx, max_nz, n_shards, nxt.blocks > 0);
  TW_ARG_CHECK((p.blocks + nxt.blocks) * (kBlock / kWave) < (1ll << 31),
               "tw_count_pairs_rank_step: grid too large");
  dim3 g((unsigned)(p.blocks + nxt.blocks)), b(kBlock);
  auto* o = (unsigned long long*)d_out;
  if (p.R == 16)
    hipLaunchKernelGGL((k_count_rank<16>), g, b, 0, st, d_x_rec, d_x_off, d_z_rec, d_z_off,
                       n_shards, p.tiles_x, p.zchunks, p.z_chunk, o, nxt);
  else
    hipLaunchKernelGGL((k_count_rank<8>), g, b, 0, st, d_x_rec, d_x_off, d_z_rec, d_z_off,
                       n_shards, p.tiles_x, p.zchunks, p.z_chunk, o, nxt);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_gather_records(const void* d_in, const uint64_t* d_rec, int64_t n, void* d_out,
                                 void* stream) {
  TW_ARG_CHECK(n >= 0, "tw_gather_records: n < 0");
  TW_ARG_CHECK(n == 0 || d_in != d_out, "tw_gather_records: in and out must differ");
  if (n == 0) return TW_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_gather_records, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_in, d_rec, n, (uint64_t*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
