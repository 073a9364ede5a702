// rankcount.hip — exact pair counts by sorting + binary search.
//
// Same integers as k_count_complete (the reference's #{x > z}, estimation-experiment/
// main.py:31; half-units for ties), in O((n+m) log m) per shard instead of O(n m):
//   #{j : z_j < x} summed over x.
// Scores become order-preserving u64 keys, which makes NumPy's comparison semantics exact:
//   float64: -0.0 -> +0.0 (they compare equal), NaN -> 0xFFFF..FF (never below anything);
//            key = sign ? ~bits : bits | 2^63
//   int64:   key = v ^ 2^63
// x-values that are NaN contribute nothing (x > z is false for every z).
//
// Kernel 1 (k_sort_chunks): one 1024-thread block per (shard, z-chunk of C <= 16384 keys):
//   load + key transform into LDS (C*8 <= 128 KiB), pad with the max key, bitonic sort in
//   LDS, write the sorted chunk to the workspace.
// Kernel 2 (k_rank_count): one 1024-thread block per (shard, x-tile): for every sorted chunk
//   of its shard, stage the chunk in LDS and let each thread binary-search its x keys
//   (log2(C) + 1 dependent ds_read_b64 per x, branchless); u32 -> u64 -> block sum -> one
//   atomic per block.  Padding keys (max) are never < a non-NaN x key.
#include "sortkeys.h"
#include "imagecount.h"
#include "records.h"
#include <algorithm>
#include <type_traits>

// Phase timestamps for kernel studies (tools/phase_codes.py builds a separate library with
// -DTW_PHASE_TIMING; the product build compiles them out).
#ifdef TW_PHASE_TIMING
__device__ unsigned long long g_tw_phase[1 << 16];
#define TW_PHASE(k)                                                                    \
  do {                                                                                 \
    if (threadIdx.x == 0) g_tw_phase[((size_t)blockIdx.x * 8 + (k)) & 0xFFFF] = clock64(); \
  } while (0)
extern "C" int tw_debug_phases(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tw_phase), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : 2;
}
#else
#define TW_PHASE(k) \
  do {              \
  } while (0)
#endif

namespace tw {

constexpr int kXPerThread = 4;

template <typename T, int PRED>
__global__ __launch_bounds__(kSortThreads) void k_rank_count(const T* __restrict__ x,
                                                             const int64_t* __restrict__ x_off,
                                                             const uint64_t* __restrict__ sorted,
                                                             int chunks, int C, int tiles_x,
                                                             unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's x-tiles share one L2
  const int s = lb / tiles_x;
  const int t = lb - s * tiles_x;
  const int64_t xb = x_off[s], xe = x_off[s + 1];
  const int64_t x0 = xb + (int64_t)t * (kSortThreads * kXPerThread);
  if (x0 >= xe) return;
  uint64_t xk[kXPerThread];
  bool valid[kXPerThread];
#pragma unroll
  for (int r = 0; r < kXPerThread; ++r) {
    const int64_t i = x0 + r * kSortThreads + threadIdx.x;
    valid[r] = i < xe;
    const T v = valid[r] ? x[i] : (T)0;
    valid[r] = valid[r] && !is_nan_score<T>(v);
    xk[r] = order_key<T>(v);
  }
  unsigned long long acc = 0;
  // stage as many sorted chunks as fit (<= 16384 keys = 128 KiB) at once, then run every
  // search of this thread back to back (independent LDS chains in flight)
  const int group = (int)std::max<int64_t>(1, kMaxChunk / C);
  for (int c0 = 0; c0 < chunks; c0 += group) {
    const int ng = std::min(group, chunks - c0);
    const uint64_t* src = sorted + ((int64_t)s * chunks + c0) * C;
    __syncthreads();
    for (int i = threadIdx.x; i < ng * C; i += kSortThreads) keys[i] = src[i];
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
      const uint64_t* kc = keys + g * C;
#pragma unroll
      for (int r = 0; r < kXPerThread; ++r) {
        if (valid[r]) {
          uint32_t v = lower_bound_lds(kc, C, xk[r]);
          if (PRED == TW_PRED_HALF) v += upper_bound_lds(kc, C, xk[r]);
          acc += v;
        }
      }
    }
  }
  acc = wave_sum_u64(acc);
  __shared__ unsigned long long part[kSortThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < kSortThreads / kWave; ++w) b += part[w];
    if (b) atomicAdd(out + s, b);
  }
}

struct RankPlan {
  int C, chunks, tiles_x;
};
static int64_t g_chunk_cap = 4096;  // tuning hook (tw_count_sorted_set_chunk)

inline RankPlan plan_rank(int64_t max_nx, int64_t max_nz) {
  RankPlan p;
  int64_t C = 1024;  // register-blocked sort needs C / 16 >= 64 threads
  while (C < max_nz && C < g_chunk_cap) C <<= 1;
  p.C = (int)C;
  p.chunks = (int)std::max<int64_t>(1, ceil_div(max_nz, C));
  p.tiles_x = (int)std::max<int64_t>(1, ceil_div(max_nx, (int64_t)kSortThreads * kXPerThread));
  return p;
}

// Rank codes without a sort (shards with nz <= kBucketMaxZ): the block loads the shard's z
// into LDS in bucket order (a counting sort by bucket), and then a code is
// (#z in lower buckets) + (#z in its own bucket below / at most v), by a scan of one bucket.
// Bucket maps, both monotone (every IEEE step in them is monotone), so bucket order is value
// order:
//   refine = 0  value range: f = clamp(floor((v - zmin) * NB / (zmax - zmin))) over the finite z;
//   refine = 1  equal depth: a histogram of a 1024-value sample of z over kBucketNC value-range
//               bins, whose piecewise-linear CDF maps v to (cs[b] + t * (cs[b+1] - cs[b])) * NB / n
//               (t = the position of v inside bin b): every bucket then holds ~nz / NB values
//               whatever the shape of the data (Gaussian scores put ~25 values in the central
//               value-range buckets of a 15625-value shard; the scans are the main cost).
// The counting sort takes ONE pass of LDS atomics: the atomicAdd that counts z in its bucket
// returns z's slot inside the bucket, so after the prefix z is stored without a second atomic.
// Exact for any data and any map: ties share a bucket; NaN z sit in no bucket (their p is the
// count of non-NaN z, above every x code), NaN x get code 0, +-inf clamp to the end buckets; a
// poor map (skewed data, an unrepresentative sample) only makes scans longer.  Every block of a
// shard rebuilds the buckets and codes its share of the shard's x and z.  Replaces
// k_sort_chunks + k_rank_codes (41 + 78 us at the bench shape).
constexpr int kBucketNB = 2048;
constexpr int kBucketNC = 256;          // value-range bins of the sampled CDF (refine = 1)
constexpr int64_t kBucketMaxZ = 16384;  // 128 KiB of z in LDS
constexpr size_t kBucketLds = sizeof(double) * kBucketMaxZ + sizeof(unsigned) * (3 * kBucketNB + 2);

template <typename T>
__device__ __forceinline__ double bucket_value(T v) { return (double)v; }

constexpr int kZPer = (int)(kBucketMaxZ / kSortThreads);  // z-values per thread (registers)
constexpr int kEPer = 8;  // code elements per thread per round, loads issued together

// Exclusive prefix of cnt[0 .. NB) into st[0 .. NB] (st[NB] = total), two buckets per thread.
__device__ __forceinline__ void bucket_prefix(const unsigned* cnt, unsigned* st,
                                              unsigned* wave_tot) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int i0 = 2 * tid;  // kBucketNB == 2 * kSortThreads
  const unsigned a = cnt[i0], b = cnt[i0 + 1];
  unsigned v = a + b;
  for (int o = 1; o < kWave; o <<= 1) {  // inclusive wave scan
    const unsigned t = __shfl_up(v, o, kWave);
    if (lane >= o) v += t;
  }
  if (lane == kWave - 1) wave_tot[wid] = v;
  __syncthreads();
  unsigned base = 0;
  for (int w = 0; w < wid; ++w) base += wave_tot[w];
  const unsigned excl = base + v - (a + b);
  st[i0] = excl;
  st[i0 + 1] = excl + a;
  if (tid == kSortThreads - 1) st[kBucketNB] = excl + a + b;
  __syncthreads();
}

// COUNT = true: the complete count instead of codes (tw_count_pairs_sorted): the same
// buckets, only the x-values, and the block's sum of their codes (#z < x, plus #z <= x for
// half-ties) added to out[s] — the integer of k_count_complete / k_rank_count.
// The shard's z is loaded ONCE into registers (kZPer per thread, all loads in flight
// together); the first round of this block's code elements is loaded beside it.  Bucket scans
// read four values per trip.
// Codes are written with row strides sx / sz (multiples of 8, so rows are 16-B aligned).
template <typename T, int PRED, bool COUNT = false>
__global__ __launch_bounds__(kSortThreads) void k_rank_codes_bucket(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, int parts, int refine, int64_t sx, int64_t sz,
    uint16_t* __restrict__ cx, uint16_t* __restrict__ cx2, uint16_t* __restrict__ pz,
    unsigned long long* __restrict__ out, NextStep nxt, EmitStep em) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* zb = (T*)smem;                                                 // z by bucket
  unsigned* cs = (unsigned*)(smem + sizeof(double) * kBucketMaxZ);  // NB + 1 sample prefix
  unsigned* st = cs + kBucketNB + 1;                                // NB + 1 bucket starts
  unsigned* cur = st + kBucketNB + 1;                               // NB counts
  __shared__ double red_min[kSortThreads / kWave], red_max[kSortThreads / kWave];
  __shared__ unsigned wave_tot[kSortThreads / kWave];
  __shared__ unsigned nan_z;
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t xb = x_off[s], nx = x_off[s + 1] - xb;
  const int64_t zo = z_off[s], nz = z_off[s + 1] - zo;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  // this block's share of the shard's elements (x first, then z; COUNT: x only)
  const int64_t tot = COUNT ? nx : nx + nz, per = (tot + parts - 1) / parts;
  const int64_t e0 = (int64_t)part * per, e1 = e0 + per < tot ? e0 + per : tot;
  auto elem = [&](int64_t e) -> T { return e < nx ? x[xb + e] : z[zo + (e - nx)]; };
  TW_PHASE(0);
  // 0. all loads of the first phase in flight at once: the shard's z, the first code round
  T zr[kZPer], er[kEPer];
#pragma unroll
  for (int r = 0; r < kZPer; ++r) {
    const int64_t j = tid + (int64_t)r * kSortThreads;
    zr[r] = j < nz ? z[zo + j] : (T)0;
  }
  // the next repartition (tw_count_pairs_sorted_step): this thread's gathers in flight
  // through the whole kernel (the z loads above go first), stored at the end; the count
  // path's first code round is then loaded in phase 5, so the batch's registers fit
  NextBatch<kSortThreads, 8> nb(nxt);
  if (COUNT) {
    next_step_zero<kSortThreads>(nxt);
    nb.issue();
  } else {
#pragma unroll
    for (int r = 0; r < kEPer; ++r) {
      const int64_t e = e0 + tid + (int64_t)r * kSortThreads;
      er[r] = e < e1 ? elem(e) : (T)0;
    }
  }
  // 1. range of the finite z
  double mn = __builtin_inf(), mx = -__builtin_inf();
#pragma unroll
  for (int r = 0; r < kZPer; ++r) {
    const double v = bucket_value<T>(zr[r]);
    if (tid + (int64_t)r * kSortThreads < nz && v - v == 0.0) {  // finite (not NaN, not inf)
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double a = __shfl_xor(mn, o, kWave), b = __shfl_xor(mx, o, kWave);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  for (int i = tid; i < kBucketNB; i += kSortThreads) cur[i] = 0;
  if (tid == 0) nan_z = 0;
  if (lane == 0) {
    red_min[wid] = mn;
    red_max[wid] = mx;
  }
  __syncthreads();
  TW_PHASE(1);
  mn = red_min[0];
  mx = red_max[0];
  for (int w = 1; w < kSortThreads / kWave; ++w) {
    mn = red_min[w] < mn ? red_min[w] : mn;
    mx = red_max[w] > mx ? red_max[w] : mx;
  }
  // the next repartition (tw_count_pairs_sorted_step): this thread's gathers in flight
  // through the LDS-bound bucketing and coding phases, stored at the end
  const int nbin = refine ? kBucketNC : kBucketNB;
  const double scale = mx > mn ? (double)nbin / (mx - mn) : 0.0;
  // value-range bin of v and its position t in [0, 1] inside it (NaN u -> bin 0, t = 0)
  auto coarse = [&](double v, double& t) -> int {
    const double u = (v - mn) * scale;
    const int b = (int)__builtin_fmin(__builtin_fmax(u, 0.0), (double)(nbin - 1));
    t = __builtin_fmin(__builtin_fmax(u - (double)b, 0.0), 1.0);
    return b;
  };
  // 2. refine: the sampled CDF.  Thread t samples z[t + (t mod 16) * 1024], spread over the
  // whole shard whatever its order.
  double fscale = 0.0;
  if (refine) {
    const int rs = tid & (kZPer - 1);
    T sv = zr[0];
#pragma unroll
    for (int r = 1; r < kZPer; ++r) sv = rs == r ? zr[r] : sv;
    const bool sin = tid + (int64_t)rs * kSortThreads < nz && !is_nan_score<T>(sv);
    double t;
    if (sin) atomicAdd(&cur[coarse(bucket_value<T>(sv), t)], 1u);
    __syncthreads();
    bucket_prefix(cur, cs, wave_tot);  // bins >= kBucketNC are empty
    fscale = (double)kBucketNB / (double)cs[kBucketNB];
    for (int i = tid; i < kBucketNB; i += kSortThreads) cur[i] = 0;
    __syncthreads();
  }
  TW_PHASE(2);
  auto bucket = [&](double v) -> int {
    double t;
    const int b = coarse(v, t);
    if (!refine) return b;
    const unsigned c0 = cs[b], c1 = cs[b + 1];
    const double pos = (double)c0 + t * (double)(c1 - c0);
    return (int)__builtin_fmin(pos * fscale, (double)(kBucketNB - 1));  // NaN (no sample): NB-1
  };
  // 3. counting sort of z by bucket: one returning atomic per z gives its slot in the bucket
  int zbk[kZPer];
  unsigned zslot[kZPer];
#pragma unroll
  for (int r = 0; r < kZPer; ++r) {
    const bool live = tid + (int64_t)r * kSortThreads < nz;
    zbk[r] = -1;
    if (live && !is_nan_score<T>(zr[r])) {
      zbk[r] = bucket(bucket_value<T>(zr[r]));
      zslot[r] = atomicAdd(&cur[zbk[r]], 1u);
    } else if (live) {
      atomicAdd(&nan_z, 1u);
    }
  }
  __syncthreads();
  bucket_prefix(cur, st, wave_tot);
  TW_PHASE(3);
#pragma unroll
  for (int r = 0; r < kZPer; ++r)
    if (zbk[r] >= 0) zb[st[zbk[r]] + zslot[r]] = zr[r];
  __syncthreads();
  TW_PHASE(4);
  const unsigned n_valid = st[kBucketNB];
  // 5. codes of this block's share (rounds of kEPer elements per thread; the first is loaded)
  unsigned long long acc = 0;
  for (int64_t r0 = e0; r0 < e1; r0 += (int64_t)kEPer * kSortThreads) {
    if (COUNT || r0 != e0) {
#pragma unroll
      for (int r = 0; r < kEPer; ++r) {
        const int64_t e = r0 + tid + (int64_t)r * kSortThreads;
        er[r] = e < e1 ? elem(e) : (T)0;
      }
    }
#pragma unroll
    for (int r = 0; r < kEPer; ++r) {
      const int64_t e = r0 + tid + (int64_t)r * kSortThreads;
      if (e >= e1) continue;
      const bool isx = e < nx;
      const T v = er[r];
      unsigned lo = 0, hi = 0;
      if (is_nan_score<T>(v)) {
        lo = isx ? 0u : n_valid;  // NaN x: below every p; NaN z: above every c
        hi = lo;
      } else {
        const int b = bucket(bucket_value<T>(v));
        const unsigned b0 = st[b], b1 = st[b + 1];
        lo = b0;
        hi = b0;
        unsigned q = b0;
        for (; q + 4 <= b1; q += 4) {  // four independent LDS reads per trip
          const T w0 = zb[q], w1 = zb[q + 1], w2 = zb[q + 2], w3 = zb[q + 3];
          lo += (unsigned)(w0 < v) + (unsigned)(w1 < v) + (unsigned)(w2 < v) + (unsigned)(w3 < v);
          if (PRED == TW_PRED_HALF)
            hi += (unsigned)(w0 <= v) + (unsigned)(w1 <= v) + (unsigned)(w2 <= v) +
                  (unsigned)(w3 <= v);
        }
        for (; q < b1; ++q) {
          const T w = zb[q];
          lo += w < v;
          if (PRED == TW_PRED_HALF) hi += w <= v;
        }
      }
      if constexpr (COUNT) {
        acc += lo + (PRED == TW_PRED_HALF ? hi : 0u);
      } else if (isx) {
        cx[(int64_t)s * sx + e] = (uint16_t)lo;
        if (PRED == TW_PRED_HALF) cx2[(int64_t)s * sx + e] = (uint16_t)hi;
      } else {
        pz[(int64_t)s * sz + (e - nx)] = (uint16_t)lo;
      }
    }
  }
  TW_PHASE(5);
  if constexpr (COUNT) {
    nb.commit();
    acc = wave_sum_u64(acc);
    __shared__ unsigned long long part_acc[kSortThreads / kWave];
    if (lane == 0) part_acc[wid] = acc;
    __syncthreads();
    if (tid == 0) {
      unsigned long long b = 0;
      for (int w = 0; w < kSortThreads / kWave; ++w) b += part_acc[w];
      if (b) atomicAdd(out + s, b);
    }
    if (em.active) {  // the next repartition as records (records.h): this block's x share
                      // and a 1/parts share of the shard's z in one staged round (the LDS of
                      // the z buckets is free now), then its stride of the tails
      const int64_t zper = (nz + parts - 1) / parts;
      const int64_t za = zo + std::min<int64_t>(nz, (int64_t)part * zper);
      const int64_t zbnd = zo + std::min<int64_t>(nz, (int64_t)(part + 1) * zper);
      const int N = em.n_shards;
      if (lb == 0)
        for (int i = tid; i <= N; i += kSortThreads) {
          if (em.zero_x) em.zero_x[i] = 0;
          if (em.zero_z) em.zero_z[i] = 0;
        }
      if ((e1 - e0) + (zbnd - za) <= (int64_t)kSortThreads * 8 && 2 * N + 2 <= kBucketNB) {
        char* lds = smem;  // zb's 128 KiB: 8192 staged records (8 + 4 + 2 B)
        uint64_t* sv = (uint64_t*)lds;
        uint32_t* sq = (uint32_t*)(lds + 8 * kSortThreads * 8);
        uint16_t* sbk = (uint16_t*)(lds + 12 * kSortThreads * 8);
        emit_block_staged<kSortThreads>(em, xb + e0, xb + e1, za, zbnd, cur, cs, st, sv, sq,
                                        sbk, wave_tot);
      } else {
        emit_range<kSortThreads, 8>(em.xv, em.xp, xb + e0, xb + e1, em.nx, em.fx, em.kx, em.dx,
                                    N, em.x_off, em.cur_x, em.nxv, em.nxp, cs, st);
        emit_range<kSortThreads, 8>(em.zv, em.zp, za, zbnd, em.nz, em.fz, em.kz, em.dz, N,
                                    em.z_off, em.cur_z, em.nzv, em.nzp, cs, st);
      }
      emit_tails<kSortThreads>(em, lb, (int)gridDim.x, cs, st);
    }
  }
}

// The first records of a tw_count_pairs_sorted_steps call: the arrays in position order
// (implicit positions) appended to their buckets under the first step's permutation.
__global__ __launch_bounds__(kSortThreads) void k_emit_records(EmitStep em) {
  __shared__ unsigned hist[kBucketNB + 1], base[kBucketNB + 1];
  constexpr int64_t C = (int64_t)kSortThreads * 8;
  for (int64_t c = (int64_t)blockIdx.x * C; c < em.nx; c += (int64_t)gridDim.x * C)
    emit_range<kSortThreads, 8>(em.xv, em.xp, c, c + C < em.nx ? c + C : em.nx, em.nx, em.fx,
                                em.kx, em.dx, em.n_shards, em.x_off, em.cur_x, em.nxv, em.nxp,
                                hist, base);
  for (int64_t c = (int64_t)blockIdx.x * C; c < em.nz; c += (int64_t)gridDim.x * C)
    emit_range<kSortThreads, 8>(em.zv, em.zp, c, c + C < em.nz ? c + C : em.nz, em.nz, em.fz,
                                em.kz, em.dz, em.n_shards, em.z_off, em.cur_z, em.nzv, em.nzp,
                                hist, base);
}

// After the last step: the records written back in position order.
__global__ __launch_bounds__(kBlock) void k_records_to_arrays(
    const uint64_t* __restrict__ xv, const uint32_t* __restrict__ xp, int64_t nx,
    const uint64_t* __restrict__ zv, const uint32_t* __restrict__ zp, int64_t nz,
    uint64_t* __restrict__ x_out, uint64_t* __restrict__ z_out) {
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < nx + nz;
       e += (int64_t)gridDim.x * kBlock) {
    if (e < nx)
      x_out[xp[e]] = xv[e];
    else
      z_out[zp[e - nx]] = zv[e - nx];
  }
}

// tw_count_sorted_set_bucket: 0 = sort + binary search, 1 = equal-depth buckets (default),
// 2 = coarse (value-range) buckets only
static int g_sorted_by_bucket = 1;

template <typename T, int PRED>
int launch_bucket_count(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                        int32_t n_shards, int64_t max_nx, uint64_t* out, const NextStep& nxt,
                        hipStream_t st, const EmitStep& em = EmitStep{}) {
  const size_t lds_b = kBucketLds;
  static bool attr = false;
  if (!attr) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_codes_bucket<T, PRED, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_b));
    attr = true;
  }
  // enough blocks per shard for the chip: each rebuilds the shard's buckets, then sums the
  // codes of its share of x
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(512, n_shards),
                                                                ceil_div(max_nx, 4096)));
  TW_ARG_CHECK((int64_t)n_shards * parts < (1ll << 31), "tw_count_pairs_sorted: grid too large");
  hipLaunchKernelGGL((k_rank_codes_bucket<T, PRED, true>), dim3(n_shards * parts),
                     dim3(kSortThreads), lds_b, st, (const T*)x, x_off, (const T*)z, z_off, parts,
                     (int)(g_sorted_by_bucket == 1), max_nx, (int64_t)0, nullptr, nullptr, nullptr,
                     (unsigned long long*)out, nxt, em);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T>
int launch_rank(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                int32_t n_shards, int64_t max_nx, int64_t max_nz, int32_t pred, void* work,
                uint64_t* out, hipStream_t st) {
  if (max_nz <= kBucketMaxZ && g_sorted_by_bucket) {
    if (pred == TW_PRED_HALF)
      return launch_bucket_count<T, TW_PRED_HALF>(x, x_off, z, z_off, n_shards, max_nx, out,
                                                  NextStep{}, st);
    return launch_bucket_count<T, TW_PRED_GT>(x, x_off, z, z_off, n_shards, max_nx, out,
                                              NextStep{}, st);
  }
  const RankPlan p = plan_rank(max_nx, max_nz);
  TW_ARG_CHECK((int64_t)n_shards * p.chunks < (1ll << 31) &&
                   (int64_t)n_shards * p.tiles_x < (1ll << 31),
               "tw_count_pairs_sorted: grid too large");
  const size_t lds = sizeof(uint64_t) * p.C;
  const size_t lds_rank = sizeof(uint64_t) * std::min<int64_t>((int64_t)p.chunks * p.C, kMaxChunk);
  static bool attrs_set = false;  // > 64 KiB of dynamic LDS must be opted into once
  if (!attrs_set) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 8>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 16>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_count<T, TW_PRED_GT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_count<T, TW_PRED_HALF>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    attrs_set = true;
  }
  const int E = std::max(4, p.C / kSortThreads);
  if (E == 4)
    hipLaunchKernelGGL((k_sort_chunks<T, 4>), dim3(n_shards * p.chunks), dim3(p.C / 4), lds, st,
                       (const T*)z, z_off, p.chunks, p.C, (uint64_t*)work);
  else if (E == 8)
    hipLaunchKernelGGL((k_sort_chunks<T, 8>), dim3(n_shards * p.chunks), dim3(p.C / 8), lds, st,
                       (const T*)z, z_off, p.chunks, p.C, (uint64_t*)work);
  else
    hipLaunchKernelGGL((k_sort_chunks<T, 16>), dim3(n_shards * p.chunks), dim3(p.C / 16), lds,
                       st, (const T*)z, z_off, p.chunks, p.C, (uint64_t*)work);
  TW_LAUNCH_CHECK();
  if (pred == TW_PRED_HALF)
    hipLaunchKernelGGL((k_rank_count<T, TW_PRED_HALF>), dim3(n_shards * p.tiles_x),
                       dim3(kSortThreads), lds_rank, st, (const T*)x, x_off, (const uint64_t*)work,
                       p.chunks, p.C, p.tiles_x, (unsigned long long*)out);
  else
    hipLaunchKernelGGL((k_rank_count<T, TW_PRED_GT>), dim3(n_shards * p.tiles_x),
                       dim3(kSortThreads), lds_rank, st, (const T*)x, x_off, (const uint64_t*)work,
                       p.chunks, p.C, p.tiles_x, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// ------------------------------------------------ ranked device-RNG incomplete count
// tw_count_pairs_rng_ws: the draws of tw_count_pairs_rng (Philox blocks of two pairs, Lemire
// index maps), but the compares read 16-bit RANK CODES from LDS instead of gathering doubles
// from L2.  With zs the shard's sorted z keys:
//   p_j  = #{zs < z_j}          (first position of z_j's value)
//   c_i  = #{zs < x_i}          x_i >  z_j  <=>  c_i  > p_j
//   c'_i = #{zs <= x_i}         x_i >= z_j  <=>  c'_i > p_j      (half-ties: add both)
// exact for any keys (order_key makes -0 == +0; NaN x gets c = c' = 0, NaN z the largest p,
// so every compare with a NaN is false, as in NumPy).  The random 8-B gathers of the plain
// kernel fetch a whole L2 line each and bound it by L2 bandwidth; the codes of a 15625-value
// shard pair are 62 KiB (94 KiB with ties) and sit in LDS.  z is sorted in the sorted-count
// path's chunks (k_sort_chunks); a code is the sum of its per-chunk binary searches.  Applies
// when every shard has nx, nz < 65536 and the codes fit in LDS; otherwise the plain kernel runs.
constexpr int kRngThreads = 1024;
#ifndef TW_CODE_ELEMS
#define TW_CODE_ELEMS 4
#endif
constexpr int kCodeElems = TW_CODE_ELEMS;  // elements per thread in k_rank_codes

template <typename T, int PRED>
__global__ __launch_bounds__(kSortThreads) void k_rank_codes(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, const uint64_t* __restrict__ sorted, int chunks, int C,
    int tiles, int64_t max_nx, int64_t max_nz, uint16_t* __restrict__ cx,
    uint16_t* __restrict__ cx2, uint16_t* __restrict__ pz) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / tiles;
  const int t = lb - s * tiles;
  const int64_t xb = x_off[s], nx = x_off[s + 1] - xb;
  const int64_t zb = z_off[s], nz = z_off[s + 1] - zb;
  // this thread's elements: x-values first, then z-values, of the shard's (nx + nz)
  const int64_t e0 = (int64_t)t * (kSortThreads * kCodeElems);
  uint64_t k[kCodeElems];
  uint32_t lo[kCodeElems], hi[kCodeElems];
  bool isx[kCodeElems], live[kCodeElems];
#pragma unroll
  for (int r = 0; r < kCodeElems; ++r) {
    const int64_t e = e0 + r * kSortThreads + threadIdx.x;
    isx[r] = e < nx;
    live[r] = e < nx + nz;
    T v = (T)0;
    if (isx[r]) v = x[xb + e];
    else if (live[r]) v = z[zb + (e - nx)];
    k[r] = order_key<T>(v);
    if (isx[r] && is_nan_score<T>(v)) live[r] = false;  // NaN x: codes 0, below every p_j
    lo[r] = hi[r] = 0;
  }
  // #{keys < k} (and <= k) summed over the shard's sorted chunks, staged as in k_rank_count
  const int group = (int)std::max<int64_t>(1, kMaxChunk / C);
  for (int c0 = 0; c0 < chunks; c0 += group) {
    const int ng = std::min(group, chunks - c0);
    const uint64_t* src = sorted + ((int64_t)s * chunks + c0) * C;
    __syncthreads();
    for (int i = threadIdx.x; i < ng * C; i += kSortThreads) keys[i] = src[i];
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
      const uint64_t* kc = keys + g * C;
#pragma unroll
      for (int r = 0; r < kCodeElems; ++r) {
        if (live[r]) {
          lo[r] += lower_bound_lds(kc, C, k[r]);
          if (PRED == TW_PRED_HALF && isx[r]) hi[r] += upper_bound_lds(kc, C, k[r]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kCodeElems; ++r) {
    const int64_t e = e0 + r * kSortThreads + threadIdx.x;
    if (isx[r]) {
      cx[(int64_t)s * max_nx + e] = (uint16_t)lo[r];
      if (PRED == TW_PRED_HALF) cx2[(int64_t)s * max_nx + e] = (uint16_t)hi[r];
    } else if (e < nx + nz) {
      pz[(int64_t)s * max_nz + (e - nx)] = (uint16_t)lo[r];
    }
  }
}

// Code rows in the work buffer and in LDS have strides rounded up to 8 codes, so a shard's
// codes are staged with 16-B loads (2 per thread for a 15625-value shard pair) issued
// together, instead of one dependent u16 load per loop trip.
__device__ __forceinline__ int64_t al8(int64_t n) { return (n + 7) & ~(int64_t)7; }

template <int PRED>
__device__ __forceinline__ void stage_codes(uint16_t* __restrict__ lds, const uint16_t* __restrict__ cx,
                                            const uint16_t* __restrict__ cx2,
                                            const uint16_t* __restrict__ pz, int64_t nx,
                                            int64_t nz) {
  constexpr int NC = PRED == TW_PRED_HALF ? 2 : 1;
  const int64_t vx = al8(nx) / 8, vz = al8(nz) / 8, tot = NC * vx + vz;
  const uint4* sx = (const uint4*)cx;
  const uint4* sx2 = (const uint4*)cx2;
  const uint4* sz = (const uint4*)pz;
  uint4* d = (uint4*)lds;  // [x codes | (x codes, >=) | z codes], each al8 long
  constexpr int U = 4;
  for (int64_t i0 = threadIdx.x; i0 < tot; i0 += (int64_t)U * blockDim.x) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < tot) v[u] = i < vx ? sx[i] : (NC == 2 && i < 2 * vx) ? sx2[i - vx] : sz[i - NC * vx];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < tot) d[i] = v[u];
    }
  }
}

template <int PRED>
__global__ __launch_bounds__(kRngThreads) void k_count_rng_ranked(
    const int64_t* __restrict__ x_off, const int64_t* __restrict__ z_off,
    const uint16_t* __restrict__ cx, const uint16_t* __restrict__ cx2,
    const uint16_t* __restrict__ pz, int64_t sx, int64_t sz, int64_t B, int parts,
    uint32_t k0, uint32_t k1, uint32_t sid, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint16_t codes[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's parts share one L2
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t nx = x_off[s + 1] - x_off[s], nz = z_off[s + 1] - z_off[s];
  unsigned acc = 0;
  if (nx > 0 && nz > 0) {
    uint16_t* lx = codes;
    uint16_t* lx2 = codes + al8(nx);
    uint16_t* lz = codes + (PRED == TW_PRED_HALF ? 2 : 1) * al8(nx);
    stage_codes<PRED>(codes, cx + (int64_t)s * sx, cx2 + (int64_t)s * sx, pz + (int64_t)s * sz,
                      nx, nz);
    __syncthreads();
    const uint32_t ss = (uint32_t)s + sid;
    const int64_t nq = (B + 1) / 2;
    const int64_t per = (nq + parts - 1) / parts;
    const int64_t q0 = (int64_t)part * per, q1 = std::min<int64_t>(nq, q0 + per);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += kRngThreads) {
      const u32x4 r = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), ss, 0u}, k0, k1);
      const uint32_t i0 = lemire_index(r.a, (uint32_t)nx, q, ss, 0, k0, k1);
      const uint32_t j0 = lemire_index(r.b, (uint32_t)nz, q, ss, 1, k0, k1);
      const uint32_t pj0 = lz[j0];
      acc += lx[i0] > pj0;
      if (PRED == TW_PRED_HALF) acc += lx2[i0] > pj0;
      if (2 * q + 1 < B) {
        const uint32_t i1 = lemire_index(r.c, (uint32_t)nx, q, ss, 2, k0, k1);
        const uint32_t j1 = lemire_index(r.d, (uint32_t)nz, q, ss, 3, k0, k1);
        const uint32_t pj1 = lz[j1];
        acc += lx[i1] > pj1;
        if (PRED == TW_PRED_HALF) acc += lx2[i1] > pj1;
      }
    }
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kRngThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < kRngThreads / kWave; ++w) b += part_sum[w];
    if (b) atomicAdd(out + s, b);
  }
}

// 16-byte vectors of pair indices: 4 int32 or 2 int64 per load.
template <typename I> struct IdxVec;
typedef int32_t tw_i32x4 __attribute__((ext_vector_type(4)));
typedef int64_t tw_i64x2 __attribute__((ext_vector_type(2)));
template <> struct IdxVec<int32_t> {
  using V = int4;
  using NVec = tw_i32x4;  // clang vector of the same 16 bytes (nontemporal builtin operand)
  static constexpr int N = 4;
  __device__ static __forceinline__ int32_t at(const V& v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
  }
};
template <> struct IdxVec<int64_t> {
  using V = longlong2;
  using NVec = tw_i64x2;
  static constexpr int N = 2;
  __device__ static __forceinline__ int64_t at(const V& v, int e) { return e == 0 ? v.x : v.y; }
};

// Incomplete count on explicit index pairs (UB replay: NumPy's randint draws, compute_stats.py:
// 22-42) through the rank codes: a block stages its shard's 16-bit codes in LDS, so the two
// per-pair gathers are LDS reads and only the indices stream from HBM — 8 B per pair with int32
// indices, 16 B with int64 (the plain k_count_idx pulls an L2 line per
// gathered score).  Indices are absolute; one outside its shard's span (allowed by
// tw_count_pairs_idx) compares the scores themselves.
// The index streams are read as 16-B vectors (VEC: the host checked the pointers' alignment;
// unaligned heads/tails of a part go through scalar loads), U vectors of each stream per
// thread and batch, the first batch issued BEFORE the codes are staged so its latency hides
// behind the staging.  PIPE: each later batch is issued before the previous one is compared
// (two register buffers); otherwise after it (one buffer; the other waves hide the latency).
// int32 indices use 32-bit offset arithmetic.  Two 1024-thread blocks per CU (62.5 KiB of
// codes each) need <= 64 VGPRs: __launch_bounds__(1024, 8) = 8 waves per SIMD.
template <typename T, int PRED, typename I, bool VEC, int UV = 2, bool NT = false,
          bool PIPE = true>
__global__ __launch_bounds__(kRngThreads, 8) void k_count_idx_ranked(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, const uint16_t* __restrict__ cx,
    const uint16_t* __restrict__ cx2, const uint16_t* __restrict__ pz, int64_t sx, int64_t sz,
    const I* __restrict__ ix, const I* __restrict__ iz, const int64_t* __restrict__ pair_off,
    int parts, unsigned long long* __restrict__ out) {
  using IV = IdxVec<I>;
  using V = typename IV::V;
  constexpr int NV = VEC ? IV::N : 1;  // pairs per load
  constexpr int U = VEC ? UV : 4;      // loads of each stream per thread and batch
  extern __shared__ __attribute__((aligned(16))) uint16_t codes[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's parts share one L2
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int tid = threadIdx.x;
  const int64_t xb = x_off[s], zb = z_off[s];
  const int64_t nx = x_off[s + 1] - xb, nz = z_off[s + 1] - zb;
  const uint16_t* lx = codes;
  const uint16_t* lx2 = codes + al8(nx);
  const uint16_t* lz = codes + (PRED == TW_PRED_HALF ? 2 : 1) * al8(nx);
  const int64_t pb = pair_off[s], pe = pair_off[s + 1];
  const int64_t per = (pe - pb + parts - 1) / parts;
  const int64_t q0 = std::min<int64_t>(pe, pb + (int64_t)part * per);
  const int64_t q1 = std::min<int64_t>(pe, q0 + per);
  // [a0, a1): the NV-aligned body of [q0, q1), loaded as vectors
  const int64_t a0 = std::min<int64_t>(q1, (q0 + NV - 1) / NV * NV);
  const int64_t a1 = std::max<int64_t>(a0, q1 / NV * NV);
  const int nv = (int)((a1 - a0) / NV);
  // span test of one pair: block-local offsets i, j (32-bit) and whether both lie in the shard
  auto local = [&](I a, I b, uint32_t& i, uint32_t& j) -> bool {
    if constexpr (sizeof(I) == 4) {  // 32-bit offsets: the arrays hold < 2^31 elements
      i = (uint32_t)(a - (int32_t)xb);
      j = (uint32_t)(b - (int32_t)zb);
      return i < (uint32_t)nx && j < (uint32_t)nz;
    } else {
      const uint64_t i64 = (uint64_t)(a - xb), j64 = (uint64_t)(b - zb);
      i = (uint32_t)i64;
      j = (uint32_t)j64;
      return i64 < (uint64_t)nx && j64 < (uint64_t)nz;
    }
  };
  // an index outside its shard's span compares the scores themselves
  auto gathered = [&](I a, I b) -> unsigned {
    const T xv = x[a], zv = z[b];
    return (unsigned)(xv > zv) + (PRED == TW_PRED_HALF ? (unsigned)(xv >= zv) : 0u);
  };
  auto one = [&](I a, I b) -> unsigned {
    uint32_t i, j;
    if (local(a, b, i, j)) {
      const unsigned pj = lz[j];
      unsigned r = (unsigned)lx[i] > pj;
      if (PRED == TW_PRED_HALF) r += (unsigned)lx2[i] > pj;
      return r;
    }
    return gathered(a, b);
  };
  const I* __restrict__ px = ix + a0;
  const I* __restrict__ pzi = iz + a0;
  auto load = [&](const I* p, int v) -> V {
    if constexpr (VEC && NT) {
      const typename IV::NVec r = __builtin_nontemporal_load(((const typename IV::NVec*)p) + v);
      return __builtin_bit_cast(V, r);
    } else if constexpr (VEC) {
      return ((const V*)p)[v];
    } else {
      V r;
      r.x = p[v];
      return r;
    }
  };
  // the batch's U x NV pairs without branches: out-of-span pairs read code 0 and count nothing,
  // and only when some lane of the wave has one (never, for slice plans) the scores are gathered
  auto compare = [&](const V (&A)[U], const V (&Bv)[U], int base) -> unsigned {
    unsigned c = 0;
#ifdef TW_IDX_STREAM_ONLY  // kernel study (tools/phase_codes.py): the index streams alone
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < NV; ++e) c += (unsigned)(IV::at(A[u], e) ^ IV::at(Bv[u], e)) & 1u;
    return c;
#endif
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = base + tid + u * kRngThreads < nv;
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        uint32_t i, j;
        const bool in = local(IV::at(A[u], e), IV::at(Bv[u], e), i, j) && live;
        bad |= live && !in;
        i = in ? i : 0u;
        j = in ? j : 0u;
        const unsigned pj = lz[j];
        unsigned r = (unsigned)lx[i] > pj;
        if (PRED == TW_PRED_HALF) r += (unsigned)lx2[i] > pj;
        c += in ? r : 0u;
      }
    }
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool live = base + tid + u * kRngThreads < nv;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          uint32_t i, j;
          const I a = IV::at(A[u], e), b = IV::at(Bv[u], e);
          if (live && !local(a, b, i, j)) c += gathered(a, b);
        }
      }
    }
    return c;
  };
  // one batch of U vectors per stream, unconditionally (positions past the end re-read the
  // last vector and count nothing): branch-free loads keep the compiler's wait counts exact
  auto load_batch = [&](V (&A)[U], V (&Bv)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = min(base + tid + u * kRngThreads, nv - 1);
      A[u] = load(px, v);
      Bv[u] = load(pzi, v);
    }
  };
  constexpr int step = U * kRngThreads;
  const int nb = (nv + step - 1) / step;  // batches (block-uniform)
  V A[U], Bv[U];
  if (nb > 0) load_batch(A, Bv, 0);  // in flight while the codes are staged
  if (nx > 0 && nz > 0)
    stage_codes<PRED>(codes, cx + (int64_t)s * sx, cx2 + (int64_t)s * sx, pz + (int64_t)s * sz,
                      nx, nz);
  __syncthreads();
  unsigned acc = 0;
  // scalar head [q0, a0) and tail [a1, q1) (fewer than NV pairs each)
  if (tid < a0 - q0) acc += one(ix[q0 + tid], iz[q0 + tid]);
  if (tid < q1 - a1) acc += one(ix[a1 + tid], iz[a1 + tid]);
  if constexpr (PIPE) {
    // two register buffers used in turn (no copies between them, which would make the
    // compiler wait for the in-flight batch): batch k+1 loads while batch k is compared
    V A2[U], B2[U];
    for (int k = 0; k < nb; k += 2) {
      load_batch(A2, B2, (k + 1) * step);
      acc += compare(A, Bv, k * step);
      load_batch(A, Bv, (k + 2) * step);
      acc += compare(A2, B2, (k + 1) * step);
    }
  } else {
    for (int k = 0; k < nb; ++k) {
      acc += compare(A, Bv, k * step);
      load_batch(A, Bv, (k + 1) * step);
    }
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kRngThreads / kWave];
  const int lane = tid & (kWave - 1), wid = tid / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (tid == 0) {
    unsigned long long sum = 0;
    for (int w = 0; w < kRngThreads / kWave; ++w) sum += part_sum[w];
    if (sum) atomicAdd(out + s, sum);
  }
}

// tw_count_rng_set_codes: 3 = float32 score images in LDS, no codes (default; falls back to
// the codes when a shard pair's images do not fit); codes by 0 = sort + binary search,
// 1 = equal-depth buckets, 2 = value-range buckets
static int g_rng_codes_by_bucket = 3;

struct RngRankPlan {
  bool ok;
  int C, chunks, tiles, parts, code_parts;
  int64_t sx, sz;  // code row strides (multiples of 8 codes: 16-B aligned rows)
  int64_t keys_bytes, cx_off, cx2_off, pz_off, total;
  size_t lds;
};

static RngRankPlan plan_rng_ranked(int32_t n_shards, int64_t max_nx, int64_t max_nz, int32_t pred,
                                   int64_t B) {
  RngRankPlan p{};
  p.ok = n_shards > 0 && max_nx > 0 && max_nz > 0 && max_nz < 65536 && max_nx < 65536 &&
         (pred == TW_PRED_GT || pred == TW_PRED_HALF);
  if (!p.ok) return p;
  const RankPlan rp = plan_rank(max_nx, max_nz);  // the sorted-count path's z chunks
  p.C = rp.C;
  p.chunks = rp.chunks;
  p.tiles = (int)ceil_div(max_nx + max_nz, (int64_t)kSortThreads * kCodeElems);
  const int nc = pred == TW_PRED_HALF ? 2 : 1;
  p.sx = (max_nx + 7) / 8 * 8;
  p.sz = (max_nz + 7) / 8 * 8;
  p.lds = (size_t)(nc * p.sx + p.sz) * sizeof(uint16_t);
  p.ok = p.lds <= 160 * 1024 - 1024;
  // ~2 blocks of 1024 threads per CU over the whole grid, >= 8192 draws per block
  const int64_t nq = std::max<int64_t>(1, (B + 1) / 2);
  p.parts = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(512, n_shards),
                                                        ceil_div(nq, 8192)));
  // bucket-code blocks per shard: each rebuilds the shard's buckets and codes a share of one
  // or more rounds of kEPer elements per thread; >= 256 blocks over the grid when possible
  p.code_parts = (int)std::max<int64_t>(
      1, std::min<int64_t>(ceil_div(256, n_shards),
                           ceil_div(max_nx + max_nz, (int64_t)kSortThreads * kEPer)));
  auto al = [](int64_t b) { return ceil_div(b, 256) * 256; };
  p.keys_bytes = al((int64_t)n_shards * p.chunks * p.C * 8);
  p.cx_off = p.keys_bytes;
  p.cx2_off = p.cx_off + al((int64_t)n_shards * p.sx * 2);
  p.pz_off = p.cx2_off + (pred == TW_PRED_HALF ? al((int64_t)n_shards * p.sx * 2) : 0);
  p.total = p.pz_off + al((int64_t)n_shards * p.sz * 2);
  return p;
}

// Rank codes of every shard into the work buffer (plan_rng_ranked's layout): bucket codes for
// shards of <= kBucketMaxZ z-values, else sort + binary search.  Shared by the device-RNG and the
// replay (explicit index) draw-and-count kernels.
template <typename T, int PRED>
int launch_codes(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                 int32_t n_shards, int64_t max_nx, int64_t max_nz, const RngRankPlan& p,
                 void* work, hipStream_t st) {
  static bool attrs_set = false;
  if (!attrs_set) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 8>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<T, 16>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_codes<T, PRED>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(sizeof(uint64_t) * kMaxChunk)));
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_rank_codes_bucket<T, PRED>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)kBucketLds));
    attrs_set = true;
  }
  char* w = (char*)work;
  uint64_t* keys = (uint64_t*)w;
  uint16_t* cx = (uint16_t*)(w + p.cx_off);
  uint16_t* cx2 = (uint16_t*)(w + p.cx2_off);
  uint16_t* pz = (uint16_t*)(w + p.pz_off);
  if (max_nz <= kBucketMaxZ && g_rng_codes_by_bucket) {
    hipLaunchKernelGGL((k_rank_codes_bucket<T, PRED>), dim3(n_shards * p.code_parts),
                       dim3(kSortThreads), kBucketLds, st, (const T*)x, x_off, (const T*)z, z_off,
                       p.code_parts, (int)(g_rng_codes_by_bucket == 1), p.sx, p.sz, cx, cx2, pz,
                       nullptr, NextStep{}, EmitStep{});
  } else {
  const size_t lds_sort = sizeof(uint64_t) * p.C;
  const size_t lds_codes = sizeof(uint64_t) * std::min<int64_t>((int64_t)p.chunks * p.C, kMaxChunk);
  const int E = std::max(4, p.C / kSortThreads);
  const dim3 gs((unsigned)(n_shards * p.chunks));
  if (E == 4)
    hipLaunchKernelGGL((k_sort_chunks<T, 4>), gs, dim3(p.C / 4), lds_sort, st, (const T*)z,
                       z_off, p.chunks, p.C, keys);
  else if (E == 8)
    hipLaunchKernelGGL((k_sort_chunks<T, 8>), gs, dim3(p.C / 8), lds_sort, st, (const T*)z,
                       z_off, p.chunks, p.C, keys);
  else
    hipLaunchKernelGGL((k_sort_chunks<T, 16>), gs, dim3(p.C / 16), lds_sort, st, (const T*)z,
                       z_off, p.chunks, p.C, keys);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL((k_rank_codes<T, PRED>), dim3(n_shards * p.tiles), dim3(kSortThreads),
                     lds_codes, st, (const T*)x, x_off, (const T*)z, z_off, keys, p.chunks, p.C,
                     p.tiles, p.sx, p.sz, cx, cx2, pz);
  }
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T, int PRED>
int launch_rng_ranked(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, int64_t max_nx, int64_t max_nz, int64_t B, uint64_t seed,
                      uint64_t sid, const RngRankPlan& p, void* work, uint64_t* out,
                      hipStream_t st) {
  static bool attrs_set = false;
  if (!attrs_set) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_count_rng_ranked<PRED>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - 1024));
    attrs_set = true;
  }
  const int rc = launch_codes<T, PRED>(x, x_off, z, z_off, n_shards, max_nx, max_nz, p, work, st);
  if (rc != TW_OK) return rc;
  char* w = (char*)work;
  uint16_t* cx = (uint16_t*)(w + p.cx_off);
  uint16_t* cx2 = (uint16_t*)(w + p.cx2_off);
  uint16_t* pz = (uint16_t*)(w + p.pz_off);
  hipLaunchKernelGGL((k_count_rng_ranked<PRED>), dim3(n_shards * p.parts), dim3(kRngThreads),
                     p.lds, st, x_off, z_off, cx, cx2, pz, p.sx, p.sz, B, p.parts,
                     (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)sid,
                     (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T, int PRED, typename I, bool VEC, int UV = 2, bool NT = false,
          bool PIPE = true>
int launch_idx_ranked_v(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                        int32_t n_shards, int64_t max_nx, int64_t max_nz, const I* ix,
                        const I* iz, const int64_t* pair_off, const RngRankPlan& p, void* work,
                        uint64_t* out, hipStream_t st) {
  static bool attrs_set = false;
  if (!attrs_set) {
    TW_HIP_CHECK(hipFuncSetAttribute(
        (const void*)k_count_idx_ranked<T, PRED, I, VEC, UV, NT, PIPE>,
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024));
    attrs_set = true;
  }
  const int rc = launch_codes<T, PRED>(x, x_off, z, z_off, n_shards, max_nx, max_nz, p, work, st);
  if (rc != TW_OK) return rc;
  char* w = (char*)work;
  hipLaunchKernelGGL((k_count_idx_ranked<T, PRED, I, VEC, UV, NT, PIPE>),
                     dim3(n_shards * p.parts), dim3(kRngThreads), p.lds, st, (const T*)x, x_off,
                     (const T*)z, z_off, (const uint16_t*)(w + p.cx_off),
                     (const uint16_t*)(w + p.cx2_off), (const uint16_t*)(w + p.pz_off), p.sx,
                     p.sz, ix, iz, pair_off, p.parts, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// tw_count_idx_set_variant: int32 index streams, 0 = two 16-B loads per stream and batch,
// pipelined (default), 1 = the same as nontemporal loads, 2/3 = four loads, one buffer
// (plain / nontemporal), 4/5 = four loads pipelined (plain / nontemporal)
static int g_idx_variant = 0;

template <typename T, int PRED, typename I>
int launch_idx_ranked(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, int64_t max_nx, int64_t max_nz, const I* ix, const I* iz,
                      const int64_t* pair_off, const RngRankPlan& p, void* work, uint64_t* out,
                      hipStream_t st) {
  // 16-B vector loads of the index streams need 16-B aligned base pointers
  if ((((uintptr_t)ix | (uintptr_t)iz) & 15) == 0) {
    if constexpr (sizeof(I) == 4) {  // tuning variants (tw_count_idx_set_variant)
#define TW_V(U, N, P) return launch_idx_ranked_v<T, PRED, I, true, U, N, P>(x, x_off, z, z_off, n_shards, max_nx, max_nz, ix, iz, pair_off, p, work, out, st)
      switch (g_idx_variant) {
        case 1: TW_V(2, true, true);
        case 2: TW_V(4, false, false);
        case 3: TW_V(4, true, false);
        case 4: TW_V(4, false, true);
        case 5: TW_V(4, true, true);
        default: break;
      }
#undef TW_V
    }
    return launch_idx_ranked_v<T, PRED, I, true>(x, x_off, z, z_off, n_shards, max_nx, max_nz, ix,
                                                 iz, pair_off, p, work, out, st);
  }
  return launch_idx_ranked_v<T, PRED, I, false>(x, x_off, z, z_off, n_shards, max_nx, max_nz, ix,
                                                iz, pair_off, p, work, out, st);
}

}  // namespace tw

using namespace tw;

extern "C" int tw_permute_pair(const void* d_x_in, void* d_x_out, int64_t n, uint64_t key_x,
                               const void* d_z_in, void* d_z_out, int64_t m, uint64_t key_z,
                               void* stream);

extern "C" int tw_count_sorted_set_chunk(int64_t cap) {
  TW_ARG_CHECK(cap >= 1024 && cap <= kMaxChunk && (cap & (cap - 1)) == 0,
               "tw_count_sorted_set_chunk: cap must be a power of two in [1024, 16384]");
  g_chunk_cap = cap;
  return TW_OK;
}

extern "C" int64_t tw_count_pairs_sorted_work_bytes(int32_t n_shards, int64_t max_nz) {
  const RankPlan p = plan_rank(1, std::max<int64_t>(1, max_nz));
  return (int64_t)n_shards * p.chunks * p.C * (int64_t)sizeof(uint64_t);
}

extern "C" int tw_count_pairs_sorted(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                     const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                     int64_t max_nz, int32_t dtype, int32_t pred, void* d_work,
                                     uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0, "tw_count_pairs_sorted: bad sizes");
  TW_ARG_CHECK(pred == TW_PRED_GT || pred == TW_PRED_HALF,
               "tw_count_pairs_sorted: predicate must be TW_PRED_GT or TW_PRED_HALF");
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (max_nx == 0 || max_nz == 0) return TW_OK;
  if (dtype == TW_F64) return launch_rank<double>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, pred, d_work, d_out, st);
  if (dtype == TW_I64) return launch_rank<long long>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, pred, d_work, d_out, st);
  set_error("tw_count_pairs_sorted: unknown dtype %d", dtype);
  return TW_ERR_ARG;
}

// One est.UnNT step with the exact sorted count (the bucket path, shards with nz <= 16384):
// the counts of the current partition into d_out (zero on entry) and the next repartition into
// d_x_next / d_z_next (as tw_permute_pair) with d_out_next zeroed, in one launch — the
// permutation's gathers ride in the count threads (NextBatch).  Elsewhere: the count call,
// tw_permute_pair and a memset in turn.
extern "C" int tw_count_pairs_sorted_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                          const int64_t* d_z_off, int32_t n_shards,
                                          int64_t max_nx, int64_t max_nz, int32_t dtype,
                                          int32_t pred, void* d_work, uint64_t* d_out,
                                          int64_t n_x, void* d_x_next, uint64_t key_x,
                                          int64_t n_z, void* d_z_next, uint64_t key_z,
                                          uint64_t* d_out_next, int32_t n_next_shards,
                                          void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && n_x >= 0 && n_z >= 0 &&
                   n_x < (1ll << 60) && n_z < (1ll << 60) && n_next_shards >= 0,
               "tw_count_pairs_sorted_step: bad sizes");
  TW_ARG_CHECK(pred == TW_PRED_GT || pred == TW_PRED_HALF,
               "tw_count_pairs_sorted_step: predicate must be TW_PRED_GT or TW_PRED_HALF");
  TW_ARG_CHECK(d_x_next == nullptr || ((n_x == 0 || d_x_next != d_x) &&
                                       (n_z == 0 || (d_z_next != nullptr && d_z_next != d_z))),
               "tw_count_pairs_sorted_step: next arrays must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  if (n_shards > 0 && max_nx > 0 && max_nz > 0 && max_nz <= kBucketMaxZ && g_sorted_by_bucket &&
      (dtype == TW_F64 || dtype == TW_I64)) {
    NextStep nxt{};
    if (d_x_next != nullptr)
      nxt = NextStep{(const uint64_t*)d_x, (uint64_t*)d_x_next, n_x, (const uint64_t*)d_z,
                     (uint64_t*)d_z_next, n_z, (unsigned long long*)d_out_next,
                     d_out_next ? (int64_t)n_next_shards : 0,
                     make_feistel(std::max<int64_t>(n_x, 1), key_x),
                     make_feistel(std::max<int64_t>(n_z, 1), key_z), 1, 0, 0};
    else if (d_out_next != nullptr && n_next_shards > 0)
      TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
#define TW_BSTEP(T, P) return launch_bucket_count<T, P>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, d_out, nxt, st)
    if (dtype == TW_F64) {
      if (pred == TW_PRED_HALF) TW_BSTEP(double, TW_PRED_HALF);
      TW_BSTEP(double, TW_PRED_GT);
    }
    if (pred == TW_PRED_HALF) TW_BSTEP(long long, TW_PRED_HALF);
    TW_BSTEP(long long, TW_PRED_GT);
#undef TW_BSTEP
  }
  int rc = tw_count_pairs_sorted(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, dtype,
                                 pred, d_work, d_out, stream);
  if (rc != TW_OK) return rc;
  if (d_x_next != nullptr && n_x + n_z > 0) {
    rc = tw_permute_pair(d_x, d_x_next, n_x, key_x, d_z, d_z_next, n_z, key_z, stream);
    if (rc != TW_OK) return rc;
  }
  if (d_out_next != nullptr && n_next_shards > 0)
    TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
  return TW_OK;
}

// ---- T steps of est.UnNT with the sorted count, the partition kept as records (records.h)
namespace tw {
struct StepsWork {
  uint64_t* xv[2];
  uint64_t* zv[2];
  uint32_t* xp[2];
  uint32_t* zp[2];
  unsigned* cx[2];
  unsigned* cz[2];
  int64_t total;
};

static StepsWork steps_layout(char* w, int64_t n_x, int64_t n_z, int32_t n_shards) {
  StepsWork L{};
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    char* r = w ? w + o : nullptr;
    o += (bytes + 255) / 256 * 256;
    return r;
  };
  for (int k = 0; k < 2; ++k) {
    L.xv[k] = (uint64_t*)take(8 * std::max<int64_t>(n_x, 1));
    L.zv[k] = (uint64_t*)take(8 * std::max<int64_t>(n_z, 1));
    L.xp[k] = (uint32_t*)take(4 * std::max<int64_t>(n_x, 1));
    L.zp[k] = (uint32_t*)take(4 * std::max<int64_t>(n_z, 1));
  }
  char* c0 = w ? w + o : nullptr;
  for (int k = 0; k < 2; ++k) {
    L.cx[k] = (unsigned*)take(4 * ((int64_t)n_shards + 1));
    L.cz[k] = (unsigned*)take(4 * ((int64_t)n_shards + 1));
  }
  (void)c0;
  L.total = o;
  return L;
}

static bool steps_ok(int64_t n_x, int64_t n_z, int32_t n_shards, int64_t max_nz, int32_t dtype,
                     int32_t pred) {
  return n_shards >= 1 && n_shards + 1 <= kBucketNB + 1 && max_nz <= kBucketMaxZ &&
         g_sorted_by_bucket && (dtype == TW_F64 || dtype == TW_I64) &&
         (pred == TW_PRED_GT || pred == TW_PRED_HALF) && n_x >= 1 && n_z >= 1 &&
         n_x < (1ll << 32) && n_z < (1ll << 32);
}
}  // namespace tw

extern "C" int64_t tw_count_pairs_sorted_steps_work_bytes(int64_t n_x, int64_t n_z,
                                                          int32_t n_shards, int64_t max_nz,
                                                          int32_t dtype, int32_t pred) {
  if (!steps_ok(n_x, n_z, n_shards, max_nz, dtype, pred)) return 0;
  return steps_layout(nullptr, n_x, n_z, n_shards).total;
}

extern "C" int tw_count_pairs_sorted_steps(const void* d_x, const void* d_z, int64_t n_x,
                                           int64_t n_z, const int64_t* d_x_off,
                                           const int64_t* d_z_off, int32_t n_shards, int64_t kx,
                                           int64_t kz, int64_t max_nx, int64_t max_nz,
                                           int32_t dtype, int32_t pred, const uint64_t* keys_x,
                                           const uint64_t* keys_z, int32_t T, void* d_work,
                                           int64_t work_bytes, uint64_t* d_out, void* d_x_out,
                                           void* d_z_out, void* stream) {
  TW_ARG_CHECK(T >= 1 && keys_x != nullptr && keys_z != nullptr && kx >= 0 && kz >= 0 &&
                   max_nx >= 0 && max_nz >= 0,
               "tw_count_pairs_sorted_steps: bad sizes");
  TW_ARG_CHECK(steps_ok(n_x, n_z, n_shards, max_nz, dtype, pred),
               "tw_count_pairs_sorted_steps: not applicable (see _work_bytes)");
  const StepsWork W = steps_layout((char*)d_work, n_x, n_z, n_shards);
  TW_ARG_CHECK(d_work != nullptr && work_bytes >= W.total,
               "tw_count_pairs_sorted_steps: work buffer too small");
  TW_ARG_CHECK(d_x_out != d_x && d_z_out != d_z && d_x_out != nullptr && d_z_out != nullptr,
               "tw_count_pairs_sorted_steps: outputs must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * (size_t)T * n_shards, st));
  TW_HIP_CHECK(tw_zero_async(W.cx[0], 0, (char*)d_work + W.total - (char*)W.cx[0], st));
  const FastDiv dx = make_fastdiv((uint64_t)std::max<int64_t>(kx, 1));
  const FastDiv dz = make_fastdiv((uint64_t)std::max<int64_t>(kz, 1));
  auto emit = [&](const uint64_t* xv, const uint32_t* xp, const uint64_t* zv, const uint32_t* zp,
                  int to, unsigned* zx, unsigned* zz, int t) {
    EmitStep e{};
    e.xv = xv; e.xp = xp; e.nx = n_x;
    e.zv = zv; e.zp = zp; e.nz = n_z;
    e.nxv = W.xv[to]; e.nxp = W.xp[to]; e.nzv = W.zv[to]; e.nzp = W.zp[to];
    e.cur_x = W.cx[to]; e.cur_z = W.cz[to];
    e.zero_x = zx; e.zero_z = zz;
    e.fx = make_feistel(n_x, keys_x[t]);
    e.fz = make_feistel(n_z, keys_z[t]);
    e.dx = dx; e.dz = dz; e.kx = kx; e.kz = kz;
    e.x_off = d_x_off; e.z_off = d_z_off; e.n_shards = n_shards; e.active = 1;
    return e;
  };
  // step 0's partition: the arrays (position order) appended to their buckets
  {
    const EmitStep e = emit((const uint64_t*)d_x, nullptr, (const uint64_t*)d_z, nullptr, 0,
                            nullptr, nullptr, 0);
    const int blocks = (int)std::min<int64_t>(1024, ceil_div(n_x + n_z, (int64_t)kSortThreads * 8));
    hipLaunchKernelGGL(k_emit_records, dim3(std::max(blocks, 1)), dim3(kSortThreads), 0, st, e);
    TW_LAUNCH_CHECK();
  }
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    EmitStep e{};
    if (t + 1 < T)
      e = emit(W.xv[cur], W.xp[cur], W.zv[cur], W.zp[cur], nxt, W.cx[cur], W.cz[cur], t + 1);
    int rc;
    if (dtype == TW_F64)
      rc = pred == TW_PRED_HALF
               ? launch_bucket_count<double, TW_PRED_HALF>(W.xv[cur], d_x_off, W.zv[cur], d_z_off, n_shards, max_nx, d_out + (size_t)t * n_shards, NextStep{}, st, e)
               : launch_bucket_count<double, TW_PRED_GT>(W.xv[cur], d_x_off, W.zv[cur], d_z_off, n_shards, max_nx, d_out + (size_t)t * n_shards, NextStep{}, st, e);
    else
      rc = pred == TW_PRED_HALF
               ? launch_bucket_count<long long, TW_PRED_HALF>(W.xv[cur], d_x_off, W.zv[cur], d_z_off, n_shards, max_nx, d_out + (size_t)t * n_shards, NextStep{}, st, e)
               : launch_bucket_count<long long, TW_PRED_GT>(W.xv[cur], d_x_off, W.zv[cur], d_z_off, n_shards, max_nx, d_out + (size_t)t * n_shards, NextStep{}, st, e);
    if (rc != TW_OK) return rc;
  }
  const int last = (T - 1) & 1;
  const int blocks = (int)std::min<int64_t>(4096, ceil_div(n_x + n_z, (int64_t)kBlock));
  hipLaunchKernelGGL(k_records_to_arrays, dim3(blocks), dim3(kBlock), 0, st, W.xv[last],
                     W.xp[last], n_x, W.zv[last], W.zp[last], n_z, (uint64_t*)d_x_out,
                     (uint64_t*)d_z_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int64_t tw_count_pairs_rng_work_bytes(int32_t n_shards, int64_t max_nx,
                                                 int64_t max_nz, int32_t dtype, int32_t pred) {
  if (dtype != TW_F64 && dtype != TW_I64) return 0;
  const RngRankPlan p = plan_rng_ranked(n_shards, max_nx, max_nz, pred, 1);
  return p.ok ? p.total : 0;
}

extern "C" int tw_count_pairs_rng(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                  const int64_t* d_z_off, int32_t n_shards, int64_t B,
                                  uint64_t seed, uint64_t stream_id, int32_t dtype, int32_t pred,
                                  uint64_t* d_out, void* stream);

extern "C" int tw_count_pairs_rng_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                     const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                     int64_t max_nz, int64_t B, uint64_t seed,
                                     uint64_t stream_id, int32_t dtype, int32_t pred,
                                     void* d_work, int64_t work_bytes, uint64_t* d_out,
                                     void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && B >= 0 && max_nx >= 0 && max_nz >= 0,
               "tw_count_pairs_rng_ws: bad sizes");
  if (g_rng_codes_by_bucket == 3 && B > 0 && (dtype == TW_F64 || dtype == TW_I64)) {
    // float32 images in LDS (csrc/imagecount.hip): no codes, no workspace
    const int32_t pr = (pred == TW_PRED_SUBGT && dtype == TW_F64) ? TW_PRED_GT : pred;
    const ImgPlan ip = plan_images(n_shards, max_nx, max_nz, pr, (B + 1) / 2);
    if (ip.ok) {
      hipStream_t st = (hipStream_t)stream;
      TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
      return launch_rng_images(d_x, d_x_off, d_z, d_z_off, n_shards, B, seed, stream_id, dtype,
                               pr, ip, d_out, NextStep{}, st);
    }
  }
  const RngRankPlan p = plan_rng_ranked(n_shards, max_nx, max_nz, pred, B);
  if (!p.ok || (dtype != TW_F64 && dtype != TW_I64) || B == 0 || d_work == nullptr ||
      work_bytes < p.total)  // not applicable: the plain kernel draws the same pairs
    return tw_count_pairs_rng(d_x, d_x_off, d_z, d_z_off, n_shards, B, seed, stream_id, dtype,
                              pred, d_out, stream);
  TW_ARG_CHECK((int64_t)n_shards * p.parts < (1ll << 31) && (int64_t)n_shards * p.tiles < (1ll << 31) &&
                   (int64_t)n_shards * p.chunks < (1ll << 31),
               "tw_count_pairs_rng_ws: grid too large");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (dtype == TW_F64) {
    if (pred == TW_PRED_HALF)
      return launch_rng_ranked<double, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
    return launch_rng_ranked<double, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
  }
  if (pred == TW_PRED_HALF)
    return launch_rng_ranked<long long, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
  return launch_rng_ranked<long long, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
}

// One UnNBT step (compute_stats.py:119-123, device-RNG mode): the counts of the current
// partition into d_out (zero on entry) and the next repartition of both samples into
// d_x_next / d_z_next (as tw_permute_pair) with d_out_next zeroed.  On the float32-image path
// the next repartition's gathers ride in the count threads (csrc/imagecount.hip NextSlice):
// one launch per step.  Elsewhere: the count call, then tw_permute_pair and a memset.
extern "C" int tw_count_pairs_rng_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                       const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                       int64_t max_nz, int64_t B, uint64_t seed,
                                       uint64_t stream_id, int32_t dtype, int32_t pred,
                                       void* d_work, int64_t work_bytes, uint64_t* d_out,
                                       int64_t n_x, void* d_x_next, uint64_t key_x, int64_t n_z,
                                       void* d_z_next, uint64_t key_z, uint64_t* d_out_next,
                                       int32_t n_next_shards, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && B >= 0 && max_nx >= 0 && max_nz >= 0 && n_x >= 0 && n_z >= 0 &&
                   n_x < (1ll << 60) && n_z < (1ll << 60) && n_next_shards >= 0,
               "tw_count_pairs_rng_step: bad sizes");
  TW_ARG_CHECK(d_x_next == nullptr || ((n_x == 0 || d_x_next != d_x) &&
                                       (n_z == 0 || (d_z_next != nullptr && d_z_next != d_z))),
               "tw_count_pairs_rng_step: next arrays must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  if (g_rng_codes_by_bucket == 3 && B > 0 && n_shards > 0 && (dtype == TW_F64 || dtype == TW_I64)) {
    const int32_t pr = (pred == TW_PRED_SUBGT && dtype == TW_F64) ? TW_PRED_GT : pred;
    const ImgPlan ip = plan_images(n_shards, max_nx, max_nz, pr, (B + 1) / 2);
    if (ip.ok) {
      NextStep nxt{};
      if (d_x_next != nullptr)
        nxt = NextStep{(const uint64_t*)d_x, (uint64_t*)d_x_next, n_x, (const uint64_t*)d_z,
                       (uint64_t*)d_z_next, n_z, (unsigned long long*)d_out_next,
                       d_out_next ? (int64_t)n_next_shards : 0,
                       make_feistel(std::max<int64_t>(n_x, 1), key_x),
                       make_feistel(std::max<int64_t>(n_z, 1), key_z), 1, 0, 0};
      else if (d_out_next != nullptr && n_next_shards > 0)
        TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
      return launch_rng_images(d_x, d_x_off, d_z, d_z_off, n_shards, B, seed, stream_id, dtype,
                               pr, ip, d_out, nxt, st);
    }
  }
  int rc = tw_count_pairs_rng_ws(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed,
                                 stream_id, dtype, pred, d_work, work_bytes, d_out, stream);
  if (rc != TW_OK) return rc;
  if (d_x_next != nullptr && n_x + n_z > 0) {
    rc = tw_permute_pair(d_x, d_x_next, n_x, key_x, d_z, d_z_next, n_z, key_z, stream);
    if (rc != TW_OK) return rc;
  }
  if (d_out_next != nullptr && n_next_shards > 0)
    TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
  return TW_OK;
}

extern "C" int tw_count_rng_set_codes(int32_t by_bucket) {
  TW_ARG_CHECK(by_bucket >= 0 && by_bucket <= 3, "tw_count_rng_set_codes: 0, 1, 2 or 3");
  g_rng_codes_by_bucket = by_bucket;
  return TW_OK;
}

extern "C" int tw_count_sorted_set_bucket(int32_t by_bucket) {
  TW_ARG_CHECK(by_bucket >= 0 && by_bucket <= 2, "tw_count_sorted_set_bucket: 0, 1 or 2");
  g_sorted_by_bucket = by_bucket;
  return TW_OK;
}

extern "C" int tw_count_pairs_idx(const void* d_x, const void* d_z, const int64_t* d_ix,
                                  const int64_t* d_iz, const int64_t* d_pair_off,
                                  int32_t n_shards, int64_t max_pairs, int32_t dtype,
                                  int32_t pred, uint64_t* d_out, void* stream);
extern "C" int tw_count_pairs_idx32(const void* d_x, const void* d_z, const int32_t* d_ix,
                                    const int32_t* d_iz, const int64_t* d_pair_off,
                                    int32_t n_shards, int64_t max_pairs, int32_t dtype,
                                    int32_t pred, uint64_t* d_out, void* stream);

static int g_idx_parts = 0;  // tw_count_idx_set_parts: blocks per shard (0 = plan)

extern "C" int tw_count_idx_set_variant(int32_t v) {
  TW_ARG_CHECK(v >= 0 && v <= 5, "tw_count_idx_set_variant: 0..5");
  g_idx_variant = v;
  return TW_OK;
}

extern "C" int tw_count_idx_set_parts(int32_t parts) {
  TW_ARG_CHECK(parts >= 0 && parts <= 4096, "tw_count_idx_set_parts: 0..4096");
  g_idx_parts = parts;
  return TW_OK;
}

namespace tw {
inline int count_idx_plain(const void* x, const void* z, const int64_t* ix, const int64_t* iz,
                           const int64_t* po, int32_t n, int64_t mp, int32_t dt, int32_t pr,
                           uint64_t* out, void* st) {
  return tw_count_pairs_idx(x, z, ix, iz, po, n, mp, dt, pr, out, st);
}
inline int count_idx_plain(const void* x, const void* z, const int32_t* ix, const int32_t* iz,
                           const int64_t* po, int32_t n, int64_t mp, int32_t dt, int32_t pr,
                           uint64_t* out, void* st) {
  return tw_count_pairs_idx32(x, z, ix, iz, po, n, mp, dt, pr, out, st);
}

template <typename I>
int count_idx_ws(const void* d_x, const int64_t* d_x_off, const void* d_z, const int64_t* d_z_off,
                 int32_t n_shards, int64_t max_nx, int64_t max_nz, const I* d_ix, const I* d_iz,
                 const int64_t* d_pair_off, int64_t max_pairs, int32_t dtype, int32_t pred,
                 void* d_work, int64_t work_bytes, uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && max_pairs >= 0,
               "tw_count_pairs_idx_ws: bad sizes");
  // SUBGT on doubles is GT ((x - z) > 0 == x > z without FTZ); on int64 it wraps: plain kernel
  const int32_t pr = (pred == TW_PRED_SUBGT && dtype == TW_F64) ? TW_PRED_GT : pred;
  if (g_rng_codes_by_bucket == 3 && max_pairs > 0 && (dtype == TW_F64 || dtype == TW_I64)) {
    // float32 images in LDS (csrc/imagecount.hip): no codes, no workspace
    const ImgPlan ip = plan_images(n_shards, max_nx, max_nz, pr, max_pairs);
    if (ip.ok) {
      hipStream_t st = (hipStream_t)stream;
      TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
      return launch_idx_images<I>(d_x, d_x_off, d_z, d_z_off, n_shards, d_ix, d_iz, d_pair_off,
                                  dtype, pr, ip, d_out, st);
    }
  }
  // plan_rng_ranked's part count from the pair count (its B), so ~512 blocks fill the chip
  RngRankPlan p = plan_rng_ranked(n_shards, max_nx, max_nz, pr, max_pairs);
  if (g_idx_parts > 0) p.parts = g_idx_parts;
  if (!p.ok || (dtype != TW_F64 && dtype != TW_I64) || max_pairs == 0 || d_work == nullptr ||
      work_bytes < p.total)  // not applicable: the plain kernel gives the same counts
    return count_idx_plain(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, dtype, pred,
                           d_out, stream);
  TW_ARG_CHECK((int64_t)n_shards * p.parts < (1ll << 31) &&
                   (int64_t)n_shards * p.tiles < (1ll << 31) &&
                   (int64_t)n_shards * p.chunks < (1ll << 31) &&
                   (int64_t)n_shards * p.code_parts < (1ll << 31),
               "tw_count_pairs_idx_ws: grid too large");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
#define TW_IR(T, P) return launch_idx_ranked<T, P, I>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz, d_pair_off, p, d_work, d_out, st)
  if (dtype == TW_F64) {
    if (pr == TW_PRED_HALF) TW_IR(double, TW_PRED_HALF);
    TW_IR(double, TW_PRED_GT);
  }
  if (pr == TW_PRED_HALF) TW_IR(long long, TW_PRED_HALF);
  TW_IR(long long, TW_PRED_GT);
#undef TW_IR
}
}  // namespace tw

extern "C" int tw_count_pairs_idx_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                     const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                     int64_t max_nz, const int64_t* d_ix, const int64_t* d_iz,
                                     const int64_t* d_pair_off, int64_t max_pairs, int32_t dtype,
                                     int32_t pred, void* d_work, int64_t work_bytes,
                                     uint64_t* d_out, void* stream) {
  return count_idx_ws<int64_t>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz,
                               d_pair_off, max_pairs, dtype, pred, d_work, work_bytes, d_out,
                               stream);
}

extern "C" int tw_count_pairs_idx32_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                       const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                       int64_t max_nz, const int32_t* d_ix, const int32_t* d_iz,
                                       const int64_t* d_pair_off, int64_t max_pairs,
                                       int32_t dtype, int32_t pred, void* d_work,
                                       int64_t work_bytes, uint64_t* d_out, void* stream) {
  return count_idx_ws<int32_t>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz,
                               d_pair_off, max_pairs, dtype, pred, d_work, work_bytes, d_out,
                               stream);
}
