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
#include <algorithm>
#include <type_traits>

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
// into LDS, buckets it by VALUE — b(v) = clamp(int((v - zmin) * NB / (zmax - zmin)), 0, NB-1)
// over the finite z, a monotone map (every IEEE step in it is monotone), so bucket order is
// value order — with an LDS histogram, prefix sum and scatter, and then a code is
//   (#z in lower buckets) + (#z in its own bucket below / at most v)
// by a scan of one bucket (~nz / NB values for smooth data).  Exact for any data: ties share
// a bucket; NaN z sit in no bucket (their p is the count of non-NaN z, above every x code),
// NaN x get code 0, +-inf clamp to the end buckets; degenerate or very skewed data only make
// the scans longer.  Every block of a shard rebuilds the buckets (O(nz) LDS work) and codes
// its share of the shard's x and z.  Replaces k_sort_chunks + k_rank_codes (41 + 78 us at
// the bench shape).
constexpr int kBucketNB = 2048;
constexpr int64_t kBucketMaxZ = 16384;  // 128 KiB of z in LDS
constexpr int kBucketParts = 4;

template <typename T>
__device__ __forceinline__ double bucket_value(T v) { return (double)v; }

// COUNT = true: the complete count instead of codes (tw_count_pairs_sorted): the same
// buckets, only the x-values, and the block's sum of their codes (#z < x, plus #z <= x for
// half-ties) added to out[s] — the integer of k_count_complete / k_rank_count.
template <typename T, int PRED, bool COUNT = false>
__global__ __launch_bounds__(kSortThreads) void k_rank_codes_bucket(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, int parts, int64_t max_nx, int64_t max_nz,
    uint16_t* __restrict__ cx, uint16_t* __restrict__ cx2, uint16_t* __restrict__ pz,
    unsigned long long* __restrict__ out = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* zb = (T*)smem;                                       // z by bucket (kBucketMaxZ)
  unsigned* start = (unsigned*)(smem + sizeof(T) * kBucketMaxZ);  // NB + 1 bucket starts
  unsigned* cur = start + kBucketNB + 1;                  // NB fill cursors / counts
  __shared__ double red_min[kSortThreads / kWave], red_max[kSortThreads / kWave];
  __shared__ unsigned nan_z;
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t xb = x_off[s], nx = x_off[s + 1] - xb;
  const int64_t zo = z_off[s], nz = z_off[s + 1] - zo;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  // 1. range of the finite z
  double mn = __builtin_inf(), mx = -__builtin_inf();
  for (int64_t j = tid; j < nz; j += kSortThreads) {
    const double v = bucket_value<T>(z[zo + j]);
    if (v - v == 0.0) {  // finite (not NaN, not inf)
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
  mn = red_min[0];
  mx = red_max[0];
  for (int w = 1; w < kSortThreads / kWave; ++w) {
    mn = red_min[w] < mn ? red_min[w] : mn;
    mx = red_max[w] > mx ? red_max[w] : mx;
  }
  const double scale = mx > mn ? (double)kBucketNB / (mx - mn) : 0.0;
  auto bucket = [&](double v) -> int {
    const double t = (v - mn) * scale;  // NaN when v == mn and scale == inf: bucket 0
    return (int)__builtin_fmin(__builtin_fmax(t, 0.0), (double)(kBucketNB - 1));
  };
  // 2. histogram (NaN z counted apart)
  for (int64_t j = tid; j < nz; j += kSortThreads) {
    const T v = z[zo + j];
    if (is_nan_score<T>(v)) atomicAdd(&nan_z, 1u);
    else atomicAdd(&cur[bucket(bucket_value<T>(v))], 1u);
  }
  __syncthreads();
  // 3. exclusive prefix over NB buckets (two per thread, then a block scan of the pairs)
  {
    const int i0 = 2 * tid;  // kBucketNB == 2 * kSortThreads
    const unsigned a = cur[i0], b = cur[i0 + 1];
    unsigned v = a + b;
    for (int o = 1; o < kWave; o <<= 1) {  // inclusive wave scan
      const unsigned t = __shfl_up(v, o, kWave);
      if (lane >= o) v += t;
    }
    __shared__ unsigned wave_tot[kSortThreads / kWave];
    if (lane == kWave - 1) wave_tot[wid] = v;
    __syncthreads();
    unsigned base = 0;
    for (int w = 0; w < wid; ++w) base += wave_tot[w];
    const unsigned excl = base + v - (a + b);
    start[i0] = excl;
    start[i0 + 1] = excl + a;
    if (tid == kSortThreads - 1) start[kBucketNB] = excl + a + b;
    __syncthreads();
    cur[i0] = excl;
    cur[i0 + 1] = excl + a;
  }
  __syncthreads();
  // 4. scatter z into bucket order
  for (int64_t j = tid; j < nz; j += kSortThreads) {
    const T v = z[zo + j];
    if (!is_nan_score<T>(v)) zb[atomicAdd(&cur[bucket(bucket_value<T>(v))], 1u)] = v;
  }
  __syncthreads();
  const unsigned n_valid = start[kBucketNB];
  // 5. codes of this block's share of the shard's x and z (COUNT: of its x only)
  const int64_t tot = COUNT ? nx : nx + nz, per = (tot + parts - 1) / parts;
  const int64_t e0 = (int64_t)part * per, e1 = e0 + per < tot ? e0 + per : tot;
  unsigned long long acc = 0;
  for (int64_t e = e0 + tid; e < e1; e += kSortThreads) {
    const bool isx = e < nx;
    const T v = isx ? x[xb + e] : z[zo + (e - nx)];
    unsigned lo = 0, hi = 0;
    if (is_nan_score<T>(v)) {
      lo = isx ? 0u : n_valid;  // NaN x: below every p; NaN z: above every c
      hi = lo;
    } else {
      const int b = bucket(bucket_value<T>(v));
      const unsigned b0 = start[b], b1 = start[b + 1];
      lo = b0;
      hi = b0;
      for (unsigned q = b0; q < b1; ++q) {
        const T w = zb[q];
        lo += w < v;
        hi += w <= v;
      }
    }
    if constexpr (COUNT) {
      acc += lo + (PRED == TW_PRED_HALF ? hi : 0u);
    } else if (isx) {
      cx[(int64_t)s * max_nx + e] = (uint16_t)lo;
      if (PRED == TW_PRED_HALF) cx2[(int64_t)s * max_nx + e] = (uint16_t)hi;
    } else {
      pz[(int64_t)s * max_nz + (e - nx)] = (uint16_t)lo;
    }
  }
  if constexpr (COUNT) {
    acc = wave_sum_u64(acc);
    __shared__ unsigned long long part_acc[kSortThreads / kWave];
    if (lane == 0) part_acc[wid] = acc;
    __syncthreads();
    if (tid == 0) {
      unsigned long long b = 0;
      for (int w = 0; w < kSortThreads / kWave; ++w) b += part_acc[w];
      if (b) atomicAdd(out + s, b);
    }
  }
}

static int g_sorted_by_bucket = 1;  // tw_count_sorted_set_bucket: 0 = sort + binary search

template <typename T, int PRED>
int launch_bucket_count(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                        int32_t n_shards, int64_t max_nx, uint64_t* out, hipStream_t st) {
  const size_t lds_b = sizeof(T) * kBucketMaxZ + sizeof(unsigned) * (2 * kBucketNB + 1);
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
                     max_nx, (int64_t)0, nullptr, nullptr, nullptr, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T>
int launch_rank(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                int32_t n_shards, int64_t max_nx, int64_t max_nz, int32_t pred, void* work,
                uint64_t* out, hipStream_t st) {
  if (max_nz <= kBucketMaxZ && g_sorted_by_bucket) {
    if (pred == TW_PRED_HALF)
      return launch_bucket_count<T, TW_PRED_HALF>(x, x_off, z, z_off, n_shards, max_nx, out, st);
    return launch_bucket_count<T, TW_PRED_GT>(x, x_off, z, z_off, n_shards, max_nx, out, st);
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

template <int PRED>
__global__ __launch_bounds__(kRngThreads) void k_count_rng_ranked(
    const int64_t* __restrict__ x_off, const int64_t* __restrict__ z_off,
    const uint16_t* __restrict__ cx, const uint16_t* __restrict__ cx2,
    const uint16_t* __restrict__ pz, int64_t max_nx, int64_t max_nz, int64_t B, int parts,
    uint32_t k0, uint32_t k1, uint32_t sid, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint16_t codes[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's parts share one L2
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t nx = x_off[s + 1] - x_off[s], nz = z_off[s + 1] - z_off[s];
  unsigned acc = 0;
  if (nx > 0 && nz > 0) {
    uint16_t* lx = codes;
    uint16_t* lx2 = codes + nx;
    uint16_t* lz = codes + (PRED == TW_PRED_HALF ? 2 : 1) * nx;
    for (int64_t i = threadIdx.x; i < nx; i += kRngThreads) {
      lx[i] = cx[(int64_t)s * max_nx + i];
      if (PRED == TW_PRED_HALF) lx2[i] = cx2[(int64_t)s * max_nx + i];
    }
    for (int64_t j = threadIdx.x; j < nz; j += kRngThreads) lz[j] = pz[(int64_t)s * max_nz + j];
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

// Incomplete count on explicit index pairs (UB replay: NumPy's randint draws, compute_stats.py:
// 22-42) through the rank codes: a block stages its shard's 16-bit codes in LDS, so the two
// per-pair gathers are LDS reads and only the 16 B of indices per pair stream from HBM (the plain
// k_count_idx pulls an L2 line per gathered score).  Indices are absolute; one outside its
// shard's range (allowed by tw_count_pairs_idx) compares the scores themselves.
template <typename T, int PRED>
__global__ __launch_bounds__(kRngThreads) void k_count_idx_ranked(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, const uint16_t* __restrict__ cx,
    const uint16_t* __restrict__ cx2, const uint16_t* __restrict__ pz, int64_t max_nx,
    int64_t max_nz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz,
    const int64_t* __restrict__ pair_off, int parts, unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint16_t codes[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's parts share one L2
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t xb = x_off[s], zb = z_off[s];
  const uint64_t nx = (uint64_t)(x_off[s + 1] - xb), nz = (uint64_t)(z_off[s + 1] - zb);
  uint16_t* lx = codes;
  uint16_t* lx2 = codes + nx;
  uint16_t* lz = codes + (PRED == TW_PRED_HALF ? 2 : 1) * nx;
  if (nx > 0 && nz > 0) {
    for (int64_t i = threadIdx.x; i < (int64_t)nx; i += kRngThreads) {
      lx[i] = cx[(int64_t)s * max_nx + i];
      if (PRED == TW_PRED_HALF) lx2[i] = cx2[(int64_t)s * max_nx + i];
    }
    for (int64_t j = threadIdx.x; j < (int64_t)nz; j += kRngThreads)
      lz[j] = pz[(int64_t)s * max_nz + j];
  }
  __syncthreads();
  const int64_t pb = pair_off[s], pe = pair_off[s + 1];
  const int64_t per = (pe - pb + parts - 1) / parts;
  const int64_t q0 = pb + (int64_t)part * per;
  const int64_t q1 = std::min<int64_t>(pe, q0 + per);
  unsigned acc = 0;
  constexpr int U = 4;  // index loads in flight per thread
  for (int64_t p0 = q0 + threadIdx.x; p0 < q1; p0 += (int64_t)U * kRngThreads) {
    int64_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = p0 + (int64_t)u * kRngThreads;
      a[u] = p < q1 ? ix[p] : xb;
      b[u] = p < q1 ? iz[p] : zb;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p0 + (int64_t)u * kRngThreads >= q1) break;
      const uint64_t i = (uint64_t)(a[u] - xb), j = (uint64_t)(b[u] - zb);
      if (i < nx && j < nz) {
        const unsigned pj = lz[j];
        acc += (unsigned)lx[i] > pj;
        if (PRED == TW_PRED_HALF) acc += (unsigned)lx2[i] > pj;
      } else {
        const T xv = x[a[u]], zv = z[b[u]];
        acc += xv > zv;
        if (PRED == TW_PRED_HALF) acc += xv >= zv;
      }
    }
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kRngThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long sum = 0;
    for (int w = 0; w < kRngThreads / kWave; ++w) sum += part_sum[w];
    if (sum) atomicAdd(out + s, sum);
  }
}

static int g_rng_codes_by_bucket = 1;  // tw_count_rng_set_codes: 0 = sort + binary search

struct RngRankPlan {
  bool ok;
  int C, chunks, tiles, parts;
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
  p.lds = (size_t)(nc * max_nx + max_nz) * sizeof(uint16_t);
  p.ok = p.lds <= 160 * 1024 - 1024;
  // ~2 blocks of 1024 threads per CU over the whole grid, >= 8192 draws per block
  const int64_t nq = std::max<int64_t>(1, (B + 1) / 2);
  p.parts = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(512, n_shards),
                                                        ceil_div(nq, 8192)));
  auto al = [](int64_t b) { return ceil_div(b, 256) * 256; };
  p.keys_bytes = al((int64_t)n_shards * p.chunks * p.C * 8);
  p.cx_off = p.keys_bytes;
  p.cx2_off = p.cx_off + al((int64_t)n_shards * max_nx * 2);
  p.pz_off = p.cx2_off + (pred == TW_PRED_HALF ? al((int64_t)n_shards * max_nx * 2) : 0);
  p.total = p.pz_off + al((int64_t)n_shards * max_nz * 2);
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
                                     (int)(sizeof(T) * kBucketMaxZ +
                                           sizeof(unsigned) * (2 * kBucketNB + 1))));
    attrs_set = true;
  }
  char* w = (char*)work;
  uint64_t* keys = (uint64_t*)w;
  uint16_t* cx = (uint16_t*)(w + p.cx_off);
  uint16_t* cx2 = (uint16_t*)(w + p.cx2_off);
  uint16_t* pz = (uint16_t*)(w + p.pz_off);
  if (max_nz <= kBucketMaxZ && g_rng_codes_by_bucket) {
    const size_t lds_b = sizeof(T) * kBucketMaxZ + sizeof(unsigned) * (2 * kBucketNB + 1);
    hipLaunchKernelGGL((k_rank_codes_bucket<T, PRED>), dim3(n_shards * kBucketParts),
                       dim3(kSortThreads), lds_b, st, (const T*)x, x_off, (const T*)z, z_off,
                       kBucketParts, max_nx, max_nz, cx, cx2, pz);
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
                     p.tiles, max_nx, max_nz, cx, cx2, pz);
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
                     p.lds, st, x_off, z_off, cx, cx2, pz, max_nx, max_nz, B, p.parts,
                     (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)sid,
                     (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T, int PRED>
int launch_idx_ranked(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, int64_t max_nx, int64_t max_nz, const int64_t* ix,
                      const int64_t* iz, const int64_t* pair_off, const RngRankPlan& p,
                      void* work, uint64_t* out, hipStream_t st) {
  static bool attrs_set = false;
  if (!attrs_set) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_count_idx_ranked<T, PRED>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - 1024));
    attrs_set = true;
  }
  const int rc = launch_codes<T, PRED>(x, x_off, z, z_off, n_shards, max_nx, max_nz, p, work, st);
  if (rc != TW_OK) return rc;
  char* w = (char*)work;
  hipLaunchKernelGGL((k_count_idx_ranked<T, PRED>), dim3(n_shards * p.parts), dim3(kRngThreads),
                     p.lds, st, (const T*)x, x_off, (const T*)z, z_off,
                     (const uint16_t*)(w + p.cx_off), (const uint16_t*)(w + p.cx2_off),
                     (const uint16_t*)(w + p.pz_off), max_nx, max_nz, ix, iz, pair_off, p.parts,
                     (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

}  // namespace tw

using namespace tw;

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
  TW_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (max_nx == 0 || max_nz == 0) return TW_OK;
  if (dtype == TW_F64) return launch_rank<double>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, pred, d_work, d_out, st);
  if (dtype == TW_I64) return launch_rank<long long>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, pred, d_work, d_out, st);
  set_error("tw_count_pairs_sorted: unknown dtype %d", dtype);
  return TW_ERR_ARG;
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
  const RngRankPlan p = plan_rng_ranked(n_shards, max_nx, max_nz, pred, B);
  if (!p.ok || (dtype != TW_F64 && dtype != TW_I64) || B == 0 || d_work == nullptr ||
      work_bytes < p.total)  // not applicable: the plain kernel draws the same pairs
    return tw_count_pairs_rng(d_x, d_x_off, d_z, d_z_off, n_shards, B, seed, stream_id, dtype,
                              pred, d_out, stream);
  TW_ARG_CHECK((int64_t)n_shards * p.parts < (1ll << 31) && (int64_t)n_shards * p.tiles < (1ll << 31) &&
                   (int64_t)n_shards * p.chunks < (1ll << 31),
               "tw_count_pairs_rng_ws: grid too large");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (dtype == TW_F64) {
    if (pred == TW_PRED_HALF)
      return launch_rng_ranked<double, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
    return launch_rng_ranked<double, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
  }
  if (pred == TW_PRED_HALF)
    return launch_rng_ranked<long long, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
  return launch_rng_ranked<long long, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, B, seed, stream_id, p, d_work, d_out, st);
}

extern "C" int tw_count_rng_set_codes(int32_t by_bucket) {
  TW_ARG_CHECK(by_bucket == 0 || by_bucket == 1, "tw_count_rng_set_codes: 0 or 1");
  g_rng_codes_by_bucket = by_bucket;
  return TW_OK;
}

extern "C" int tw_count_sorted_set_bucket(int32_t by_bucket) {
  TW_ARG_CHECK(by_bucket == 0 || by_bucket == 1, "tw_count_sorted_set_bucket: 0 or 1");
  g_sorted_by_bucket = by_bucket;
  return TW_OK;
}

extern "C" int tw_count_pairs_idx(const void* d_x, const void* d_z, const int64_t* d_ix,
                                  const int64_t* d_iz, const int64_t* d_pair_off,
                                  int32_t n_shards, int64_t max_pairs, int32_t dtype,
                                  int32_t pred, uint64_t* d_out, void* stream);

static int g_idx_parts = 0;  // tw_count_idx_set_parts: blocks per shard (0 = plan)

extern "C" int tw_count_idx_set_parts(int32_t parts) {
  TW_ARG_CHECK(parts >= 0 && parts <= 4096, "tw_count_idx_set_parts: 0..4096");
  g_idx_parts = parts;
  return TW_OK;
}

extern "C" int tw_count_pairs_idx_ws(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                     const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                     int64_t max_nz, const int64_t* d_ix, const int64_t* d_iz,
                                     const int64_t* d_pair_off, int64_t max_pairs, int32_t dtype,
                                     int32_t pred, void* d_work, int64_t work_bytes,
                                     uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && max_pairs >= 0,
               "tw_count_pairs_idx_ws: bad sizes");
  // SUBGT on doubles is GT ((x - z) > 0 == x > z without FTZ); on int64 it wraps: plain kernel
  const int32_t pr = (pred == TW_PRED_SUBGT && dtype == TW_F64) ? TW_PRED_GT : pred;
  // plan_rng_ranked's part count from the pair count (its B), so ~512 blocks fill the chip
  RngRankPlan p = plan_rng_ranked(n_shards, max_nx, max_nz, pr, max_pairs);
  if (g_idx_parts > 0) p.parts = g_idx_parts;
  if (!p.ok || (dtype != TW_F64 && dtype != TW_I64) || max_pairs == 0 || d_work == nullptr ||
      work_bytes < p.total)  // not applicable: the plain kernel gives the same counts
    return tw_count_pairs_idx(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, dtype,
                              pred, d_out, stream);
  TW_ARG_CHECK((int64_t)n_shards * p.parts < (1ll << 31) && (int64_t)n_shards * p.tiles < (1ll << 31) &&
                   (int64_t)n_shards * p.chunks < (1ll << 31),
               "tw_count_pairs_idx_ws: grid too large");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (dtype == TW_F64) {
    if (pr == TW_PRED_HALF)
      return launch_idx_ranked<double, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz, d_pair_off, p, d_work, d_out, st);
    return launch_idx_ranked<double, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz, d_pair_off, p, d_work, d_out, st);
  }
  if (pr == TW_PRED_HALF)
    return launch_idx_ranked<long long, TW_PRED_HALF>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz, d_pair_off, p, d_work, d_out, st);
  return launch_idx_ranked<long long, TW_PRED_GT>(d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_ix, d_iz, d_pair_off, p, d_work, d_out, st);
}
