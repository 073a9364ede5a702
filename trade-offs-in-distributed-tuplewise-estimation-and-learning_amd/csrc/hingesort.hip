// hingesort.hip — the hinge surrogate over ALL pairs of each shard in O((n + m) log m)
// (evaluation_step's tc_AUC, make_exps.py:167-168, and SAME_AS_BATCH's
// bc_AUC, :154-157; cs.conv_AUC, compute_stats.py:129-135):
//     H_s = sum_{i,j} max(S_ij, 0),   S_ij = fl(fl(z_j - x_i) + margin).
// For a fixed x, S is monotone non-decreasing in z, so the pairs with S > 0 are the TOP c_x of
// the shard's sorted z, found by a binary search with the exact floating-point predicate (the
// same pairs the all-pairs kernel adds), and their sum is
//     sum_{top c_x} z_j + c_x * (margin - x)
// from prefix sums of the sorted z.  At 1e6 x 1e6 scores (1e12 pairs) this replaces ~107 ms of
// all-pairs f64 work by a chunk sort, a prefix pass and ~245 binary searches per x.
//
// Accuracy: prefix sums, the per-x terms and every accumulation are double-double (two-sum /
// fma two-product), so the result is the sum of the exact terms (z - x + margin) rounded once
// at the end — within a few ulp of the exact value, i.e. closer to it than NumPy's pairwise sum
// of rounded terms (the reference) or the all-pairs kernel's blocked sum; the three agree to
// ~1e-15 relative.  Pairs whose S rounds to exactly 0 contribute nothing either way.
// Deterministic: fixed scan / reduction orders, no floating-point atomics.
//
// Non-finite scores follow NumPy's elementwise semantics, decided from counts per shard:
// any NaN, or +inf on both sides, or -inf on both sides -> NaN (a NaN term); else +inf z with
// a non-(+inf) x, or -inf x with a non-(-inf) z -> +inf; else the remaining infinities only
// contribute zero terms (x = +inf or z = -inf) and the finite formula holds.
//
// Kernels (workspace from tw_pair_hinge_sum_sorted_work_bytes):
//   k_sort_chunks (sortkeys.h)  z of each shard as sorted order-key chunks of kHsC
//   k_hs_prefix                 per chunk: decoded values (non-finite -> 0), double-double
//                               exclusive prefix sums P[0..C]; z non-finite counts
//   k_hs_sum                    per (shard, x-tile): every chunk staged in LDS (keys + P),
//                               per x the predicate search, the top-c sum, double-double
//                               accumulation, block reduction -> one partial; x counts
//   k_hs_final                  per shard: partials in tile order, the non-finite rules
#include "sortkeys.h"
#include <algorithm>

namespace tw {

constexpr int kHsC = 4096;       // z per sorted chunk: 32 KiB of keys + 64 KiB of P in LDS
constexpr int kHsThreads = 1024;
constexpr int kHsXPer = 4;       // x values per thread
constexpr int kHsCounts = 8;     // per shard: x NaN, x +inf, x -inf, z NaN, z +inf, z -inf

struct ddv {
  double hi, lo;
};
__device__ __forceinline__ ddv two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ ddv quick_two_sum(double a, double b) {
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ ddv dd_add(ddv a, ddv b) {
  ddv s = two_sum(a.hi, b.hi);
  const ddv t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return quick_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ ddv dd_neg(ddv a) { return {-a.hi, -a.lo}; }
// a * c for an exact small integer c (as a double)
__device__ __forceinline__ ddv dd_mul_d(ddv a, double c) {
  const double p = a.hi * c;
  const double e = __fma_rn(a.hi, c, -p);
  return quick_two_sum(p, e + a.lo * c);
}
__device__ __forceinline__ ddv dd_shfl_xor(ddv a, int m) {
  return {__shfl_xor(a.hi, m, kWave), __shfl_xor(a.lo, m, kWave)};
}

__device__ __forceinline__ bool finite_d(double v) { return v - v == 0.0; }

// per chunk: P[k] = sum of the chunk's first k sorted values (non-finite, NaN and padding as 0)
__global__ __launch_bounds__(kHsThreads) void k_hs_prefix(const uint64_t* __restrict__ sorted,
                                                         const int64_t* __restrict__ z_off,
                                                         int chunks, double* __restrict__ P_hi,
                                                         double* __restrict__ P_lo,
                                                         int* __restrict__ counts) {
  constexpr int E = kHsC / kHsThreads;  // 4 values per thread
  __shared__ ddv wtot[kHsThreads / kWave];
  const int s = blockIdx.x / chunks, c = blockIdx.x - s * chunks;
  const int64_t nz = z_off[s + 1] - z_off[s];
  const int valid = (int)std::max<int64_t>(0, std::min<int64_t>(kHsC, nz - (int64_t)c * kHsC));
  const uint64_t* keys = sorted + (int64_t)blockIdx.x * kHsC;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  double v[E];
  int nan = 0, pinf = 0, minf = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = tid * E + e;
    const double z = key_to_double(keys[i]);
    const bool real = i < valid;
    nan += real && z != z;
    pinf += real && z == __longlong_as_double(0x7FF0000000000000ll);
    minf += real && z == -__longlong_as_double(0x7FF0000000000000ll);
    v[e] = (real && finite_d(z)) ? z : 0.0;
  }
  // thread-local inclusive sums, then a block scan of the thread totals (fixed order)
  ddv loc[E];
  ddv run = {0.0, 0.0};
#pragma unroll
  for (int e = 0; e < E; ++e) {
    run = dd_add(run, ddv{v[e], 0.0});
    loc[e] = run;
  }
  ddv inc = run;  // inclusive scan over the wave (Hillis-Steele, fixed order)
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const ddv up = {__shfl_up(inc.hi, o, kWave), __shfl_up(inc.lo, o, kWave)};
    if (lane >= o) inc = dd_add(up, inc);
  }
  if (lane == kWave - 1) wtot[wid] = inc;
  ddv excl_lane = {__shfl_up(inc.hi, 1, kWave), __shfl_up(inc.lo, 1, kWave)};
  if (lane == 0) excl_lane = {0.0, 0.0};
  __syncthreads();
  ddv before = {0.0, 0.0};  // totals of the earlier waves, in wave order
  for (int w = 0; w < wid; ++w) before = dd_add(before, wtot[w]);
  const ddv excl_thread = dd_add(before, excl_lane);
  double* ph = P_hi + (int64_t)blockIdx.x * (kHsC + 1);
  double* pl = P_lo + (int64_t)blockIdx.x * (kHsC + 1);
  if (tid == 0) {
    ph[0] = 0.0;
    pl[0] = 0.0;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const ddv p = dd_add(excl_thread, loc[e]);
    ph[tid * E + e + 1] = p.hi;
    pl[tid * E + e + 1] = p.lo;
  }
  nan = (int)wave_sum_u64((unsigned long long)nan);
  pinf = (int)wave_sum_u64((unsigned long long)pinf);
  minf = (int)wave_sum_u64((unsigned long long)minf);
  if (lane == 0 && (nan | pinf | minf)) {
    if (nan) atomicAdd(counts + s * kHsCounts + 3, nan);
    if (pinf) atomicAdd(counts + s * kHsCounts + 4, pinf);
    if (minf) atomicAdd(counts + s * kHsCounts + 5, minf);
  }
}

__global__ __launch_bounds__(kHsThreads) void k_hs_sum(
    const double* __restrict__ x, const int64_t* __restrict__ x_off,
    const int64_t* __restrict__ z_off, const uint64_t* __restrict__ sorted,
    const double* __restrict__ P_hi, const double* __restrict__ P_lo, int chunks, int tiles_x,
    double margin, double* __restrict__ part, int* __restrict__ counts) {
  __shared__ uint64_t keys[kHsC];
  __shared__ double ph[kHsC + 1], pl[kHsC + 1];
  __shared__ ddv wpart[kHsThreads / kWave];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's x-tiles share one L2
  const int s = lb / tiles_x, t = lb - s * tiles_x;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int64_t xb = x_off[s], xe = x_off[s + 1];
  const int64_t nz = z_off[s + 1] - z_off[s];
  const int64_t x0 = xb + (int64_t)t * (kHsThreads * kHsXPer);
  double xv[kHsXPer];
  bool live[kHsXPer];
  int nan = 0, pinf = 0, minf = 0;
#pragma unroll
  for (int r = 0; r < kHsXPer; ++r) {
    const int64_t i = x0 + r * kHsThreads + tid;
    live[r] = i < xe;
    xv[r] = live[r] ? x[i] : 0.0;
    nan += live[r] && xv[r] != xv[r];
    pinf += live[r] && xv[r] == __longlong_as_double(0x7FF0000000000000ll);
    minf += live[r] && xv[r] == -__longlong_as_double(0x7FF0000000000000ll);
    live[r] = live[r] && finite_d(xv[r]);  // non-finite x: NaN/+inf add no term, -inf -> +inf
  }
  ddv acc = {0.0, 0.0};
  if (x0 < xe) {
    for (int c = 0; c < chunks; ++c) {
      const int valid =
          (int)std::max<int64_t>(0, std::min<int64_t>(kHsC, nz - (int64_t)c * kHsC));
      if (valid == 0) break;  // block-uniform
      const int64_t cb = (int64_t)s * chunks + c;
      __syncthreads();
      for (int i = tid; i < kHsC; i += kHsThreads) keys[i] = sorted[cb * kHsC + i];
      for (int i = tid; i <= kHsC; i += kHsThreads) {
        ph[i] = P_hi[cb * (kHsC + 1) + i];
        pl[i] = P_lo[cb * (kHsC + 1) + i];
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kHsXPer; ++r) {
        if (!live[r]) continue;
        // first index f in [0, valid) with S = fl(fl(z - x) + margin) > 0 (S is monotone in z)
        int f = 0;
        for (int st = kHsC >> 1; st > 0; st >>= 1) {
          const int idx = f + st - 1;
          if (idx < valid) {
            const double z = key_to_double(keys[idx]);
            if (!((z - xv[r]) + margin > 0.0)) f += st;
          }
        }
        if (f < valid) {
          const double z = key_to_double(keys[f]);
          if (!((z - xv[r]) + margin > 0.0)) ++f;
        }
        const int cnt = valid - f;
        if (cnt > 0) {  // sum of the top cnt z + cnt * (margin - x), double-double
          const ddv top = dd_add(ddv{ph[valid], pl[valid]}, dd_neg(ddv{ph[f], pl[f]}));
          const ddv mxd = two_sum(margin, -xv[r]);
          acc = dd_add(acc, dd_add(top, dd_mul_d(mxd, (double)cnt)));
        }
      }
    }
  }
  // block reduction in a fixed order: butterfly in the wave, then the waves in order
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) acc = dd_add(acc, dd_shfl_xor(acc, o));
  if (lane == 0) wpart[wid] = acc;
  nan = (int)wave_sum_u64((unsigned long long)nan);
  pinf = (int)wave_sum_u64((unsigned long long)pinf);
  minf = (int)wave_sum_u64((unsigned long long)minf);
  if (lane == 0 && (nan | pinf | minf)) {
    if (nan) atomicAdd(counts + s * kHsCounts + 0, nan);
    if (pinf) atomicAdd(counts + s * kHsCounts + 1, pinf);
    if (minf) atomicAdd(counts + s * kHsCounts + 2, minf);
  }
  __syncthreads();
  if (tid == 0) {
    ddv b = {0.0, 0.0};
    for (int w = 0; w < kHsThreads / kWave; ++w) b = dd_add(b, wpart[w]);
    part[((int64_t)s * tiles_x + t) * 2] = b.hi;
    part[((int64_t)s * tiles_x + t) * 2 + 1] = b.lo;
  }
}

__global__ __launch_bounds__(kBlock) void k_hs_final(const double* __restrict__ part,
                                                    const int* __restrict__ counts,
                                                    const int64_t* __restrict__ x_off,
                                                    const int64_t* __restrict__ z_off,
                                                    int n_shards, int tiles_x,
                                                    double* __restrict__ out) {
  const int s = blockIdx.x * kBlock + threadIdx.x;
  if (s >= n_shards) return;
  const int64_t nx = x_off[s + 1] - x_off[s], nz = z_off[s + 1] - z_off[s];
  ddv b = {0.0, 0.0};
  for (int t = 0; t < tiles_x; ++t)
    b = dd_add(b, ddv{part[((int64_t)s * tiles_x + t) * 2], part[((int64_t)s * tiles_x + t) * 2 + 1]});
  const int* k = counts + s * kHsCounts;
  const double inf = __longlong_as_double(0x7FF0000000000000ll);
  double r = b.hi + b.lo;
  if (nx == 0 || nz == 0)
    r = 0.0;
  else if (k[0] || k[3] || (k[1] && k[4]) || (k[2] && k[5]))
    r = __longlong_as_double(0x7FF8000000000000ll);  // a NaN term
  else if ((k[4] && nx - k[1] > 0) || (k[2] && nz - k[5] > 0))
    r = inf;  // an infinite term
  out[s] = r;
}

struct HsPlan {
  int chunks, tiles_x;
  int64_t keys, P, part, counts;  // workspace byte offsets
  int64_t bytes;
};

static HsPlan plan_hs(int32_t n_shards, int64_t max_nx, int64_t max_nz) {
  HsPlan p{};
  p.chunks = (int)std::max<int64_t>(1, ceil_div(max_nz, kHsC));
  p.tiles_x = (int)std::max<int64_t>(1, ceil_div(max_nx, (int64_t)kHsThreads * kHsXPer));
  const int64_t nc = (int64_t)n_shards * p.chunks;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  p.keys = 0;
  p.P = al(nc * kHsC * 8);
  p.part = p.P + al(2 * nc * (kHsC + 1) * 8);
  p.counts = p.part + al((int64_t)n_shards * p.tiles_x * 16);
  p.bytes = p.counts + al((int64_t)n_shards * kHsCounts * 4);
  return p;
}

}  // namespace tw

using namespace tw;

extern "C" int64_t tw_pair_hinge_sum_sorted_work_bytes(int32_t n_shards, int64_t max_nx,
                                                       int64_t max_nz) {
  if (n_shards <= 0 || max_nx < 0 || max_nz < 0) return 0;
  return plan_hs(n_shards, max_nx, max_nz).bytes;
}

extern "C" int tw_pair_hinge_sum_sorted(const double* d_x, const int64_t* d_x_off,
                                        const double* d_z, const int64_t* d_z_off,
                                        int32_t n_shards, int64_t max_nx, int64_t max_nz,
                                        double margin, void* d_work, double* d_out,
                                        void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && d_work != nullptr,
               "tw_pair_hinge_sum_sorted: bad arguments");
  TW_ARG_CHECK(max_nz < (1ll << 31) && max_nx < (1ll << 40),
               "tw_pair_hinge_sum_sorted: shard too large");
  if (n_shards == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  const HsPlan p = plan_hs(n_shards, max_nx, max_nz);
  char* w = (char*)d_work;
  uint64_t* keys = (uint64_t*)(w + p.keys);
  double* P_hi = (double*)(w + p.P);
  double* P_lo = P_hi + (int64_t)n_shards * p.chunks * (kHsC + 1);
  double* part = (double*)(w + p.part);
  int* counts = (int*)(w + p.counts);
  TW_HIP_CHECK(tw_zero_async(counts, 0, (size_t)n_shards * kHsCounts * 4, st));
  static bool attr = false;
  if (!attr) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_sort_chunks<double, 4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kHsC * 8));
    attr = true;
  }
  const int64_t nc = (int64_t)n_shards * p.chunks;
  TW_ARG_CHECK(nc < (1ll << 31) && (int64_t)n_shards * p.tiles_x < (1ll << 31),
               "tw_pair_hinge_sum_sorted: too many blocks");
  hipLaunchKernelGGL((k_sort_chunks<double, 4>), dim3((unsigned)nc), dim3(kHsC / 4),
                     (size_t)kHsC * 8, st, d_z, d_z_off, p.chunks, kHsC, keys, (int64_t)0);
  hipLaunchKernelGGL(k_hs_prefix, dim3((unsigned)nc), dim3(kHsThreads), 0, st, keys, d_z_off,
                     p.chunks, P_hi, P_lo, counts);
  hipLaunchKernelGGL(k_hs_sum, dim3((unsigned)(n_shards * p.tiles_x)), dim3(kHsThreads), 0, st,
                     d_x, d_x_off, d_z_off, keys, P_hi, P_lo, p.chunks, p.tiles_x, margin, part,
                     counts);
  hipLaunchKernelGGL(k_hs_final, dim3((unsigned)ceil_div(n_shards, kBlock)), dim3(kBlock), 0, st,
                     part, counts, d_x_off, d_z_off, (int)n_shards, p.tiles_x, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
