// pairsum.hip — float-valued pair kernels (SURVEY.md §8 row A2 prod/gini, row f1 conv_AUC;
// the logistic surrogate is the row-L3 extension).
//
//   cs.Un(kernel="prod")   compute_stats.py:15-16   mean(X_col.dot(Z_row))
//   cs.Un(kernel="gini")   compute_stats.py:17-18   mean(|X_col - Z_row|)
//   conv_AUC(margin)       compute_stats.py:129-135 mean(max(Z_row - X_col + margin, 0))
//   UB_indices prod/gini   compute_stats.py:26-29 ; conv_AUC_deter_pairs compute_stats.py:137-144
// NumPy reduces these with pairwise summation; the parity bar is a relative tolerance
// (tests/test_pairsum.py), not bits.  Sums here are deterministic: each block writes one
// partial in a fixed lane/wave order and a second kernel adds a shard's partials in order.
#include "tw_common.h"
#include <algorithm>

namespace tw {

template <int K>
__device__ __forceinline__ double fkern(double x, double z, double margin) {
  if constexpr (K == TW_KERN_PROD) return x * z;
  else if constexpr (K == TW_KERN_GINI) return fabs(x - z);
  else if constexpr (K == TW_KERN_HINGE) {  // np.maximum(t, 0): a NaN t stays NaN (not fmax)
    const double t = z - x + margin;
    return !(t <= 0.0) ? t : 0.0;
  }
  else {  // TW_KERN_LOGISTIC: softplus as NumPy's logaddexp(0, t) evaluates it
    const double t = z - x + margin;
    return t == 0.0 ? 0.6931471805599453 : fmax(t, 0.0) + log1p(exp(-fabs(t)));
  }
}

constexpr int kSumR = 4;           // x-values per lane
constexpr int64_t kSumZChunk = 2048;

struct SumPlan {
  int tiles_x, zchunks;
};
inline SumPlan plan_sum(int64_t max_nx, int64_t max_nz) {
  SumPlan p;
  p.tiles_x = (int)std::max<int64_t>(1, ceil_div(max_nx, (int64_t)kBlock * kSumR));
  p.zchunks = (int)std::max<int64_t>(1, ceil_div(max_nz, kSumZChunk));
  return p;
}

__device__ __forceinline__ double block_sum_f64(double v) {
  v = wave_sum_f64(v);
  __shared__ double part[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part[wid] = v;
  __syncthreads();
  double b = 0.0;
  if (threadIdx.x == 0) b = (part[0] + part[1]) + (part[2] + part[3]);
  return b;
}

// bit 0: NaN, bit 1: +inf, bit 2: -inf
__device__ __forceinline__ int nonfinite_bits(double v) {
  const double inf = __longlong_as_double(0x7FF0000000000000ll);
  return (v != v ? 1 : 0) | (v == inf ? 2 : 0) | (v == -inf ? 4 : 0);
}

// The all-pairs block sums the hinge with fmax (one v_max_f64 per pair; it drops NaN terms)
// and restores NumPy's NaN afterwards: a pair's t = fl(z - x) + margin is NaN iff x or z is
// NaN or both are infinite with the same sign, so the block's (x tile, z chunk) holds a NaN
// term iff its non-finite bits say so.
template <int K>
__device__ __forceinline__ double fkern_loop(double x, double z, double margin) {
  if constexpr (K == TW_KERN_HINGE) return fmax(z - x + margin, 0.0);
  else return fkern<K>(x, z, margin);
}

template <int K>
__global__ __launch_bounds__(kBlock) void k_pair_sum(const double* __restrict__ x,
                                                     const int64_t* __restrict__ x_off,
                                                     const double* __restrict__ z,
                                                     const int64_t* __restrict__ z_off,
                                                     int tiles_x, int zchunks, double margin,
                                                     double* __restrict__ work) {
  const int per_shard = tiles_x * zchunks;
  const int s = blockIdx.x / per_shard;
  const int rem = blockIdx.x - s * per_shard;
  const int cz = rem / tiles_x;
  const int tx = rem - cz * tiles_x;
  const int64_t xb = x_off[s], xe = x_off[s + 1];
  const int64_t zb = z_off[s], ze = z_off[s + 1];
  const int64_t x0 = xb + (int64_t)tx * (kBlock * kSumR);
  const int64_t z0 = zb + (int64_t)cz * kSumZChunk;
  if (x0 >= xe || z0 >= ze) {  // block-uniform; the slot must still be written
    if (threadIdx.x == 0) work[blockIdx.x] = 0.0;
    return;
  }
  const int64_t z1 = std::min(ze, z0 + kSumZChunk);
  double xv[kSumR], acc[kSumR];
  bool valid[kSumR];
#pragma unroll
  for (int r = 0; r < kSumR; ++r) {
    const int64_t i = x0 + r * kBlock + threadIdx.x;
    valid[r] = i < xe;
    xv[r] = valid[r] ? x[i] : 0.0;
    acc[r] = 0.0;
  }
  const double* __restrict__ zp = z + z0;
  const int nz = (int)(z1 - z0);
#pragma unroll 4
  for (int j = 0; j < nz; ++j) {
    const double zv = zp[j];
#pragma unroll
    for (int r = 0; r < kSumR; ++r) acc[r] += fkern_loop<K>(xv[r], zv, margin);
  }
  double t = 0.0;
#pragma unroll
  for (int r = 0; r < kSumR; ++r) t += valid[r] ? acc[r] : 0.0;
  int xbits = 0, zbits = 0;
  if constexpr (K == TW_KERN_HINGE) {
#pragma unroll
    for (int r = 0; r < kSumR; ++r) xbits |= valid[r] ? nonfinite_bits(xv[r]) : 0;
    for (int j = threadIdx.x; j < nz; j += kBlock) zbits |= nonfinite_bits(zp[j]);
  }
  const double b = block_sum_f64(t);
  if constexpr (K == TW_KERN_HINGE) {
    xbits = __syncthreads_or(xbits & 1) | (__syncthreads_or(xbits & 2) ? 2 : 0) |
            (__syncthreads_or(xbits & 4) ? 4 : 0);
    zbits = __syncthreads_or(zbits & 1) | (__syncthreads_or(zbits & 2) ? 2 : 0) |
            (__syncthreads_or(zbits & 4) ? 4 : 0);
    if (threadIdx.x == 0)
      work[blockIdx.x] = ((xbits | zbits) & 1) || (xbits & zbits & 6)
                             ? __longlong_as_double(0x7FF8000000000000ll)
                             : b;
  } else {
    if (threadIdx.x == 0) work[blockIdx.x] = b;
  }
}

// I: int64_t or int32_t indices.  COUNT: the same pass also counts x > z per shard into
// count[s] (evaluation_step's br_AUC = UB_pairs(kernel="AUC") on the monitor pairs whose hinge
// mean it computes, make_exps.py:162-168): one read of the index streams for both statistics.
template <int K, int PPT, typename I, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_pair_sum_idx(const double* __restrict__ x,
                                                         const double* __restrict__ z,
                                                         const I* __restrict__ ix,
                                                         const I* __restrict__ iz,
                                                         const int64_t* __restrict__ pair_off,
                                                         int blocks_per_shard, double margin,
                                                         double* __restrict__ work,
                                                         unsigned long long* __restrict__ count) {
  const int s = blockIdx.x / blocks_per_shard;
  const int bi = blockIdx.x - s * blocks_per_shard;
  const int64_t pb = pair_off[s], pe = pair_off[s + 1];
  const int64_t p0 = pb + (int64_t)bi * (kBlock * PPT);
  double acc = 0.0;
  unsigned cnt = 0;
  if (p0 < pe) {
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int64_t p = p0 + k * kBlock + threadIdx.x;
      if (p < pe) {
        const double xv = x[ix[p]], zv = z[iz[p]];
        acc += fkern<K>(xv, zv, margin);
        if (COUNT) cnt += xv > zv;
      }
    }
  }
  const double b = block_sum_f64(acc);
  if (threadIdx.x == 0) work[blockIdx.x] = b;
  if constexpr (COUNT) {
    const unsigned long long w = wave_sum_u64((unsigned long long)cnt);
    if ((threadIdx.x & (kWave - 1)) == 0 && w) atomicAdd(count + s, w);
  }
}

// out[s] = ordered sum of work[s*per : (s+1)*per]; one wave per shard, lane-strided partial
// sums in a fixed order, then a fixed butterfly.
__global__ __launch_bounds__(kWave) void k_reduce_partials(const double* __restrict__ work,
                                                           int per, double* __restrict__ out) {
  const int s = blockIdx.x;
  double v = 0.0;
  for (int i = threadIdx.x; i < per; i += kWave) v += work[(int64_t)s * per + i];
  v = wave_sum_f64(v);
  if (threadIdx.x == 0) out[s] = v;
}

constexpr int kSumPPT = 8;

}  // namespace tw

using namespace tw;

extern "C" int64_t tw_pair_sum_work_per_shard(int64_t max_nx, int64_t max_nz) {
  const SumPlan p = plan_sum(max_nx, max_nz);
  return (int64_t)p.tiles_x * p.zchunks;
}

extern "C" int64_t tw_pair_sum_idx_work_per_shard(int64_t max_pairs) {
  return std::max<int64_t>(1, ceil_div(max_pairs, (int64_t)kBlock * kSumPPT));
}

extern "C" int tw_pair_sum_f64(const double* d_x, const int64_t* d_x_off, const double* d_z,
                               const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                               int64_t max_nz, int32_t kern, double margin, double* d_work,
                               double* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0, "tw_pair_sum_f64: bad sizes");
  TW_ARG_CHECK(kern >= TW_KERN_PROD && kern <= TW_KERN_LOGISTIC, "tw_pair_sum_f64: unknown kernel %d", kern);
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  const SumPlan p = plan_sum(max_nx, max_nz);
  const int64_t per = (int64_t)p.tiles_x * p.zchunks;
  TW_ARG_CHECK(per * n_shards < (1ll << 31), "tw_pair_sum_f64: grid too large");
  dim3 g((unsigned)(per * n_shards)), b(kBlock);
  if (kern == TW_KERN_PROD) hipLaunchKernelGGL(k_pair_sum<TW_KERN_PROD>, g, b, 0, st, d_x, d_x_off, d_z, d_z_off, p.tiles_x, p.zchunks, margin, d_work);
  else if (kern == TW_KERN_GINI) hipLaunchKernelGGL(k_pair_sum<TW_KERN_GINI>, g, b, 0, st, d_x, d_x_off, d_z, d_z_off, p.tiles_x, p.zchunks, margin, d_work);
  else if (kern == TW_KERN_HINGE) hipLaunchKernelGGL(k_pair_sum<TW_KERN_HINGE>, g, b, 0, st, d_x, d_x_off, d_z, d_z_off, p.tiles_x, p.zchunks, margin, d_work);
  else hipLaunchKernelGGL(k_pair_sum<TW_KERN_LOGISTIC>, g, b, 0, st, d_x, d_x_off, d_z, d_z_off, p.tiles_x, p.zchunks, margin, d_work);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_reduce_partials, dim3(n_shards), dim3(kWave), 0, st, d_work, (int)per, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

namespace tw {
template <typename I, bool COUNT>
int pair_sum_idx(const double* d_x, const double* d_z, const I* d_ix, const I* d_iz,
                 const int64_t* d_pair_off, int32_t n_shards, int64_t max_pairs, int32_t kern,
                 double margin, double* d_work, double* d_out, uint64_t* d_count,
                 hipStream_t st) {
  const int64_t per = tw_pair_sum_idx_work_per_shard(max_pairs);
  TW_ARG_CHECK(per * n_shards < (1ll << 31), "tw_pair_sum_idx_f64: grid too large");
  dim3 g((unsigned)(per * n_shards)), b(kBlock);
  unsigned long long* cnt = (unsigned long long*)d_count;
  if (kern == TW_KERN_PROD) hipLaunchKernelGGL((k_pair_sum_idx<TW_KERN_PROD, kSumPPT, I, COUNT>), g, b, 0, st, d_x, d_z, d_ix, d_iz, d_pair_off, (int)per, margin, d_work, cnt);
  else if (kern == TW_KERN_GINI) hipLaunchKernelGGL((k_pair_sum_idx<TW_KERN_GINI, kSumPPT, I, COUNT>), g, b, 0, st, d_x, d_z, d_ix, d_iz, d_pair_off, (int)per, margin, d_work, cnt);
  else if (kern == TW_KERN_HINGE) hipLaunchKernelGGL((k_pair_sum_idx<TW_KERN_HINGE, kSumPPT, I, COUNT>), g, b, 0, st, d_x, d_z, d_ix, d_iz, d_pair_off, (int)per, margin, d_work, cnt);
  else hipLaunchKernelGGL((k_pair_sum_idx<TW_KERN_LOGISTIC, kSumPPT, I, COUNT>), g, b, 0, st, d_x, d_z, d_ix, d_iz, d_pair_off, (int)per, margin, d_work, cnt);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_reduce_partials, dim3(n_shards), dim3(kWave), 0, st, d_work, (int)per, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
}  // namespace tw

extern "C" int tw_pair_sum_idx_f64(const double* d_x, const double* d_z, const int64_t* d_ix,
                                   const int64_t* d_iz, const int64_t* d_pair_off,
                                   int32_t n_shards, int64_t max_pairs, int32_t kern,
                                   double margin, double* d_work, double* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_pairs >= 0, "tw_pair_sum_idx_f64: bad sizes");
  TW_ARG_CHECK(kern >= TW_KERN_PROD && kern <= TW_KERN_LOGISTIC, "tw_pair_sum_idx_f64: unknown kernel %d", kern);
  if (n_shards == 0) return TW_OK;
  return pair_sum_idx<int64_t, false>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, kern,
                                      margin, d_work, d_out, nullptr, (hipStream_t)stream);
}

extern "C" int tw_pair_sum_idx32_f64(const double* d_x, const double* d_z, const int32_t* d_ix,
                                     const int32_t* d_iz, const int64_t* d_pair_off,
                                     int32_t n_shards, int64_t max_pairs, int32_t kern,
                                     double margin, double* d_work, double* d_out,
                                     uint64_t* d_count, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_pairs >= 0, "tw_pair_sum_idx32_f64: bad sizes");
  TW_ARG_CHECK(kern >= TW_KERN_PROD && kern <= TW_KERN_LOGISTIC, "tw_pair_sum_idx32_f64: unknown kernel %d", kern);
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  if (d_count == nullptr)
    return pair_sum_idx<int32_t, false>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs,
                                        kern, margin, d_work, d_out, nullptr, st);
  TW_HIP_CHECK(tw_zero_async(d_count, 0, sizeof(uint64_t) * n_shards, st));
  return pair_sum_idx<int32_t, true>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, kern,
                                     margin, d_work, d_out, d_count, st);
}
