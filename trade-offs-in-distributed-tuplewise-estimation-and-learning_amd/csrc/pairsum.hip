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

__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v) {
  v = wave_sum_u64(v);
  __shared__ unsigned long long partc[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) partc[wid] = v;
  __syncthreads();
  unsigned long long b = 0;
  if (threadIdx.x == 0) b = (partc[0] + partc[1]) + (partc[2] + partc[3]);
  return b;
}

// One block of k_pair_sum — (shard, x tile, z chunk) number `bid` — returning its partial (on
// thread 0).  CNT: also #{x > z} over the block's pairs into *cnt (thread 0; a NaN compares
// false, as k_count_complete's v_cmp_gt_f64).
template <int K, bool CNT>
__device__ __forceinline__ double pair_sum_block(const double* __restrict__ x,
                                                 const int64_t* __restrict__ x_off,
                                                 const double* __restrict__ z,
                                                 const int64_t* __restrict__ z_off, int tiles_x,
                                                 int zchunks, double margin, int bid,
                                                 unsigned long long* cnt) {
  const int per_shard = tiles_x * zchunks;
  const int s = bid / per_shard;
  const int rem = bid - s * per_shard;
  const int cz = rem / tiles_x;
  const int tx = rem - cz * tiles_x;
  const int64_t xb = x_off[s], xe = x_off[s + 1];
  const int64_t zb = z_off[s], ze = z_off[s + 1];
  const int64_t x0 = xb + (int64_t)tx * (kBlock * kSumR);
  const int64_t z0 = zb + (int64_t)cz * kSumZChunk;
  if (x0 >= xe || z0 >= ze) {  // block-uniform; the slot must still be written
    if (CNT) *cnt = 0;
    return 0.0;
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
  unsigned cr[kSumR] = {};
#pragma unroll 4
  for (int j = 0; j < nz; ++j) {
    const double zv = zp[j];
#pragma unroll
    for (int r = 0; r < kSumR; ++r) {
      acc[r] += fkern_loop<K>(xv[r], zv, margin);
      if (CNT) cr[r] += xv[r] > zv;
    }
  }
  double t = 0.0;
#pragma unroll
  for (int r = 0; r < kSumR; ++r) t += valid[r] ? acc[r] : 0.0;
  if (CNT) {
    unsigned long long c = 0;
#pragma unroll
    for (int r = 0; r < kSumR; ++r) c += valid[r] ? cr[r] : 0u;
    *cnt = block_sum_u64(c);
  }
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
    return ((xbits | zbits) & 1) || (xbits & zbits & 6)
               ? __longlong_as_double(0x7FF8000000000000ll)
               : b;
  }
  return b;
}

template <int K>
__global__ __launch_bounds__(kBlock) void k_pair_sum(const double* __restrict__ x,
                                                     const int64_t* __restrict__ x_off,
                                                     const double* __restrict__ z,
                                                     const int64_t* __restrict__ z_off,
                                                     int tiles_x, int zchunks, double margin,
                                                     double* __restrict__ work) {
  const double b = pair_sum_block<K, false>(x, x_off, z, z_off, tiles_x, zchunks, margin,
                                            (int)blockIdx.x, nullptr);
  if (threadIdx.x == 0) work[blockIdx.x] = b;
}

// One block of k_pair_sum_idx, number `bid`: its partial (thread 0) and, COUNT, its pairs'
// #{x > z} (every lane's own count; the caller reduces them)
template <int K, int PPT, typename I, bool COUNT>
__device__ __forceinline__ double pair_sum_idx_block(const double* __restrict__ x,
                                                     const double* __restrict__ z,
                                                     const I* __restrict__ ix,
                                                     const I* __restrict__ iz,
                                                     const int64_t* __restrict__ pair_off,
                                                     int blocks_per_shard, double margin,
                                                     int bid, unsigned* lane_cnt) {
  const int s = bid / blocks_per_shard;
  const int bi = bid - s * blocks_per_shard;
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
  if (COUNT) *lane_cnt = cnt;
  return block_sum_f64(acc);
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
  unsigned cnt = 0;
  const double b = pair_sum_idx_block<K, PPT, I, COUNT>(x, z, ix, iz, pair_off,
                                                        blocks_per_shard, margin,
                                                        (int)blockIdx.x, &cnt);
  if (threadIdx.x == 0) work[blockIdx.x] = b;
  if constexpr (COUNT) {
    const int s = (int)blockIdx.x / blocks_per_shard;
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

// ---------------------------------------------------------------- fused evaluation (round 3)
// evaluation_step's FIXED_PAIRS statistics for small problems (make_exps.py:143-190: the C4
// loop evaluates every 25 steps) in TWO launches instead of a dozen: k_eval_scores computes the
// four score vectors (train X, train Z, test X, test Z) with k_gemv's per-row arithmetic;
// k_eval_pairs runs the blocks of k_pair_sum_idx (the monitor pairs: surrogate sum + AUC count)
// and of k_pair_sum (all test pairs: surrogate sum + AUC count) side by side, and the block
// that arrives last reduces both partial arrays with k_reduce_partials' order.  Same bits as
// the separate launches (tests/test_gpu_learning.py).  Hand-off: every block's thread 0 stores
// its partials write-through (sc1), waits for them (vmcnt(0)) and takes a ticket; the last
// ticket's block reads them with sc1 loads (MI355X_MICROARCH.md "Valid forms", row 1).
__device__ __forceinline__ void st_sc1_u64(void* p, unsigned long long v) {
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1_u64(const void* p) {
  return __hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBlock) void k_eval_scores(const double* __restrict__ a0, int64_t n0,
                                                        const double* __restrict__ a1, int64_t n1,
                                                        const double* __restrict__ a2, int64_t n2,
                                                        const double* __restrict__ a3, int64_t n3,
                                                        int64_t d, const double* __restrict__ w,
                                                        double* __restrict__ out) {
  const int64_t tot = n0 + n1 + n2 + n3;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * kBlock) {
    const double* row = i < n0             ? a0 + i * d
                        : i < n0 + n1      ? a1 + (i - n0) * d
                        : i < n0 + n1 + n2 ? a2 + (i - n0 - n1) * d
                                           : a3 + (i - n0 - n1 - n2) * d;
    double a = 0.0;  // k_gemv's order: j = 0 .. d-1, multiply then add (no contraction)
    for (int64_t j = 0; j < d; ++j) a += row[j] * w[j];
    out[i] = a;
  }
}

template <int K>
__global__ __launch_bounds__(kBlock) void k_eval_pairs(
    const double* __restrict__ sx, const double* __restrict__ sz, const int32_t* __restrict__ ix,
    const int32_t* __restrict__ iz, const int64_t* __restrict__ offs, int per_idx,
    const double* __restrict__ tx, const double* __restrict__ tz, int tiles_x, int zchunks,
    double margin, double* work, unsigned long long* cwork, unsigned* ticket, double* out) {
  const int nb = per_idx + tiles_x * zchunks;
  double v;
  unsigned long long c = 0;
  if ((int)blockIdx.x < per_idx) {
    unsigned lc = 0;
    v = pair_sum_idx_block<K, kSumPPT, int32_t, true>(sx, sz, ix, iz, offs, per_idx, margin,
                                                      (int)blockIdx.x, &lc);
    c = block_sum_u64(lc);
  } else {
    v = pair_sum_block<K, true>(tx, offs + 2, tz, offs + 4, tiles_x, zchunks, margin,
                                (int)blockIdx.x - per_idx, &c);
  }
  __shared__ int last;
  if (threadIdx.x == 0) {
    st_sc1_u64(work + blockIdx.x, __double_as_longlong(v));
    st_sc1_u64(cwork + blockIdx.x, c);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // release: this block's partials before its ticket; acquire: the last block's loads of
    // every other block's partials after the ticket that saw them all
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)nb - 1;
  }
  __syncthreads();
  if (!last) return;
  const int wid = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  if (wid < 2) {  // wave 0: the monitor pairs' partials, wave 1: the test pairs'
    const int base = wid == 0 ? 0 : per_idx, per = wid == 0 ? per_idx : nb - per_idx;
    double sum = 0.0;
    unsigned long long cc = 0;
    for (int i = lane; i < per; i += kWave) {
      sum += __longlong_as_double(ld_sc1_u64(work + base + i));
      cc += ld_sc1_u64(cwork + base + i);
    }
    sum = wave_sum_f64(sum);
    cc = wave_sum_u64(cc);
    if (lane == 0) {
      out[2 * wid] = sum;
      out[2 * wid + 1] = __longlong_as_double((long long)cc);
    }
  }
  if (threadIdx.x == 0)  // the next launch starts from zero (no memset node in its graph)
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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

extern "C" int64_t tw_eval_small_work(int64_t n_pairs, int64_t n_test_x, int64_t n_test_z) {
  const SumPlan p = plan_sum(n_test_x, n_test_z);
  return tw_pair_sum_idx_work_per_shard(n_pairs) + (int64_t)p.tiles_x * p.zchunks;
}

extern "C" int tw_eval_small(const double* d_trX, int64_t n_trX, const double* d_trZ,
                             int64_t n_trZ, const double* d_teX, int64_t n_teX,
                             const double* d_teZ, int64_t n_teZ, int64_t d, const double* d_w,
                             const int32_t* d_ix, const int32_t* d_iz, int64_t n_pairs,
                             const int64_t* d_offs, int32_t kern, double margin,
                             double* d_scores, double* d_work, uint64_t* d_cwork,
                             uint32_t* d_ticket, double* d_out, void* stream) {
  TW_ARG_CHECK(n_trX >= 1 && n_trZ >= 1 && n_teX >= 1 && n_teZ >= 1 && d >= 1 && n_pairs >= 1,
               "tw_eval_small: empty operand");
  TW_ARG_CHECK(kern == TW_KERN_HINGE || kern == TW_KERN_LOGISTIC,
               "tw_eval_small: hinge or logistic only (kernel %d)", kern);
  const SumPlan p = plan_sum(n_teX, n_teZ);
  const int64_t per_idx = tw_pair_sum_idx_work_per_shard(n_pairs);
  const int64_t nb = per_idx + (int64_t)p.tiles_x * p.zchunks;
  TW_ARG_CHECK(nb < (1ll << 31), "tw_eval_small: grid too large");
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = n_trX + n_trZ + n_teX + n_teZ;
  const int gs = (int)std::min<int64_t>(4096, ceil_div(rows, kBlock));
  hipLaunchKernelGGL(k_eval_scores, dim3(gs), dim3(kBlock), 0, st, d_trX, n_trX, d_trZ, n_trZ,
                     d_teX, n_teX, d_teZ, n_teZ, d, d_w, d_scores);
  TW_LAUNCH_CHECK();
  const double* sx = d_scores;
  const double* sz = sx + n_trX;
  const double* tx = sz + n_trZ;
  const double* tz = tx + n_teX;
  auto go = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, sx, sz, d_ix, d_iz,
                       d_offs, (int)per_idx, tx, tz, p.tiles_x, p.zchunks, margin, d_work,
                       (unsigned long long*)d_cwork, d_ticket, d_out);
  };
  if (kern == TW_KERN_HINGE)
    go(k_eval_pairs<TW_KERN_HINGE>);
  else
    go(k_eval_pairs<TW_KERN_LOGISTIC>);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
