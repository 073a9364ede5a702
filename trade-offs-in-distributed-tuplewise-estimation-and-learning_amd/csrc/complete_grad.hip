// complete_grad.hip — complete-block gradient of the pairwise surrogate, computed as
// per-point pair-coefficient reductions followed by X^T c (BASELINE.json north_star item (2)).
//
// The reference's learner uses B sampled pairs per block (grad_inc_block,
// learning-experiment/compute_stats.py:146-162; csrc/hinge.hip).  Over ALL pairs of a block
// (kx X-rows, kz Z-rows) the same surrogate's gradient factorises:
//   S_ij = z_j.w - x_i.w + margin,   g = (1/(kx kz)) sum_ij phi'(S_ij) (z_j - x_i)
//     = (1/(kx kz)) (sum_j a_j z_j - sum_i b_i x_i),
//   a_j = sum_i phi'(S_ij),  b_i = sum_j phi'(S_ij),  phi' = 1{S > 0} (hinge) or sigma(S).
// So the O(kx kz) work is on SCALARS (scores), and the rows are read twice: once for the
// scores (a GEMV) and once for the coefficient-weighted column sums (a transposed GEMV).
// Plain VALU: the pair step is compare/exp + add, not a dense contraction.
//
// Kernels (all deterministic: every sum has a fixed order):
//   k_row_scores     one wave per row: lane-strided partial dot + fixed butterfly
//   k_pair_coef      (logistic) thread per point, the other side's scores staged in LDS
//                    chunks; the point's coefficient is summed in the other side's index order
//   k_sort_chunks +  (hinge) the coefficients are COUNTS: b_i = #{j : S_ij > 0}, a_j =
//   k_hinge_coef     #{i : S_ij > 0}.  S = fl(fl(sz - sx) + m) is monotone in each score, so
//                    over the other side's sorted chunks each count is a binary search with
//                    the exact floating-point predicate: O(k log k) instead of O(k^2), and the
//                    same integers as summing 1{S > 0} pair by pair
//   k_wcolsum_part   thread per column, 256-row chunks of [Z rows (+a) | X rows (-b)] in order
//   k_wcolsum_final  chunk partials added in chunk order, / (kx kz)
#include "sortkeys.h"
#include <algorithm>
#include <type_traits>

namespace tw {

constexpr int kCoefChunk = 4096;  // other-side scores staged per pass (32 KiB)
constexpr int kColRows = 256;     // rows per column-sum chunk
constexpr int kCgMaxD = 4096;

__global__ __launch_bounds__(kBlock) void k_row_scores(const double* __restrict__ A, int64_t d,
                                                       const int64_t* __restrict__ rows,
                                                       int64_t total,
                                                       const double* __restrict__ w,
                                                       double* __restrict__ out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t waves = (int64_t)gridDim.x * (kBlock / kWave);
  if ((d & 1) == 0) {  // 16-B loads: lane takes column pairs 2j, 2j+1 (rows are 16-B aligned)
    const int64_t d2 = d >> 1;
    const double2* __restrict__ w2 = (const double2*)w;
    for (int64_t r = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave; r < total;
         r += waves) {
      const double2* __restrict__ a2 = (const double2*)(A + (rows ? rows[r] : r) * d);
      double p0 = 0.0, p1 = 0.0;
#pragma unroll 4
      for (int64_t j = lane; j < d2; j += kWave) {
        const double2 v = a2[j], ww = w2[j];
        p0 += v.x * ww.x;
        p1 += v.y * ww.y;
      }
      const double p = wave_sum_dpp_f64(p0 + p1);
      if (lane == 0) out[r] = p;
    }
    return;
  }
  for (int64_t r = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave; r < total; r += waves) {
    const double* a = A + (rows ? rows[r] : r) * d;
    double p = 0.0;
    for (int64_t j = lane; j < d; j += kWave) p += a[j] * w[j];
    p = wave_sum_dpp_f64(p);
    if (lane == 0) out[r] = p;
  }
}

// A @ w for a row-major (n, d) matrix, one wave per row (tw_gemv_f64 for d > 32)
int launch_row_scores(const double* A, int64_t d, int64_t n, const double* w, double* out,
                      hipStream_t st) {
  const int blocks = (int)std::min<int64_t>(256 * 16, ceil_div(n, kBlock / kWave));
  hipLaunchKernelGGL(k_row_scores, dim3(blocks), dim3(kBlock), 0, st, A, d,
                     (const int64_t*)nullptr, n, w, out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// SIDE 0: coef of x-point i = sum_j phi'(sz_j - sx_i + m); SIDE 1: of z-point j, over i.
template <int LOSS, int SIDE>
__global__ __launch_bounds__(kBlock) void k_pair_coef(const double* __restrict__ s_own,
                                                      int64_t k_own,
                                                      const double* __restrict__ s_other,
                                                      int64_t k_other, double margin, int tiles,
                                                      double* __restrict__ coef) {
  __shared__ double buf[kCoefChunk];
  const int s = blockIdx.x / tiles;
  const int tile = blockIdx.x - s * tiles;
  const double* own = s_own + (int64_t)s * k_own;
  const double* oth = s_other + (int64_t)s * k_other;
  const int64_t p = (int64_t)tile * kBlock + threadIdx.x;
  const bool valid = p < k_own;
  const double v = valid ? own[p] : 0.0;
  double acc = 0.0;
  for (int64_t c0 = 0; c0 < k_other; c0 += kCoefChunk) {
    const int n = (int)std::min<int64_t>(kCoefChunk, k_other - c0);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kBlock) buf[i] = oth[c0 + i];
    __syncthreads();
    for (int j = 0; j < n; ++j) {
      const double S = SIDE == 0 ? (buf[j] - v) + margin : (v - buf[j]) + margin;
      acc += pair_weight<LOSS>(S);
    }
  }
  if (valid) coef[(int64_t)s * k_own + p] = acc;
}

// Number of leading entries of the sorted chunk a[0, C) (C a power of two) with pred true, for
// pred monotone true...true false...false along the chunk.
template <typename P>
__device__ __forceinline__ uint32_t prefix_count(const uint64_t* a, int C, P pred) {
  uint32_t i = 0;
  for (int st = C >> 1; st > 0; st >>= 1) i += pred(a[i + st - 1]) ? st : 0;
  return i + (pred(a[i]) ? 1 : 0);
}

// Hinge coefficients by threshold search.  SIDE 0: own = x-scores, b_i = #{j : (sz_j - v) + m
// > 0}; SIDE 1: own = z-scores, a_j = #{i : (v - sx_i) + m > 0}; the other side's scores are
// sorted chunks of order keys (padding / NaN = ~0, never counted).  A NaN own score counts 0.
constexpr int kHcPer = 4;  // own points per thread
template <int SIDE>
__global__ __launch_bounds__(kSortThreads) void k_hinge_coef(const double* __restrict__ s_own,
                                                             int64_t k_own,
                                                             const uint64_t* __restrict__ keys_other,
                                                             int chunks, int C, double margin,
                                                             int tiles, double* __restrict__ coef) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / tiles;
  const int tile = lb - s * tiles;
  const double* own = s_own + (int64_t)s * k_own;
  double v[kHcPer];
  uint32_t cnt[kHcPer];
  bool live[kHcPer];
#pragma unroll
  for (int r = 0; r < kHcPer; ++r) {
    const int64_t p = (int64_t)tile * (kSortThreads * kHcPer) + r * kSortThreads + threadIdx.x;
    live[r] = p < k_own;
    v[r] = live[r] ? own[p] : 0.0;
    live[r] = live[r] && v[r] == v[r];
    cnt[r] = 0;
  }
  const int group = (int)std::max<int64_t>(1, kMaxChunk / C);
  for (int c0 = 0; c0 < chunks; c0 += group) {
    const int ng = std::min(group, chunks - c0);
    const uint64_t* src = keys_other + ((int64_t)s * chunks + c0) * C;
    __syncthreads();
    for (int i = threadIdx.x; i < ng * C; i += kSortThreads) keys[i] = src[i];
    __syncthreads();
    for (int g = 0; g < ng; ++g) {
      const uint64_t* kc = keys + g * C;
#pragma unroll
      for (int r = 0; r < kHcPer; ++r) {
        if (!live[r]) continue;
        const double vv = v[r];
        if (SIDE == 1) {  // true for small sx: (v - sx) + m > 0
          cnt[r] += prefix_count(kc, C, [=](uint64_t k) {
            return k != ~0ull && (vv - key_to_double(k)) + margin > 0.0;
          });
        } else {  // true for large sz: count = valid - #{leading sz with S <= 0}
          const uint32_t valid = lower_bound_lds(kc, C, ~0ull);
          const uint32_t below = prefix_count(kc, C, [=](uint64_t k) {
            return k != ~0ull && !((key_to_double(k) - vv) + margin > 0.0);
          });
          cnt[r] += valid - below;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kHcPer; ++r) {
    const int64_t p = (int64_t)tile * (kSortThreads * kHcPer) + r * kSortThreads + threadIdx.x;
    if (p < k_own) coef[(int64_t)s * k_own + p] = (double)cnt[r];
  }
}

// Logistic coefficients in ONE pass over the pairs (each sigma(S_ij) is evaluated once and
// feeds both sums).  A 512-thread block holds kLgR = 8 x-scores per lane (a tile of 4096
// x-points of one shard) and streams the shard's z-scores through LDS in chunks of kLgChunk:
//   b_i += sigma(S_ij)              per lane, in j order (registers)
//   a_j  = sum over the tile's x    lane butterfly, then the 8 waves in wave order (LDS),
// writing one partial of a_j per (tile, j); k_apart_final adds the tiles in tile order.
// Deterministic.  With the separated exponent (below) a sigma is an FMA and a reciprocal.
constexpr int kLgR = 16;
constexpr int kLgThreads = 256;
constexpr int kLgChunk = 512;
__global__ __launch_bounds__(kLgThreads, 2) void k_logistic_coef(const double* __restrict__ sx,
                                                              int64_t kx,
                                                              const double* __restrict__ sz,
                                                              int64_t kz, double margin,
                                                              int tiles,
                                                              double* __restrict__ bx,
                                                              double* __restrict__ apart) {
  __shared__ double zc[kLgChunk];
  __shared__ double eb[kLgChunk];  // exp(-sz_j), or NaN where that is out of range
  __shared__ double wpart[kLgThreads / kWave][kLgChunk];
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / tiles;
  const int tile = lb - s * tiles;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  // e^-S_ij = e^(sx_i - m) * e^(-sz_j): the exponent SEPARATES, so a sigma is one FMA and a
  // Newton reciprocal instead of an exp and an IEEE division.  Used for a (tile, chunk) when
  // every factor's exponent is within +-350 (the product then stays a normal double); any
  // other chunk takes the direct formula, so the result never depends on the data's range.
  // registers: the factors e^(sx - m) and the b sums (the scores themselves are re-read
  // only by the rare direct-formula chunks), so 16 x-values per lane fit
  double b[kLgR], ea[kLgR];
  unsigned valid = 0;  // bit r: x-value r of this lane exists
  int tile_sep = 1, tile_sep40 = 1;
  const double* xs = sx + (int64_t)s * kx + (int64_t)tile * (kLgThreads * kLgR) + threadIdx.x;
#pragma unroll
  for (int r = 0; r < kLgR; ++r) {
    const int64_t i = (int64_t)tile * (kLgThreads * kLgR) + r * kLgThreads + threadIdx.x;
    const bool ok = i < kx;
    valid |= (unsigned)ok << r;
    const double u = (ok ? xs[r * kLgThreads] : 0.0) - margin;
    b[r] = 0.0;
    tile_sep &= __builtin_fabs(u) <= 350.0;
    tile_sep40 &= __builtin_fabs(u) <= 40.0;
    ea[r] = exp(u);
  }
  tile_sep = __syncthreads_and(tile_sep);
  tile_sep40 = __syncthreads_and(tile_sep40);
  const int tile_full = __syncthreads_and(valid == (1u << kLgR) - 1u);
  const double* zs = sz + (int64_t)s * kz;
  double* ap = apart + ((int64_t)s * tiles + tile) * kz;
  for (int64_t c0 = 0; c0 < kz; c0 += kLgChunk) {
    const int n = (int)std::min<int64_t>(kLgChunk, kz - c0);
    __syncthreads();
    int chunk_sep = tile_sep, chunk_sep40 = 1;
    for (int j = threadIdx.x; j < n; j += kLgThreads) {
      const double zj = zs[c0 + j];
      zc[j] = zj;
      eb[j] = exp(-zj);
      chunk_sep &= __builtin_fabs(zj) <= 350.0;
      chunk_sep40 &= __builtin_fabs(zj) <= 40.0;
    }
    chunk_sep = __syncthreads_and(chunk_sep);  // block-uniform
    chunk_sep40 = __syncthreads_and(chunk_sep40);
    // a block whose x-values all exist (every tile but a shard's last) adds y to t without a
    // select: 8 VALU per pair instead of 10 (the same sums in the same order)
    // sigma = 1 / q, q = 1 + e^(sx_i - m) e^(-sz_j), from v_rcp_f64 (2^-24 relative on gfx950)
    // plus ONE Newton step (<= 10 ulp; tools/mb_rcp.hip, profiles/r02_mb_rcp_accuracy.log).
    // BATCH: when every factor's exponent is within +-40 (q <= 1 + e^80), the reciprocals of
    // 8 q's come from one (Montgomery's batch inversion): prefix products P_k = q_0...q_k
    // (<= e^640, a normal double), I = 1 / P_7, then y_k = I_k P_(k-1), I_(k-1) = I_k q_k —
    // 3.4 multiplies per sigma instead of a quarter-rate reciprocal and its Newton step.
    // Relative error <= ~20 ulp per sigma either way (the oracle tolerance is 1e-10).
    auto sep_chunk = [&](auto all_valid, auto batch) {
      // NJ z-values at a time: independent chains interleave (2 waves per SIMD at this
      // register count); every sum still takes its terms in the same order
      auto step = [&](auto nj, int j0) {
        constexpr int NJ = decltype(nj)::value;
        double ejv[NJ], t[NJ];
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
          ejv[u] = eb[j0 + u];
          t[u] = 0.0;
        }
        if constexpr (decltype(batch)::value) {
#pragma unroll
          for (int g = 0; g < kLgR; g += 8) {
            double q[NJ][8], P[NJ][7], I[NJ], tg[NJ];
#pragma unroll
            for (int u = 0; u < NJ; ++u) {
#pragma unroll
              for (int k = 0; k < 8; ++k) q[u][k] = __builtin_fma(ea[g + k], ejv[u], 1.0);
              P[u][0] = q[u][0];
#pragma unroll
              for (int k = 1; k < 7; ++k) P[u][k] = P[u][k - 1] * q[u][k];
              const double P7 = P[u][6] * q[u][7];
              I[u] = __builtin_amdgcn_rcp(P7);
              I[u] = __builtin_fma(__builtin_fma(-P7, I[u], 1.0), I[u], I[u]);
              tg[u] = 0.0;  // the group's sigmas are consumed as they appear (k = 7 .. 0)
            }
#pragma unroll
            for (int k = 7; k >= 0; --k) {
#pragma unroll
              for (int u = 0; u < NJ; ++u) {
                const double y = k ? I[u] * P[u][k - 1] : I[u];
                if (k) I[u] = I[u] * q[u][k];
                b[g + k] += y;
                if constexpr (decltype(all_valid)::value)
                  tg[u] += y;
                else
                  tg[u] += (valid >> (g + k)) & 1u ? y : 0.0;
              }
            }
#pragma unroll
            for (int u = 0; u < NJ; ++u) t[u] += tg[u];
          }
        } else {
#pragma unroll
          for (int u = 0; u < NJ; ++u) {
#pragma unroll
            for (int r = 0; r < kLgR; ++r) {
              const double q = __builtin_fma(ea[r], ejv[u], 1.0);  // 1 + e^-S in [1, e^700]
              double y = __builtin_amdgcn_rcp(q);
              y = __builtin_fma(__builtin_fma(-q, y, 1.0), y, y);
              b[r] += y;
              if constexpr (decltype(all_valid)::value)
                t[u] += y;
              else
                t[u] += (valid >> r) & 1u ? y : 0.0;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < NJ; ++u) {
          const double tt = wave_sum_dpp_f64(t[u]);
          if (lane == 0) wpart[wid][j0 + u] = tt;
        }
      };
      int j = 0;
      for (; j + 1 < n; j += 2) step(std::integral_constant<int, 2>{}, j);
      if (j < n) step(std::integral_constant<int, 1>{}, j);
    };
    if (chunk_sep) {
      // both block-uniform (the wave sums inside need every lane)
      const bool batch = tile_sep40 && chunk_sep40;
      if (tile_full && batch)
        sep_chunk(std::true_type{}, std::true_type{});
      else if (tile_full)
        sep_chunk(std::true_type{}, std::false_type{});
      else if (batch)
        sep_chunk(std::false_type{}, std::true_type{});
      else
        sep_chunk(std::false_type{}, std::false_type{});
    } else {
      for (int j = 0; j < n; ++j) {
        const double zj = zc[j];
        double t = 0.0;
#pragma unroll 1
        for (int r = 0; r < kLgR; ++r) {
          const bool ok = (valid >> r) & 1u;
          const double vr = ok ? xs[r * kLgThreads] : 0.0;
          const double p = pair_weight<TW_LOSS_LOGISTIC>((zj - vr) + margin);
          b[r] += p;
          t += ok ? p : 0.0;
        }
        t = wave_sum_dpp_f64(t);
        if (lane == 0) wpart[wid][j] = t;
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += kLgThreads) {
      double a = 0.0;
#pragma unroll
      for (int w = 0; w < kLgThreads / kWave; ++w) a += wpart[w][j];
      ap[c0 + j] = a;
    }
  }
#pragma unroll
  for (int r = 0; r < kLgR; ++r) {
    const int64_t i = (int64_t)tile * (kLgThreads * kLgR) + r * kLgThreads + threadIdx.x;
    if ((valid >> r) & 1u) bx[(int64_t)s * kx + i] = b[r];
  }
}

__global__ __launch_bounds__(kBlock) void k_apart_final(const double* __restrict__ apart,
                                                        int n_shards, int tiles, int64_t kz,
                                                        double* __restrict__ az) {
  const int64_t total = (int64_t)n_shards * kz;
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t s = e / kz, j = e - s * kz;
    const double* p = apart + (int64_t)s * tiles * kz + j;
    double a = 0.0;
    for (int t = 0; t < tiles; ++t) a += p[(int64_t)t * kz];
    az[e] = a;
  }
}

// partial[s][c][col] = sum over rows r of chunk c (in order) of w_r * row_r[col], rows of shard
// s being [Z rows j (w = +a_j) | X rows i (w = -b_i)].
__global__ __launch_bounds__(kBlock) void k_wcolsum_part(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const double* __restrict__ b, const double* __restrict__ a, int chunks,
    int ctiles, double* __restrict__ partial) {
  const int per = chunks * ctiles;
  const int s = blockIdx.x / per;
  const int rem = blockIdx.x - s * per;
  const int c = rem / ctiles;
  const int64_t r0 = (int64_t)c * kColRows, r1 = std::min<int64_t>(r0 + kColRows, kx + kz);
  if ((d & 1) == 0) {  // two columns per thread, 16-B loads; each column still in row order
    const int64_t col2 = (int64_t)(rem - c * ctiles) * kBlock + threadIdx.x;
    if (2 * col2 >= d) return;
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll 4
    for (int64_t r = r0; r < r1; ++r) {
      double wr;
      const double* rowp;
      if (r < kz) {
        wr = a[(int64_t)s * kz + r];
        rowp = Z + (rows_z ? rows_z[(int64_t)s * kz + r] : (int64_t)s * kz + r) * d;
      } else {
        const int64_t i = r - kz;
        wr = -b[(int64_t)s * kx + i];
        rowp = X + (rows_x ? rows_x[(int64_t)s * kx + i] : (int64_t)s * kx + i) * d;
      }
      const double2 v = ((const double2*)rowp)[col2];
      acc0 += wr * v.x;
      acc1 += wr * v.y;
    }
    double* dst = partial + ((int64_t)s * chunks + c) * d + 2 * col2;
    dst[0] = acc0;
    dst[1] = acc1;
    return;
  }
  const int64_t col = (int64_t)(rem - c * ctiles) * kBlock + threadIdx.x;
  if (col >= d) return;
  double acc = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    double wr, v;
    if (r < kz) {
      wr = a[(int64_t)s * kz + r];
      const int64_t row = rows_z ? rows_z[(int64_t)s * kz + r] : (int64_t)s * kz + r;
      v = Z[row * d + col];
    } else {
      const int64_t i = r - kz;
      wr = -b[(int64_t)s * kx + i];
      const int64_t row = rows_x ? rows_x[(int64_t)s * kx + i] : (int64_t)s * kx + i;
      v = X[row * d + col];
    }
    acc += wr * v;
  }
  partial[((int64_t)s * chunks + c) * d + col] = acc;
}

__global__ __launch_bounds__(kBlock) void k_wcolsum_final(const double* __restrict__ partial,
                                                          int n_shards, int chunks, int64_t d,
                                                          double denom, double* __restrict__ out) {
  const int64_t total = (int64_t)n_shards * d;
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t s = e / d, col = e - s * d;
    const double* p = partial + (int64_t)s * chunks * d + col;
    double acc = 0.0;
    for (int c = 0; c < chunks; ++c) acc += p[(int64_t)c * d];
    out[e] = acc / denom;
  }
}

struct CgLayout {
  int64_t sx, sz, bx, az, part, keys_x, keys_z;  // offsets (8-B words) into the workspace
  int64_t total;
  int chunks;
  int Cx, chx, Cz, chz;  // sorted-chunk length and count of the x / z scores (hinge)
  int64_t apart;         // per-(x tile, z point) partials of a_j (logistic)
  int lg_tiles;
};

// sorted chunks of C <= 4096 keys (the sorted-count path's best chunk, rankcount.hip)
static void score_chunks(int64_t k, int& C, int& ch) {
  int64_t c = 1024;
  while (c < k && c < 4096) c <<= 1;
  C = (int)c;
  ch = (int)std::max<int64_t>(1, ceil_div(k, c));
}

static CgLayout cg_layout(int32_t n_shards, int64_t kx, int64_t kz, int64_t d) {
  CgLayout l;
  const int64_t nx = (int64_t)n_shards * kx, nz = (int64_t)n_shards * kz;
  l.chunks = (int)std::max<int64_t>(1, ceil_div(kx + kz, kColRows));
  score_chunks(kx, l.Cx, l.chx);
  score_chunks(kz, l.Cz, l.chz);
  l.sx = 0;
  l.sz = l.sx + nx;
  l.bx = l.sz + nz;
  l.az = l.bx + nx;
  l.part = l.az + nz;
  l.keys_x = l.part + (int64_t)n_shards * l.chunks * d;
  l.keys_z = l.keys_x + (int64_t)n_shards * l.chx * l.Cx;
  l.lg_tiles = (int)ceil_div(kx, (int64_t)kLgThreads * kLgR);
  l.apart = l.keys_z + (int64_t)n_shards * l.chz * l.Cz;
  l.total = l.apart + (int64_t)n_shards * l.lg_tiles * kz;
  return l;
}

static int launch_hinge_coef(const double* sx, int64_t kx, const double* sz, int64_t kz,
                             int32_t n_shards, double margin, const CgLayout& l, double* work,
                             double* bx, double* az, hipStream_t st) {
  static bool attrs_set = false;
  if (!attrs_set) {
    for (const void* f : {(const void*)k_sort_chunks<double, 4>, (const void*)k_hinge_coef<0>,
                          (const void*)k_hinge_coef<1>})
      TW_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(sizeof(uint64_t) * kMaxChunk)));
    attrs_set = true;
  }
  uint64_t* keys_x = (uint64_t*)(work + l.keys_x);
  uint64_t* keys_z = (uint64_t*)(work + l.keys_z);
  TW_ARG_CHECK((int64_t)n_shards * std::max(l.chx, l.chz) < (1ll << 31),
               "tw_pair_grad_complete: grid too large");
  // C <= 4096 -> E = 4, C / 4 threads per block
  hipLaunchKernelGGL((k_sort_chunks<double, 4>), dim3(n_shards * l.chx), dim3(l.Cx / 4),
                     sizeof(uint64_t) * l.Cx, st, sx, nullptr, l.chx, l.Cx, keys_x, kx);
  hipLaunchKernelGGL((k_sort_chunks<double, 4>), dim3(n_shards * l.chz), dim3(l.Cz / 4),
                     sizeof(uint64_t) * l.Cz, st, sz, nullptr, l.chz, l.Cz, keys_z, kz);
  const int tx = (int)ceil_div(kx, (int64_t)kSortThreads * kHcPer);
  const int tz = (int)ceil_div(kz, (int64_t)kSortThreads * kHcPer);
  const size_t lds_x = sizeof(uint64_t) * std::min<int64_t>((int64_t)l.chz * l.Cz, kMaxChunk);
  const size_t lds_z = sizeof(uint64_t) * std::min<int64_t>((int64_t)l.chx * l.Cx, kMaxChunk);
  hipLaunchKernelGGL((k_hinge_coef<0>), dim3(n_shards * tx), dim3(kSortThreads), lds_x, st, sx,
                     kx, keys_z, l.chz, l.Cz, margin, tx, bx);
  hipLaunchKernelGGL((k_hinge_coef<1>), dim3(n_shards * tz), dim3(kSortThreads), lds_z, st, sz,
                     kz, keys_x, l.chx, l.Cx, margin, tz, az);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <int LOSS>
static void launch_coef(const double* sx, int64_t kx, const double* sz, int64_t kz,
                        int32_t n_shards, double margin, double* bx, double* az,
                        hipStream_t st) {
  const int tx = (int)ceil_div(kx, kBlock), tz = (int)ceil_div(kz, kBlock);
  hipLaunchKernelGGL((k_pair_coef<LOSS, 0>), dim3(n_shards * tx), dim3(kBlock), 0, st, sx, kx,
                     sz, kz, margin, tx, bx);
  hipLaunchKernelGGL((k_pair_coef<LOSS, 1>), dim3(n_shards * tz), dim3(kBlock), 0, st, sz, kz,
                     sx, kx, margin, tz, az);
}

static int g_hinge_by_search = 1;  // tw_pair_grad_complete_set_search: 0 = all-pairs sums
static int g_logistic_one_pass = 1;  // likewise: 0 = the two-pass k_pair_coef

}  // namespace tw

using namespace tw;

extern "C" int tw_pair_grad_complete_set_search(int32_t on) {
  TW_ARG_CHECK(on == 0 || on == 1, "tw_pair_grad_complete_set_search: 0 or 1");
  g_hinge_by_search = on;
  g_logistic_one_pass = on;
  return TW_OK;
}

extern "C" int64_t tw_pair_grad_complete_work_bytes(int32_t n_shards, int64_t kx, int64_t kz,
                                                    int64_t d) {
  if (n_shards <= 0 || kx <= 0 || kz <= 0 || d <= 0) return 0;
  return cg_layout(n_shards, kx, kz, d).total * (int64_t)sizeof(double);
}

extern "C" int tw_pair_grad_complete(const double* d_X, const double* d_Z, int64_t d,
                                     const int64_t* d_rows_x, int64_t kx,
                                     const int64_t* d_rows_z, int64_t kz, int32_t n_shards,
                                     const double* d_w, double margin, int32_t loss,
                                     void* d_work, double* d_out, void* stream) {
  TW_ARG_CHECK(d >= 1 && d <= kCgMaxD, "tw_pair_grad_complete: d=%lld outside [1, %d]",
               (long long)d, kCgMaxD);
  TW_ARG_CHECK(n_shards >= 0 && kx >= 1 && kz >= 1, "tw_pair_grad_complete: bad sizes");
  TW_ARG_CHECK(loss == TW_LOSS_HINGE || loss == TW_LOSS_LOGISTIC,
               "tw_pair_grad_complete: unknown loss %d", loss);
  TW_ARG_CHECK((int64_t)n_shards * ceil_div(std::max(kx, kz), kBlock) < (1ll << 31),
               "tw_pair_grad_complete: grid too large");
  if (n_shards == 0) return TW_OK;
  TW_ARG_CHECK(d_X && d_Z && d_w && d_work && d_out, "tw_pair_grad_complete: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const CgLayout l = cg_layout(n_shards, kx, kz, d);
  double* work = (double*)d_work;
  const int64_t nx = (int64_t)n_shards * kx, nz = (int64_t)n_shards * kz;
  const int rs_blocks_x = (int)std::min<int64_t>(256 * 16, ceil_div(nx, kBlock / kWave));
  const int rs_blocks_z = (int)std::min<int64_t>(256 * 16, ceil_div(nz, kBlock / kWave));
  hipLaunchKernelGGL(k_row_scores, dim3(rs_blocks_x), dim3(kBlock), 0, st, d_X, d, d_rows_x,
                     nx, d_w, work + l.sx);
  hipLaunchKernelGGL(k_row_scores, dim3(rs_blocks_z), dim3(kBlock), 0, st, d_Z, d, d_rows_z,
                     nz, d_w, work + l.sz);
  if (loss == TW_LOSS_LOGISTIC && g_logistic_one_pass) {
    TW_ARG_CHECK((int64_t)n_shards * l.lg_tiles < (1ll << 31),
                 "tw_pair_grad_complete: grid too large");
    hipLaunchKernelGGL(k_logistic_coef, dim3(n_shards * l.lg_tiles), dim3(kLgThreads), 0, st,
                       work + l.sx, kx, work + l.sz, kz, margin, l.lg_tiles, work + l.bx,
                       work + l.apart);
    const int fb = (int)std::min<int64_t>(256 * 8, ceil_div((int64_t)n_shards * kz, kBlock));
    hipLaunchKernelGGL(k_apart_final, dim3(fb), dim3(kBlock), 0, st, work + l.apart,
                       (int)n_shards, l.lg_tiles, kz, work + l.az);
  } else if (loss == TW_LOSS_LOGISTIC)
    launch_coef<TW_LOSS_LOGISTIC>(work + l.sx, kx, work + l.sz, kz, n_shards, margin,
                                  work + l.bx, work + l.az, st);
  else if (g_hinge_by_search) {
    const int rc = launch_hinge_coef(work + l.sx, kx, work + l.sz, kz, n_shards, margin, l, work,
                                     work + l.bx, work + l.az, st);
    if (rc != TW_OK) return rc;
  } else
    launch_coef<TW_LOSS_HINGE>(work + l.sx, kx, work + l.sz, kz, n_shards, margin, work + l.bx,
                               work + l.az, st);
  const int ctiles = (int)ceil_div((d & 1) == 0 ? d / 2 : d, kBlock);  // column (pair) tiles
  TW_ARG_CHECK((int64_t)n_shards * l.chunks * ctiles < (1ll << 31),
               "tw_pair_grad_complete: grid too large");
  hipLaunchKernelGGL(k_wcolsum_part, dim3(n_shards * l.chunks * ctiles), dim3(kBlock), 0, st,
                     d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, work + l.bx, work + l.az, l.chunks,
                     ctiles, work + l.part);
  const int fin_blocks = (int)std::min<int64_t>(256 * 8, ceil_div((int64_t)n_shards * d, kBlock));
  hipLaunchKernelGGL(k_wcolsum_final, dim3(fin_blocks), dim3(kBlock), 0, st, work + l.part,
                     (int)n_shards, l.chunks, d, (double)kx * (double)kz, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
