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
//   k_pair_coef      thread per point, the other side's scores staged in LDS chunks; the
//                    point's coefficient is summed in the other side's index order
//   k_wcolsum_part   thread per column, 256-row chunks of [Z rows (+a) | X rows (-b)] in order
//   k_wcolsum_final  chunk partials added in chunk order, / (kx kz)
#include "tw_common.h"
#include <algorithm>

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
  for (int64_t r = ((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave; r < total; r += waves) {
    const double* a = A + (rows ? rows[r] : r) * d;
    double p = 0.0;
    for (int64_t j = lane; j < d; j += kWave) p += a[j] * w[j];
    p = wave_sum_f64(p);
    if (lane == 0) out[r] = p;
  }
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
  const int64_t col = (int64_t)(rem - c * ctiles) * kBlock + threadIdx.x;
  if (col >= d) return;
  const int64_t r0 = (int64_t)c * kColRows, r1 = std::min<int64_t>(r0 + kColRows, kx + kz);
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
  int64_t sx, sz, bx, az, part;  // offsets (doubles) into the workspace
  int64_t total;
  int chunks;
};

static CgLayout cg_layout(int32_t n_shards, int64_t kx, int64_t kz, int64_t d) {
  CgLayout l;
  const int64_t nx = (int64_t)n_shards * kx, nz = (int64_t)n_shards * kz;
  l.chunks = (int)std::max<int64_t>(1, ceil_div(kx + kz, kColRows));
  l.sx = 0;
  l.sz = l.sx + nx;
  l.bx = l.sz + nz;
  l.az = l.bx + nx;
  l.part = l.az + nz;
  l.total = l.part + (int64_t)n_shards * l.chunks * d;
  return l;
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

}  // namespace tw

using namespace tw;

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
  if (loss == TW_LOSS_LOGISTIC)
    launch_coef<TW_LOSS_LOGISTIC>(work + l.sx, kx, work + l.sz, kz, n_shards, margin,
                                  work + l.bx, work + l.az, st);
  else
    launch_coef<TW_LOSS_HINGE>(work + l.sx, kx, work + l.sz, kz, n_shards, margin, work + l.bx,
                               work + l.az, st);
  const int ctiles = (int)ceil_div(d, kBlock);
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
