// hinge.hip — pairwise hinge SGD on shards (f1 GEMV).
//
//   grad_inc_block(w, B, margin)   learning-experiment/compute_stats.py:146-162
//       X_sel = X[randint(0,n_X,B)]; Z_sel = Z[randint(0,n_Z,B)]; diff = Z_sel - X_sel
//       S = diff.dot(w) + margin; filt = S > 0; return diff[filt].sum(axis=0) / B
//   UN_split(X_s, Z_s, f)          compute_stats.py:44-46  np.mean([...], axis=0)
//   learning_process update        learning-experiment/make_exps.py:130-141
//
// Numerics (compiled with -ffp-contract=off, like NumPy which never fuses multiply-add):
//   * diff and the column sums are bit-identical to NumPy: the filtered rows are added in
//     row order starting from +0.0, as NumPy's axis-0 add.reduce does (so an empty filter
//     gives +0.0 and a column of -0.0 sums to +0.0, exactly like the reference).
//   * S uses lane-strided partial dots + a fixed butterfly; NumPy uses BLAS dgemv, whose
//     summation order is library-specific.  Only the SIGN of S matters, so the gradient
//     differs from NumPy's only when |S| is within a few ulps of 0 (tolerance 1e-5 rel).
//
// Layout: one block per shard; the block streams its B pairs in chunks of CH pairs whose diff
// rows are staged in LDS (CH*d doubles <= 64 KiB), so every X/Z row is read from HBM once.
#include "sgd_common.h"
#include <algorithm>

// Per-block timestamps of the streaming wide kernel for studies (tools/phase_hinge.py builds
// a separate library with -DTW_HINGE_TIMING; the product build compiles them out): thread 0
// stamps the 100 MHz wall clock at 0 entry, 1 rows resolved, 2 first chunk reduced, 3 exit.
#ifdef TW_HINGE_TIMING
__device__ unsigned long long g_hg_t[1 << 14];
#define HG_STAMP(p)                                                                        \
  do {                                                                                     \
    if (threadIdx.x == 0) g_hg_t[((size_t)blockIdx.x * 4 + (p)) & 0x3FFF] = wall_clock64(); \
  } while (0)
extern "C" int tw_debug_hinge_times(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hg_t), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : 2;
}
#else
#define HG_STAMP(p) \
  do {              \
  } while (0)
#endif

namespace tw {

constexpr int kLdsDoubles = 8192;  // 64 KiB of diff rows per block
constexpr int kMaxColsPerThread = 16;  // d <= 16 * block size
constexpr int kMaxD = 4096;


template <int BS, int LOSS>
__global__ __launch_bounds__(BS) void k_hinge_grad(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz, int64_t B,
    int CH, const double* __restrict__ w, double margin, double* __restrict__ out,
    uint64_t seed, const uint64_t* __restrict__ d_step, uint32_t shard_base,
    double* __restrict__ s_out, SwrMap swr) {
  // s_out (tw_pair_grad_audit): S_b = diff_b . w + margin of every pair, as this kernel
  // computed it, at s_out[s * B + b] — the value whose sign is the hinge filter
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* diff = (double*)smem;                             // CH * d
  int64_t* rx = (int64_t*)(smem + sizeof(double) * CH * d);  // CH
  int64_t* rz = rx + CH;                                     // CH
  double* flag = (double*)(rz + CH);                         // CH pair weights

  const int s = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  double acc[kMaxColsPerThread];
#pragma unroll
  for (int q = 0; q < kMaxColsPerThread; ++q) acc[q] = 0.0;

  const uint64_t step = d_step ? *d_step : 0;
  for (int64_t b0 = 0; b0 < B; b0 += CH) {
    const int nb = (int)std::min<int64_t>(CH, B - b0);
    // rows of this chunk: compose the SWR shard draw with the per-step pair draw
    for (int t = threadIdx.x; t < nb; t += BS) {
      const int64_t p = (int64_t)s * B + b0 + t;
      int64_t ax, az;
      if (ix) {  // replay: NumPy's randint draws
        ax = ix[p];
        az = iz[p];
      } else {  // device RNG
        const u32x4 r = sgd_draw(seed, step, (uint32_t)(b0 + t), shard_base + (uint32_t)s,
                                  kTagPairs);
        ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
        az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
      }
      int64_t rxt, rzt;
      swr_rows_of(swr, rows_x, kx, rows_z, kz, s, shard_base, ax, az, seed, step, rxt, rzt);
      if (d <= 32) {  // narrow rows: this thread stages its own pair right away (no barrier)
        const double* zr = Z + rzt * d;
        const double* xr = X + rxt * d;
        double* dr = diff + (int64_t)t * d;
        double part = 0.0;
#pragma unroll 4
        for (int j = 0; j < (int)d; ++j) {
          const double v = zr[j] - xr[j];
          dr[j] = v;
          part += v * w[j];
        }
        flag[t] = pair_weight<LOSS>(part + margin);
        if (s_out) s_out[p] = part + margin;
      } else {
        rx[t] = rxt;
        rz[t] = rzt;
      }
    }
    __syncthreads();
    // stage diff rows Z[rz] - X[rx] in LDS and reduce S = diff . w + margin on the way.
    // Narrow rows (d <= 32): one thread per pair, sequential j (all row loads independent).
    // Wide rows: one wave per pair, coalesced lane-strided loads + fixed butterfly.
    if (d > 32) for (int t = wid; t < nb; t += BS / kWave) {
      const double* zr = Z + rz[t] * d;
      const double* xr = X + rx[t] * d;
      double* dr = diff + (int64_t)t * d;
      double part = 0.0;
      // batches of 8 lane-strided columns: all 16 row loads in flight before the first use
      for (int64_t j0 = lane; j0 < d; j0 += 8 * kWave) {
        double zv[8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t j = j0 + u * kWave;
          zv[u] = j < d ? zr[j] : 0.0;
          xv[u] = j < d ? xr[j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t j = j0 + u * kWave;
          if (j < d) {
            const double v = zv[u] - xv[u];
            dr[j] = v;
            part += v * w[j];
          }
        }
      }
      part = wave_sum_dpp_f64(part);
      if (lane == 0) flag[t] = pair_weight<LOSS>(part + margin);
      if (lane == 0 && s_out) s_out[(int64_t)s * B + b0 + t] = part + margin;
    }
    __syncthreads();
    // column sums over the filtered rows, in row order
#pragma unroll
    for (int q = 0; q < kMaxColsPerThread; ++q) {
      const int64_t j = threadIdx.x + (int64_t)q * BS;
      if (j < d) {
        // branch-free: an unfiltered row adds -0.0, which leaves every value (incl. +-0.0)
        // bit-identical, so the order and result are NumPy's; 8 LDS reads in flight
        double a = acc[q];
        int t = 0;
        for (; t + 8 <= nb; t += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[t + u], diff[(int64_t)(t + u) * d + j]);
#pragma unroll
          for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; t < nb; ++t) a += weighted<LOSS>(flag[t], diff[(int64_t)t * d + j]);
        acc[q] = a;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < kMaxColsPerThread; ++q) {
    const int64_t j = threadIdx.x + (int64_t)q * BS;
    if (j < d) out[(int64_t)s * d + j] = acc[q] / (double)B;
  }
}

// Wide rows, 32 < d <= 512 (C5: d = 512) — the HBM-bound case, pipelined:
//  * per phase of up to kIdxPhase pairs the block resolves every pair's absolute X/Z row
//    (SWR row table composed with the pair draw) into LDS: one dependent round trip per phase
//    instead of one per chunk;
//  * chunks of kWideCH = 16 waves x kWidePW pairs: a wave holds its pairs' two rows in
//    registers (8 columns per lane), writes diff = Z[rz] - X[rx] to LDS and the filter flag;
//  * the rows of chunk c+1 are loaded right after the barrier, so their HBM latency overlaps
//    chunk c's column sums (thread j adds column j over the filtered rows, in row order).
// Arithmetic and order are those of k_hinge_grad (same lane-strided dot + butterfly, same
// row-order sums from +0.0), so both kernels give identical bits.
constexpr int kWidePW = 2;
constexpr int kWideCH = (kWideBlock / kWave) * kWidePW;  // 32 pairs per chunk

template <int LOSS>
__global__ __launch_bounds__(kWideBlock) void k_hinge_grad_wide(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz, int64_t B,
    const double* __restrict__ w, double margin, double* __restrict__ out, uint64_t seed,
    const uint64_t* __restrict__ d_step, uint32_t shard_base, SwrMap swr) {
  __shared__ double diff[kWideCH * kWideMaxD];  // 128 KiB
  __shared__ int64_t prx[kIdxPhase], prz[kIdxPhase];  // 16 KiB
  __shared__ double flag[kWideCH];  // pair weights
  const int s = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int dd = (int)d;
  const uint64_t step = d_step ? *d_step : 0;
  double wv[kWideCols];
#pragma unroll
  for (int c = 0; c < kWideCols; ++c) {
    const int j = lane + c * kWave;
    wv[c] = j < dd ? w[j] : 0.0;
  }
  double acc = 0.0;  // thread j < d: column j
  double zv[kWidePW][kWideCols], xv[kWidePW][kWideCols];

  for (int64_t P0 = 0; P0 < B; P0 += kIdxPhase) {
    const int np = (int)std::min<int64_t>(kIdxPhase, B - P0);
    __syncthreads();  // the previous phase's readers of prx/prz are done
    for (int t = threadIdx.x; t < np; t += kWideBlock) {
      const int64_t b = P0 + t;
      int64_t ax, az;
      if (ix) {  // replay: NumPy's randint draws
        ax = ix[(int64_t)s * B + b];
        az = iz[(int64_t)s * B + b];
      } else {  // device RNG
        const u32x4 r = sgd_draw(seed, step, (uint32_t)b, shard_base + (uint32_t)s, kTagPairs);
        ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
        az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
      }
      swr_rows_of(swr, rows_x, kx, rows_z, kz, s, shard_base, ax, az, seed, step, prx[t],
                  prz[t]);
    }
    __syncthreads();

    auto load = [&](int c0) {
#pragma unroll
      for (int u = 0; u < kWidePW; ++u) {
        const int t = c0 + wid * kWidePW + u;
        if (t < np) {
          const double* zr = Z + prz[t] * d;
          const double* xr = X + prx[t] * d;
#pragma unroll
          for (int c = 0; c < kWideCols; ++c) {
            const int j = lane + c * kWave;
            zv[u][c] = j < dd ? zr[j] : 0.0;
            xv[u][c] = j < dd ? xr[j] : 0.0;
          }
        }
      }
    };
    load(0);
    for (int c0 = 0; c0 < np; c0 += kWideCH) {
      const int nb = std::min(kWideCH, np - c0);
#pragma unroll
      for (int u = 0; u < kWidePW; ++u) {
        const int t = wid * kWidePW + u;
        if (t < nb) {
          double part = 0.0;
#pragma unroll
          for (int c = 0; c < kWideCols; ++c) {
            const int j = lane + c * kWave;
            if (j < dd) {
              const double v = zv[u][c] - xv[u][c];
              diff[t * dd + j] = v;
              part += v * wv[c];
            }
          }
          part = wave_sum_dpp_f64(part);
          if (lane == 0) flag[t] = pair_weight<LOSS>(part + margin);
        }
      }
      __syncthreads();
      if (c0 + kWideCH < np) load(c0 + kWideCH);  // in flight during the sums below
      if (threadIdx.x < dd) {
        const int j = threadIdx.x;
        double a = acc;
        int t = 0;
        for (; t + 8 <= nb; t += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[t + u], diff[(t + u) * dd + j]);
#pragma unroll
          for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; t < nb; ++t) a += weighted<LOSS>(flag[t], diff[t * dd + j]);
        acc = a;
      }
      __syncthreads();
    }
  }
  if (threadIdx.x < dd) out[(int64_t)s * d + threadIdx.x] = acc / (double)B;
}

// Streaming variant of k_hinge_grad_wide (the default for 32 < d <= 512): one pair per wave
// per chunk (16-pair chunks) and TWO register stages, so the rows of chunks k+1 and k+2 are
// in flight while chunk k is reduced — the loads form a continuous stream instead of one
// 32-pair burst per chunk that drains HBM before the next is issued.  Diff rows and weights are
// double-buffered in LDS (2 x 16 rows): chunk k+1 writes the buffer chunk k-1's sums read,
// which every thread finished before chunk k's barrier.  Same arithmetic and order as
// k_hinge_grad_wide (per pair: lane partial dots over the same 8 columns + the same butterfly;
// column sums in row order), so identical bits.

template <int LOSS>
__global__ __launch_bounds__(kWideBlock) void k_hinge_grad_stream(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz, int64_t B,
    const double* __restrict__ w, double margin, double* __restrict__ out, uint64_t seed,
    const uint64_t* __restrict__ d_step, uint32_t shard_base, SwrMap swr) {
  __shared__ double diff[2][kStreamCH * kWideMaxD];  // 128 KiB
  __shared__ int64_t prx[kIdxPhase], prz[kIdxPhase];  // 16 KiB
  __shared__ double flag[2][kStreamCH];
  const int s = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int dd = (int)d;
  const uint64_t step = d_step ? *d_step : 0;
  double wv[kWideCols];
#pragma unroll
  for (int c = 0; c < kWideCols; ++c) {
    const int j = lane + c * kWave;
    wv[c] = j < dd ? w[j] : 0.0;
  }
  double acc = 0.0;  // thread j < d: column j
  double zv[2][kWideCols], xv[2][kWideCols];

  HG_STAMP(0);
  for (int64_t P0 = 0; P0 < B; P0 += kIdxPhase) {
    const int np = (int)std::min<int64_t>(kIdxPhase, B - P0);
    __syncthreads();  // the previous phase's readers of prx/prz and diff/flag are done
    for (int t = threadIdx.x; t < np; t += kWideBlock) {
      const int64_t b = P0 + t;
      int64_t ax, az;
      if (ix) {
        ax = ix[(int64_t)s * B + b];
        az = iz[(int64_t)s * B + b];
      } else {
        const u32x4 r = sgd_draw(seed, step, (uint32_t)b, shard_base + (uint32_t)s, kTagPairs);
        ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
        az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
      }
      swr_rows_of(swr, rows_x, kx, rows_z, kz, s, shard_base, ax, az, seed, step, prx[t],
                  prz[t]);
    }
    __syncthreads();
    if (P0 == 0) HG_STAMP(1);

    auto load = [&](int st, int c0) {  // this wave's pair of the chunk at c0 into stage st
      const int t = c0 + wid;
      if (t < np) {
        const double* zr = Z + prz[t] * d;
        const double* xr = X + prx[t] * d;
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          zv[st][c] = j < dd ? zr[j] : 0.0;
          xv[st][c] = j < dd ? xr[j] : 0.0;
        }
      }
    };
    auto chunk = [&](int st, int c0) {
      const int nb = std::min(kStreamCH, np - c0);
      const int t = wid;
      if (t < nb) {
        double part = 0.0;
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          if (j < dd) {
            const double v = zv[st][c] - xv[st][c];
            diff[st][t * dd + j] = v;
            part += v * wv[c];
          }
        }
        part = wave_sum_dpp_f64(part);
        if (lane == 0) flag[st][t] = pair_weight<LOSS>(part + margin);
      }
      if (c0 + 2 * kStreamCH < np) load(st, c0 + 2 * kStreamCH);  // refill: chunk k+2
      __syncthreads();
      if (P0 == 0 && c0 == 0) HG_STAMP(2);
      if (threadIdx.x < dd) {
        const int j = threadIdx.x;
        double a = acc;
        int u0 = 0;
        for (; u0 + 8 <= nb; u0 += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[st][u0 + u], diff[st][(u0 + u) * dd + j]);
#pragma unroll
          for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; u0 < nb; ++u0) a += weighted<LOSS>(flag[st][u0], diff[st][u0 * dd + j]);
        acc = a;
      }
    };
    load(0, 0);
    if (kStreamCH < np) load(1, kStreamCH);
    int c0 = 0;
    for (; c0 + kStreamCH < np; c0 += 2 * kStreamCH) {  // stages alternate; constant indices
      chunk(0, c0);
      chunk(1, c0 + kStreamCH);
    }
    if (c0 < np) chunk(0, c0);
  }
  if (threadIdx.x < dd) out[(int64_t)s * d + threadIdx.x] = acc / (double)B;
  HG_STAMP(3);
}

// One whole SGD step for narrow rows (d <= 32, C4) in ONE launch: the update of the PREVIOUS
// step (make_exps.py:130-141) runs as this kernel's prologue, redundantly in every block, and
// then the gradient of this step (compute_stats.py:146-162) with the updated w.
//   * The prologue's loads (the previous step's N x d shard gradients, w, dw) are issued first
//     and the pair chain (draws -> row tables -> rows -> diff rows in LDS) runs while they are in
//     flight; the two dependent chains overlap instead of running in two launches.
//   * Ping-pong buffers: step k reads w/dw/grads of slot (k-1)&1 and writes slot k&1 (block 0
//     writes w/dw), so no block overwrites what another block of the same launch still reads.
//   * Arithmetic is that of k_sgd_update (shard-order sum from +0.0, /N, + reg*w, momentum)
//     followed by k_hinge_grad's narrow path (same diff, same sequential dot, same row-order
//     column sums), so a fused segment gives the bits of grad+update launches.
// grads_in == nullptr: no pending update (the first step of a segment reads w_in as is).
constexpr int kFuseMaxGrads = 4096;                  // N*d staged per block (32 KiB)
constexpr int kFusePerThread = kFuseMaxGrads / kBlock;
constexpr int kFuseMaxD = 32;

template <int LOSS>
__global__ __launch_bounds__(kBlock) void k_sgd_step_narrow(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz, int64_t B,
    int CH, double margin, uint64_t seed, const uint64_t* __restrict__ d_step,
    uint32_t step_off, uint32_t shard_base, int n_shards, const double* __restrict__ w_in,
    const double* __restrict__ dw_in, const double* __restrict__ grads_in, double reg,
    double lr, double momentum, double* __restrict__ w_out, double* __restrict__ dw_out,
    double* __restrict__ grads_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* diff = (double*)smem;    // CH * d
  double* flag = diff + CH * d;    // CH pair weights
  double* wsh = flag + CH;         // kFuseMaxD: this step's w
  double* gt = wsh + kFuseMaxD;    // n_shards * d: the previous step's shard gradients
  const int s = blockIdx.x, tid = threadIdx.x, dd = (int)d;
  const int ng = grads_in ? n_shards * dd : 0;

  double gv[kFusePerThread];  // prologue loads first: in flight during the pair chain
#pragma unroll
  for (int u = 0; u < kFusePerThread; ++u) {
    const int e = tid + u * kBlock;
    gv[u] = e < ng ? grads_in[e] : 0.0;
  }
  double wj = 0.0, dwj = 0.0;
  if (tid < dd) {
    wj = w_in[tid];
    if (grads_in) dwj = dw_in[tid];
  }
  const uint64_t step = (d_step ? *d_step : 0) + step_off;
  double acc = 0.0;  // thread tid < d: column tid

  for (int64_t b0 = 0; b0 < B; b0 += CH) {
    const int nb = (int)std::min<int64_t>(CH, B - b0);
    for (int t = tid; t < nb; t += kBlock) {  // this thread's pair -> its diff row in LDS
      const int64_t p = (int64_t)s * B + b0 + t;
      int64_t ax, az;
      if (ix) {
        ax = ix[p];
        az = iz[p];
      } else {
        const u32x4 r = sgd_draw(seed, step, (uint32_t)(b0 + t), shard_base + (uint32_t)s,
                                 kTagPairs);
        ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
        az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
      }
      const int64_t rxt = rows_x ? rows_x[(int64_t)s * kx + ax] : ax;
      const int64_t rzt = rows_z ? rows_z[(int64_t)s * kz + az] : az;
      const double* zr = Z + rzt * d;
      const double* xr = X + rxt * d;
      double* dr = diff + (int64_t)t * d;
#pragma unroll 4
      for (int j = 0; j < dd; ++j) dr[j] = zr[j] - xr[j];
    }
    if (b0 == 0) {  // prologue: w of this step = update(w, dw, grads of the previous step)
#pragma unroll
      for (int u = 0; u < kFusePerThread; ++u) {
        const int e = tid + u * kBlock;
        if (e < ng) gt[e] = gv[u];
      }
      __syncthreads();
      if (tid < dd) {
        double wt = wj;
        if (grads_in) {
          double sum = 0.0;  // shard order, as np.mean(axis=0) / k_sgd_update
          int r = 0;
          for (; r + 8 <= n_shards; r += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = gt[(r + u) * dd + tid];
#pragma unroll
            for (int u = 0; u < 8; ++u) sum += v[u];
          }
          for (; r < n_shards; ++r) sum += gt[r * dd + tid];
          const double g = sum / (double)n_shards + reg * wj;
          const double st = momentum >= 0.0 ? momentum * dwj + lr * g : lr * g;
          wt = wj - st;
          if (s == 0) {
            w_out[tid] = wt;
            dw_out[tid] = st;
          }
        }
        wsh[tid] = wt;
      }
    }
    __syncthreads();
    for (int t = tid; t < nb; t += kBlock) {  // S = diff . w + margin, sequential j
      const double* dr = diff + (int64_t)t * d;
      double part = 0.0;
      for (int j = 0; j < dd; ++j) part += dr[j] * wsh[j];
      flag[t] = pair_weight<LOSS>(part + margin);
    }
    __syncthreads();
    if (tid < dd) {  // column sums over the filtered rows, in row order (as k_hinge_grad)
      double a = acc;
      int t = 0;
      for (; t + 8 <= nb; t += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[t + u], diff[(t + u) * dd + tid]);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
      }
      for (; t < nb; ++t) a += weighted<LOSS>(flag[t], diff[t * dd + tid]);
      acc = a;
    }
    __syncthreads();
  }
  if (tid < dd) grads_out[(int64_t)s * d + tid] = acc / (double)B;
}

// SWR_divide row draws on the device: rows[s*k + t] uniform in [0, n) (with replacement).
__global__ __launch_bounds__(kBlock) void k_swr_rows(int64_t* __restrict__ rows, int n_shards,
                                                     int64_t k, int64_t n, uint64_t seed,
                                                     const uint64_t* __restrict__ d_step,
                                                     uint32_t tag, uint32_t shard_base) {
  const uint64_t step = *d_step;
  const int64_t total = (int64_t)n_shards * k;
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * kBlock) {
    const int64_t s = e / k, t = e - s * k;
    const u32x4 r = sgd_draw(seed, step, (uint32_t)t, shard_base + (uint32_t)s, tag);
    rows[e] = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)n);
  }
}

// g = (sum_s grads[s]) / N + reg*w ; dw = momentum*dw + lr*g (SGD: dw = lr*g) ; w = w - dw
// d_step (optional): the device-RNG step counter, advanced once per update.
// One block per kUpdCols columns: shard rows are staged in LDS (coalesced), then one thread
// per column adds them in shard order — the sequential order of np.mean(axis=0).
constexpr int kUpdCols = 8;     // d = 512: 64 blocks
constexpr int kUpdRows = 1024;  // shard rows staged per pass: 1024 x 8 doubles = 64 KiB
constexpr int kUpdBatch = 16;   // staging loads in flight per thread
// w_in/dw_in may equal w/dw (in place); step_inc: how far the step counter advances.
__global__ __launch_bounds__(kBlock) void k_sgd_update(const double* w_in, const double* dw_in,
                                                       double* w, double* dw,
                                                       const double* __restrict__ grads,
                                                       int n_shards, int64_t d, double reg,
                                                       double lr, double momentum,
                                                       uint64_t* __restrict__ d_step,
                                                       uint32_t step_inc) {
  __shared__ double tile[kUpdRows * kUpdCols];
  if (d_step && blockIdx.x == 0 && threadIdx.x == 0) *d_step += step_inc;
  const int64_t j0 = (int64_t)blockIdx.x * kUpdCols;
  const int nc = (int)std::min<int64_t>(kUpdCols, d - j0);
  double sum = 0.0;  // thread c < nc: 0.0 + g_0 + g_1 + ... in shard order
  for (int s0 = 0; s0 < n_shards; s0 += kUpdRows) {
    const int ns = std::min(kUpdRows, n_shards - s0);
    __syncthreads();
    // batches of kUpdBatch independent loads per thread, then the LDS stores (a load-store
    // loop waited for every load in turn: 10 us for the C5 update, 256 shards x 512 columns)
    for (int e0 = 0; e0 < ns * kUpdCols; e0 += kBlock * kUpdBatch) {
      double v[kUpdBatch];
#pragma unroll
      for (int u = 0; u < kUpdBatch; ++u) {
        const int e = e0 + u * kBlock + threadIdx.x;
        const int r = e / kUpdCols, c = e - r * kUpdCols;
        v[u] = (e < ns * kUpdCols && c < nc) ? grads[(int64_t)(s0 + r) * d + j0 + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kUpdBatch; ++u) {
        const int e = e0 + u * kBlock + threadIdx.x;
        if (e < ns * kUpdCols) tile[e] = v[u];
      }
    }
    __syncthreads();
    if (threadIdx.x < nc) {  // shard order kept; 4 batches of 8 LDS reads scheduled ahead
      int r = 0;
#pragma unroll 4
      for (; r + 8 <= ns; r += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tile[(r + u) * kUpdCols + threadIdx.x];
#pragma unroll
        for (int u = 0; u < 8; ++u) sum += v[u];
      }
      for (; r < ns; ++r) sum += tile[r * kUpdCols + threadIdx.x];
    }
  }
  if (threadIdx.x < nc) {
    const int64_t j = j0 + threadIdx.x;
    const double wj = w_in[j];
    const double g = sum / (double)n_shards + reg * wj;
    const double step = momentum >= 0.0 ? momentum * dw_in[j] + lr * g : lr * g;
    dw[j] = step;
    w[j] = wj - step;
  }
}

__global__ __launch_bounds__(kBlock) void k_gemv(const double* __restrict__ A, int64_t n,
                                                 int64_t d, const double* __restrict__ w,
                                                 double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const double* row = A + i * d;
    double a = 0.0;
    for (int64_t j = 0; j < d; ++j) a += row[j] * w[j];
    out[i] = a;
  }
}

static int g_hinge_legacy_wide = 0;  // tw_hinge_set_variant: 1 = unpipelined wide kernel

template <int LOSS>
void launch_grad_kernel(const double* X, const double* Z, int64_t d, const int64_t* rows_x,
                        int64_t kx, const int64_t* rows_z, int64_t kz, const int64_t* ix,
                        const int64_t* iz, int32_t n_shards, int64_t B, const double* w,
                        double margin, uint64_t seed, const uint64_t* d_step,
                        uint32_t shard_base, double* out, hipStream_t st,
                        double* s_out = nullptr, SwrMap swr = SwrMap{0, 0, 1, 1}) {
  // per staged pair: d diff doubles + two row indices + one weight, <= 64 KiB in all
  const int CH = (int)std::max<int64_t>(1, std::min<int64_t>(B, kLdsDoubles / (d + 3)));
  const size_t lds = sizeof(double) * CH * d + 2 * sizeof(int64_t) * CH + sizeof(double) * CH;
  if (s_out) {  // audit: the generic kernel (its narrow and wide paths compute S in the same
                // orders as the streaming / fused kernels) with the scores written out
    if (d <= 32)
      hipLaunchKernelGGL((k_hinge_grad<kBlock, LOSS>), dim3(n_shards), dim3(kBlock), lds, st, X,
                         Z, d, rows_x, kx, rows_z, kz, ix, iz, B, CH, w, margin, out, seed,
                         d_step, shard_base, s_out, swr);
    else
      hipLaunchKernelGGL((k_hinge_grad<kWideBlock, LOSS>), dim3(n_shards), dim3(kWideBlock), lds,
                         st, X, Z, d, rows_x, kx, rows_z, kz, ix, iz, B, CH, w, margin, out,
                         seed, d_step, shard_base, s_out, swr);
    return;
  }
  if (d <= 32)
    hipLaunchKernelGGL((k_hinge_grad<kBlock, LOSS>), dim3(n_shards), dim3(kBlock), lds, st, X, Z,
                       d, rows_x, kx, rows_z, kz, ix, iz, B, CH, w, margin, out, seed, d_step,
                       shard_base, nullptr, swr);
  else if (d <= kWideMaxD && g_hinge_legacy_wide == 0)
    hipLaunchKernelGGL(k_hinge_grad_stream<LOSS>, dim3(n_shards), dim3(kWideBlock), 0, st, X, Z,
                       d, rows_x, kx, rows_z, kz, ix, iz, B, w, margin, out, seed, d_step,
                       shard_base, swr);
  else if (d <= kWideMaxD && g_hinge_legacy_wide == 2)
    hipLaunchKernelGGL(k_hinge_grad_wide<LOSS>, dim3(n_shards), dim3(kWideBlock), 0, st, X, Z, d,
                       rows_x, kx, rows_z, kz, ix, iz, B, w, margin, out, seed, d_step,
                       shard_base, swr);
  else
    hipLaunchKernelGGL((k_hinge_grad<kWideBlock, LOSS>), dim3(n_shards), dim3(kWideBlock), lds, st,
                       X, Z, d, rows_x, kx, rows_z, kz, ix, iz, B, CH, w, margin, out, seed,
                       d_step, shard_base, nullptr, swr);
}

int launch_hinge(const double* X, const double* Z, int64_t d, const int64_t* rows_x, int64_t kx,
                 const int64_t* rows_z, int64_t kz, const int64_t* ix, const int64_t* iz,
                 int32_t n_shards, int64_t B, const double* w, double margin, uint64_t seed,
                 const uint64_t* d_step, uint32_t shard_base, double* out, hipStream_t st,
                 int32_t loss = TW_LOSS_HINGE, double* s_out = nullptr,
                 SwrMap swr = SwrMap{0, 0, 1, 1}) {
  if (loss == TW_LOSS_LOGISTIC)
    launch_grad_kernel<TW_LOSS_LOGISTIC>(X, Z, d, rows_x, kx, rows_z, kz, ix, iz, n_shards, B, w,
                                         margin, seed, d_step, shard_base, out, st, s_out, swr);
  else
    launch_grad_kernel<TW_LOSS_HINGE>(X, Z, d, rows_x, kx, rows_z, kz, ix, iz, n_shards, B, w,
                                      margin, seed, d_step, shard_base, out, st, s_out, swr);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

}  // namespace tw

using namespace tw;

static int check_loss(int32_t loss) {
  TW_ARG_CHECK(loss == TW_LOSS_HINGE || loss == TW_LOSS_LOGISTIC, "unknown loss %d", loss);
  return TW_OK;
}

extern "C" int tw_pair_grad(const double* d_X, const double* d_Z, int64_t d,
                            const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                            int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                            int32_t n_shards, int64_t B, const double* d_w, double margin,
                            int32_t loss, double* d_out, void* stream) {
  TW_ARG_CHECK(d >= 1 && d <= kMaxD, "tw_hinge_grad: d=%lld outside [1, %d]", (long long)d, kMaxD);
  TW_ARG_CHECK(n_shards >= 0 && B >= 1, "tw_hinge_grad: bad n_shards/B");
  if (int rc = check_loss(loss)) return rc;
  if (n_shards == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  TW_ARG_CHECK(d_ix != nullptr && d_iz != nullptr, "tw_hinge_grad: pair indices required");
  return launch_hinge(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, n_shards, B, d_w,
                      margin, 0, nullptr, 0, d_out, st, loss);
}

extern "C" int tw_pair_grad_audit(const double* d_X, const double* d_Z, int64_t d,
                                  const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                                  int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                                  int32_t n_shards, int64_t B, const double* d_w, double margin,
                                  int32_t loss, double* d_out, double* d_scores, void* stream) {
  TW_ARG_CHECK(d >= 1 && d <= kMaxD, "tw_pair_grad_audit: d=%lld outside [1, %d]", (long long)d,
               kMaxD);
  TW_ARG_CHECK(n_shards >= 0 && B >= 1 && d_scores != nullptr, "tw_pair_grad_audit: bad args");
  TW_ARG_CHECK(d_ix != nullptr && d_iz != nullptr, "tw_pair_grad_audit: pair indices required");
  if (int rc = check_loss(loss)) return rc;
  if (n_shards == 0) return TW_OK;
  return launch_hinge(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, n_shards, B, d_w,
                      margin, 0, nullptr, 0, d_out, (hipStream_t)stream, loss, d_scores);
}

extern "C" int tw_hinge_grad(const double* d_X, const double* d_Z, int64_t d,
                             const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                             int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                             int32_t n_shards, int64_t B, const double* d_w, double margin,
                             double* d_out, void* stream) {
  return tw_pair_grad(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, n_shards, B, d_w,
                      margin, TW_LOSS_HINGE, d_out, stream);
}

// Replay draws arrive narrowed to uint16 / uint8 (tw_np_randint_pairs_steps_u16 / _u8): widened
// here, in stream order, into the int64 buffer the segment graphs read.  The source is usually
// pinned host memory read in place over PCIe, so every lane reads 16 B (8 or 16 indices): few,
// wide requests; a tail of < 16 B (or a misaligned source) goes element by element.
template <typename T>
static __global__ __launch_bounds__(256) void k_widen(const T* __restrict__ in, int64_t n,
                                                      int64_t* __restrict__ out) {
  constexpr int kPer = 16 / (int)sizeof(T);
  const bool vec = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  const int64_t nv = vec ? n / kPer : 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += stride) {
    const uint4 v = reinterpret_cast<const uint4*>(in)[i];
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int k = 0; k < kPer; ++k) out[i * kPer + k] = (int64_t)e[k];
  }
  for (int64_t i = nv * kPer + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    out[i] = (int64_t)in[i];
}

template <typename T>
static int widen(const T* d_in, int64_t n, int64_t* d_out, void* stream) {
  if (n == 0) return TW_OK;
  const unsigned g = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, ceil_div(n, 256 * (16 / (int64_t)sizeof(T)))));
  hipLaunchKernelGGL(k_widen<T>, dim3(g), dim3(256), 0, (hipStream_t)stream, d_in, n, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_widen_u16(const uint16_t* d_in, int64_t n, int64_t* d_out, void* stream) {
  TW_ARG_CHECK(n >= 0, "tw_widen_u16: n < 0");
  return widen(d_in, n, d_out, stream);
}

extern "C" int tw_widen_u8(const uint8_t* d_in, int64_t n, int64_t* d_out, void* stream) {
  TW_ARG_CHECK(n >= 0, "tw_widen_u8: n < 0");
  return widen(d_in, n, d_out, stream);
}

// The replay loop's per-segment upload in ONE launch: blocks [0, gw) widen the narrowed draws
// (as k_widen), the rest copy a reshuffle's SWR row tables (nx words to rows_x, then nz to
// rows_z, from one source) — both sources usually pinned host memory read over PCIe.  One
// launch instead of three: each launch on the segment's critical path costs its own gap.
template <typename T>
static __global__ __launch_bounds__(256) void k_ship(const T* __restrict__ in, int64_t n,
                                                     int64_t* __restrict__ out,
                                                     const uint64_t* __restrict__ rin,
                                                     int64_t nx, uint64_t* __restrict__ rx,
                                                     int64_t nz, uint64_t* __restrict__ rz,
                                                     int gw) {
  if ((int)blockIdx.x < gw) {
    constexpr int kPer = 16 / (int)sizeof(T);
    const int64_t nv = (reinterpret_cast<uintptr_t>(in) & 15) == 0 ? n / kPer : 0;
    const int64_t stride = (int64_t)gw * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += stride) {
      const uint4 v = reinterpret_cast<const uint4*>(in)[i];
      const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int k = 0; k < kPer; ++k) out[i * kPer + k] = (int64_t)e[k];
    }
    for (int64_t i = nv * kPer + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = (int64_t)in[i];
    return;
  }
  const int64_t stride = (int64_t)(gridDim.x - gw) * 256;
  for (int64_t i = (int64_t)(blockIdx.x - gw) * 256 + threadIdx.x; i < nx + nz; i += stride) {
    const uint64_t v = rin[i];
    if (i < nx)
      rx[i] = v;
    else
      rz[i - nx] = v;
  }
}

extern "C" int tw_ship_draws(const void* d_in, int32_t width, int64_t n, int64_t* d_out,
                             const void* d_rows, int64_t nx, int64_t* d_rows_x, int64_t nz,
                             int64_t* d_rows_z, void* stream) {
  TW_ARG_CHECK(width == 1 || width == 2, "tw_ship_draws: width must be 1 or 2");
  TW_ARG_CHECK(n >= 0 && nx >= 0 && nz >= 0, "tw_ship_draws: negative size");
  TW_ARG_CHECK(n == 0 || (d_in != nullptr && d_out != nullptr), "tw_ship_draws: null draws");
  TW_ARG_CHECK(nx + nz == 0 || (d_rows != nullptr && (nx == 0 || d_rows_x != nullptr) &&
                                (nz == 0 || d_rows_z != nullptr)),
               "tw_ship_draws: null row tables");
  const int64_t per = 256 * (16 / (int64_t)width);
  const int gw = n > 0 ? (int)std::min<int64_t>(1024, ceil_div(n, per)) : 0;
  const int gr = nx + nz > 0 ? (int)std::min<int64_t>(256, ceil_div(nx + nz, 256)) : 0;
  if (gw + gr == 0) return TW_OK;
  if (width == 1)
    hipLaunchKernelGGL(k_ship<uint8_t>, dim3(gw + gr), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, n, d_out, (const uint64_t*)d_rows, nx,
                       (uint64_t*)d_rows_x, nz, (uint64_t*)d_rows_z, gw);
  else
    hipLaunchKernelGGL(k_ship<uint16_t>, dim3(gw + gr), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)d_in, n, d_out, (const uint64_t*)d_rows, nx,
                       (uint64_t*)d_rows_x, nz, (uint64_t*)d_rows_z, gw);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// A replay segment through reshuffles: its narrowed pair draws widened (as k_ship) and ntab row
// tables, laid out [x rows | z rows] per table in the mapped pinned buffer, into consecutive
// tables of the device stacks (x tables nx words apart, z tables nz apart), in one launch.
template <typename T, typename R>
static __global__ __launch_bounds__(256) void k_ship_tables(
    const T* __restrict__ in, int64_t n, int64_t* __restrict__ out,
    const R* __restrict__ rows, int ntab, int64_t nx, int64_t* __restrict__ rows_x,
    int64_t nz, int64_t* __restrict__ rows_z, int gw) {
  if ((int)blockIdx.x < gw) {
    constexpr int U = 16 / (int)sizeof(T);
    const int64_t nv = n / U;
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nv;
         v += (int64_t)gw * 256) {
      const uint4 q = ((const uint4*)in)[v];
      const T* e = (const T*)&q;
#pragma unroll
      for (int u = 0; u < U; ++u) out[v * U + u] = (int64_t)e[u];
    }
    for (int64_t i = nv * U + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gw * 256)
      out[i] = (int64_t)in[i];
    return;
  }
  const int64_t per = nx + nz, tot = per * ntab;
  for (int64_t i = (int64_t)(blockIdx.x - gw) * 256 + threadIdx.x; i < tot;
       i += (int64_t)(gridDim.x - gw) * 256) {
    const int64_t t = i / per, j = i - t * per;
    const int64_t v = (int64_t)rows[i];
    if (j < nx)
      rows_x[t * nx + j] = v;
    else
      rows_z[t * nz + (j - nx)] = v;
  }
}

template <typename R>
static void ship_tables_launch(const void* d_in, int32_t width, int64_t n, int64_t* d_out,
                               const void* d_rows, int32_t ntab, int64_t nx, int64_t* d_rows_x,
                               int64_t nz, int64_t* d_rows_z, int gw, int gr, hipStream_t st) {
  if (width == 1)
    hipLaunchKernelGGL((k_ship_tables<uint8_t, R>), dim3(gw + gr), dim3(256), 0, st,
                       (const uint8_t*)d_in, n, d_out, (const R*)d_rows, (int)ntab, nx,
                       d_rows_x, nz, d_rows_z, gw);
  else
    hipLaunchKernelGGL((k_ship_tables<uint16_t, R>), dim3(gw + gr), dim3(256), 0, st,
                       (const uint16_t*)d_in, n, d_out, (const R*)d_rows, (int)ntab, nx,
                       d_rows_x, nz, d_rows_z, gw);
}

extern "C" int tw_ship_draws_tables(const void* d_in, int32_t width, int64_t n, int64_t* d_out,
                                    const void* d_rows, int32_t row_width, int32_t ntab,
                                    int64_t nx, int64_t* d_rows_x, int64_t nz,
                                    int64_t* d_rows_z, void* stream) {
  TW_ARG_CHECK(width == 1 || width == 2, "tw_ship_draws_tables: width must be 1 or 2");
  TW_ARG_CHECK(row_width == 2 || row_width == 8, "tw_ship_draws_tables: row_width 2 or 8");
  TW_ARG_CHECK(n >= 0 && nx >= 0 && nz >= 0 && ntab >= 0, "tw_ship_draws_tables: negative size");
  TW_ARG_CHECK(n == 0 || (d_in != nullptr && d_out != nullptr), "tw_ship_draws_tables: draws");
  TW_ARG_CHECK(ntab == 0 || nx + nz == 0 ||
                   (d_rows != nullptr && d_rows_x != nullptr && d_rows_z != nullptr),
               "tw_ship_draws_tables: null row tables");
  const int64_t per = 256 * (16 / (int64_t)width);
  const int gw = n > 0 ? (int)std::min<int64_t>(1024, ceil_div(n, per)) : 0;
  const int64_t tot = (nx + nz) * ntab;
  const int gr = tot > 0 ? (int)std::min<int64_t>(512, ceil_div(tot, 256)) : 0;
  if (gw + gr == 0) return TW_OK;
  if (row_width == 2)
    ship_tables_launch<uint16_t>(d_in, width, n, d_out, d_rows, ntab, nx, d_rows_x, nz,
                                 d_rows_z, gw, gr, (hipStream_t)stream);
  else
    ship_tables_launch<uint64_t>(d_in, width, n, d_out, d_rows, ntab, nx, d_rows_x, nz,
                                 d_rows_z, gw, gr, (hipStream_t)stream);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// 8-byte words from a (host-mapped) staging buffer into device memory: the replay loop's SWR
// row tables, read by the kernel straight from pinned host memory.
static __global__ __launch_bounds__(256) void k_copy_words(const uint64_t* __restrict__ in,
                                                           int64_t n, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = in[i];
}

extern "C" int tw_copy_words(const void* d_in, int64_t n, void* d_out, void* stream) {
  TW_ARG_CHECK(n >= 0, "tw_copy_words: n < 0");
  if (n == 0) return TW_OK;
  const unsigned g = (unsigned)std::min<int64_t>(1024, ceil_div(n, 256));
  hipLaunchKernelGGL(k_copy_words, dim3(g), dim3(256), 0, (hipStream_t)stream,
                     (const uint64_t*)d_in, n, (uint64_t*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// One evaluation's results of the learning loop into its pinned host slot in ONE launch (vector
// stores into host-mapped memory, read after the launch's event): the nres statistics, the nw
// words of w and, when ctl is not null, the engine's abort word — instead of three DMA copies
// of a few words each (~4.6 us apiece on the stream).
static __global__ __launch_bounds__(64) void k_stage_eval(const uint64_t* __restrict__ res,
                                                          int nres, const uint64_t* __restrict__ w,
                                                          int nw, const uint32_t* __restrict__ ctl,
                                                          uint64_t* __restrict__ out) {
  for (int i = threadIdx.x; i < nres + nw + 1; i += 64) {
    if (i < nres)
      out[i] = res[i];
    else if (i < nres + nw)
      out[i] = w[i - nres];
    else if (ctl != nullptr)
      out[i] = (uint64_t)ctl[0];
  }
}

extern "C" int tw_stage_eval(const void* d_res, int32_t nres, const void* d_w, int32_t nw,
                             const uint32_t* d_ctl, void* h_out, void* stream) {
  TW_ARG_CHECK(nres >= 0 && nw >= 0 && h_out != nullptr, "tw_stage_eval: bad arguments");
  hipLaunchKernelGGL(k_stage_eval, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const uint64_t*)d_res, (int)nres, (const uint64_t*)d_w, (int)nw, d_ctl,
                     (uint64_t*)h_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_hinge_set_variant(int32_t legacy_wide) {
  TW_ARG_CHECK(legacy_wide >= 0 && legacy_wide <= 2, "tw_hinge_set_variant: 0, 1 or 2");
  g_hinge_legacy_wide = legacy_wide;
  return TW_OK;
}

extern "C" int tw_pair_grad_rng(const double* d_X, const double* d_Z, int64_t d,
                                const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                                int64_t kz, int32_t n_shards, int64_t B, const double* d_w,
                                double margin, int32_t loss, uint64_t seed,
                                const uint64_t* d_step, int32_t shard_base, double* d_out,
                                void* stream) {
  TW_ARG_CHECK(d >= 1 && d <= kMaxD, "tw_hinge_grad_rng: d=%lld outside [1, %d]", (long long)d,
               kMaxD);
  TW_ARG_CHECK(n_shards >= 0 && B >= 1 && B < (1ll << 32) && kx >= 1 && kz >= 1,
               "tw_hinge_grad_rng: bad n_shards/B/kx/kz");
  TW_ARG_CHECK(d_step != nullptr, "tw_hinge_grad_rng: step counter required");
  if (int rc = check_loss(loss)) return rc;
  if (n_shards == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  TW_ARG_CHECK(shard_base >= 0, "tw_hinge_grad_rng: shard_base < 0");
  return launch_hinge(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, nullptr, nullptr, n_shards, B,
                      d_w, margin, seed, d_step, (uint32_t)shard_base, d_out, st, loss);
}

extern "C" int tw_pair_grad_rng_swr(const double* d_X, const double* d_Z, int64_t d,
                                    int64_t n_X, int64_t n_Z, int64_t kx, int64_t kz,
                                    int32_t n_shards, int64_t B, const double* d_w,
                                    double margin, int32_t loss, uint64_t seed,
                                    const uint64_t* d_step, int32_t shard_base, int64_t swr_mod,
                                    uint64_t swr_base, double* d_out, void* stream) {
  TW_ARG_CHECK(d >= 1 && d <= kMaxD, "tw_pair_grad_rng_swr: d=%lld outside [1, %d]",
               (long long)d, kMaxD);
  TW_ARG_CHECK(n_shards >= 0 && B >= 1 && B < (1ll << 32) && kx >= 1 && kz >= 1 &&
                   n_X >= 1 && n_Z >= 1 && swr_mod >= 1 && shard_base >= 0,
               "tw_pair_grad_rng_swr: bad sizes");
  TW_ARG_CHECK(d_step != nullptr, "tw_pair_grad_rng_swr: step counter required");
  if (int rc = check_loss(loss)) return rc;
  if (n_shards == 0) return TW_OK;
  return launch_hinge(d_X, d_Z, d, nullptr, kx, nullptr, kz, nullptr, nullptr, n_shards, B, d_w,
                      margin, seed, d_step, (uint32_t)shard_base, d_out, (hipStream_t)stream,
                      loss, nullptr, SwrMap{(uint64_t)swr_mod, swr_base, n_X, n_Z});
}

extern "C" int tw_hinge_grad_rng(const double* d_X, const double* d_Z, int64_t d,
                                 const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                                 int64_t kz, int32_t n_shards, int64_t B, const double* d_w,
                                 double margin, uint64_t seed, const uint64_t* d_step,
                                 int32_t shard_base, double* d_out, void* stream) {
  return tw_pair_grad_rng(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, n_shards, B, d_w, margin,
                          TW_LOSS_HINGE, seed, d_step, shard_base, d_out, stream);
}

extern "C" int tw_swr_rows_rng(int64_t* d_rows, int32_t n_shards, int64_t k, int64_t n,
                               uint64_t seed, const uint64_t* d_step, int32_t side,
                               int32_t shard_base, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && k >= 0 && n >= 1 && k < (1ll << 32) && d_step != nullptr,
               "tw_swr_rows_rng: bad sizes");
  TW_ARG_CHECK(side == 0 || side == 1, "tw_swr_rows_rng: side must be 0 (X) or 1 (Z)");
  const int64_t total = (int64_t)n_shards * k;
  if (total == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 8, ceil_div(total, kBlock));
  hipLaunchKernelGGL(k_swr_rows, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, d_rows,
                     (int)n_shards, k, n, seed, d_step, side == 0 ? kTagRowsX : kTagRowsZ,
                     (uint32_t)shard_base);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_sgd_update(double* d_w, double* d_dw, const double* d_grads, int32_t n_shards,
                             int64_t d, double reg, double lr, double momentum, uint64_t* d_step,
                             void* stream) {
  TW_ARG_CHECK(n_shards >= 1 && d >= 1, "tw_sgd_update: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)ceil_div(d, kUpdCols);
  hipLaunchKernelGGL(k_sgd_update, dim3(blocks), dim3(kBlock), 0, st, d_w, d_dw, d_w, d_dw,
                     d_grads, n_shards, d, reg, lr, momentum, d_step, 1u);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_sgd_update_to(const double* d_w_in, const double* d_dw_in, double* d_w,
                                double* d_dw, const double* d_grads, int32_t n_shards, int64_t d,
                                double reg, double lr, double momentum, uint64_t* d_step,
                                int32_t step_inc, void* stream) {
  TW_ARG_CHECK(n_shards >= 1 && d >= 1 && step_inc >= 0, "tw_sgd_update_to: bad sizes");
  const int blocks = (int)ceil_div(d, kUpdCols);
  hipLaunchKernelGGL(k_sgd_update, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, d_w_in,
                     d_dw_in, d_w, d_dw, d_grads, n_shards, d, reg, lr, momentum, d_step,
                     (uint32_t)step_inc);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_sgd_step_fusable(int64_t d, int32_t n_shards) {
  return d >= 1 && d <= kFuseMaxD && n_shards >= 1 && (int64_t)n_shards * d <= kFuseMaxGrads;
}

extern "C" int tw_sgd_step(const double* d_X, const double* d_Z, int64_t d,
                           const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                           int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                           int32_t n_shards, int64_t B, double margin, int32_t loss,
                           uint64_t seed, const uint64_t* d_step, int32_t step_off,
                           int32_t shard_base, const double* d_w_in, const double* d_dw_in,
                           const double* d_grads_in, double reg, double lr, double momentum,
                           double* d_w_out, double* d_dw_out, double* d_grads_out,
                           void* stream) {
  TW_ARG_CHECK(tw_sgd_step_fusable(d, n_shards), "tw_sgd_step: d=%lld, n_shards=%d not fusable",
               (long long)d, n_shards);
  TW_ARG_CHECK(B >= 1 && B < (1ll << 32) && kx >= 1 && kz >= 1 && step_off >= 0 &&
                   shard_base >= 0, "tw_sgd_step: bad B/kx/kz/step_off/shard_base");
  TW_ARG_CHECK((d_ix == nullptr) == (d_iz == nullptr), "tw_sgd_step: ix and iz go together");
  TW_ARG_CHECK(d_ix != nullptr || d_step != nullptr, "tw_sgd_step: device draws need d_step");
  TW_ARG_CHECK(d_grads_in == nullptr || (d_dw_in != nullptr && d_w_out != nullptr &&
                                         d_dw_out != nullptr),
               "tw_sgd_step: a pending update needs dw_in, w_out, dw_out");
  if (int rc = check_loss(loss)) return rc;
  // diff rows + weights + w + the staged shard gradients within 64 KiB
  const int64_t room = kLdsDoubles - kFuseMaxD - (int64_t)n_shards * d;  // >= 4064
  const int CH = (int)std::max<int64_t>(1, std::min<int64_t>(B, room / (d + 1)));
  const size_t lds = sizeof(double) * ((size_t)CH * d + CH + kFuseMaxD + (size_t)n_shards * d);
  hipStream_t st = (hipStream_t)stream;
  if (loss == TW_LOSS_LOGISTIC)
    hipLaunchKernelGGL(k_sgd_step_narrow<TW_LOSS_LOGISTIC>, dim3(n_shards), dim3(kBlock), lds, st,
                       d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, B, CH, margin, seed,
                       d_step, (uint32_t)step_off, (uint32_t)shard_base, (int)n_shards, d_w_in,
                       d_dw_in, d_grads_in, reg, lr, momentum, d_w_out, d_dw_out, d_grads_out);
  else
    hipLaunchKernelGGL(k_sgd_step_narrow<TW_LOSS_HINGE>, dim3(n_shards), dim3(kBlock), lds, st,
                       d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, B, CH, margin, seed,
                       d_step, (uint32_t)step_off, (uint32_t)shard_base, (int)n_shards, d_w_in,
                       d_dw_in, d_grads_in, reg, lr, momentum, d_w_out, d_dw_out, d_grads_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

static int g_gemv_rows = 1;  // tw_gemv_set_variant: 1 = wave per row for d > 32

extern "C" int tw_gemv_set_variant(int32_t rows) {
  TW_ARG_CHECK(rows == 0 || rows == 1, "tw_gemv_set_variant: 0 or 1");
  g_gemv_rows = rows;
  return TW_OK;
}

extern "C" int tw_gemv_f64(const double* d_A, int64_t n, int64_t d, const double* d_w,
                           double* d_out, void* stream) {
  TW_ARG_CHECK(n >= 0 && d >= 1, "tw_gemv_f64: bad sizes");
  if (n == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  // wide rows: one wave per row, coalesced 16-B loads (a thread per row reads 64 rows per wave
  // instruction, one line each); rows must be 16-B aligned for the double2 loads
  if (d > 32 && g_gemv_rows && ((uintptr_t)d_A & 15) == 0 && ((uintptr_t)d_w & 15) == 0)
    return launch_row_scores(d_A, d, n, d_w, d_out, st);
  const int blocks = (int)std::min<int64_t>(4096, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_gemv, dim3(blocks), dim3(kBlock), 0, st, d_A, n, d, d_w, d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
