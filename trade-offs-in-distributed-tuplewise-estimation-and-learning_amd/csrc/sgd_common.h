// sgd_common.h — constants and draws shared by the SGD gradient kernels (hinge.hip) and the
// persistent segment kernel (sgdseg.hip).
#pragma once
#include "tw_common.h"

namespace tw {

constexpr int kWideBlock = 1024;  // d > 32: 16 waves = 16 diff rows in flight per CU

// Device-RNG mode counters: Philox4x32-10 keyed by the run's seed; counter words
// (index, shard, step lo, tag | step hi).  Tags separate the three draw streams.
constexpr uint32_t kTagPairs = 0x80000000u, kTagRowsX = 0x40000000u, kTagRowsZ = 0x20000000u;

__device__ __forceinline__ u32x4 sgd_draw(uint64_t seed, uint64_t step, uint32_t idx,
                                          uint32_t shard, uint32_t tag) {
  return philox4x32_10(u32x4{idx, shard, (uint32_t)step, tag | (uint32_t)(step >> 32)},
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Device-RNG SWR rows drawn IN the gradient kernel (round 3): with reshuffles every `mod` steps
// from counter `base`, the row of draw position a in shard s at step counter c is the one
// k_swr_rows drew at the last reshuffle, counter c - (c - base) % mod — one Philox block per
// side instead of a table read, and no table-drawing launch per reshuffle.  mod == 0: tables.
struct SwrMap {
  uint64_t mod, base;
  int64_t n_x, n_z;
};

// rows of pair (ax, az) of local shard s (global shard_base + s) at step counter `step`
__device__ __forceinline__ void swr_rows_of(const SwrMap& m, const int64_t* __restrict__ rows_x,
                                            int64_t kx, const int64_t* __restrict__ rows_z,
                                            int64_t kz, int s, uint32_t shard_base, int64_t ax,
                                            int64_t az, uint64_t seed, uint64_t step,
                                            int64_t& rx, int64_t& rz) {
  if (m.mod) {
    const uint64_t rc = step - (step - m.base) % m.mod;
    const u32x4 qx = sgd_draw(seed, rc, (uint32_t)ax, shard_base + (uint32_t)s, kTagRowsX);
    const u32x4 qz = sgd_draw(seed, rc, (uint32_t)az, shard_base + (uint32_t)s, kTagRowsZ);
    rx = (int64_t)mulhi_u64(((uint64_t)qx.b << 32) | qx.a, (uint64_t)m.n_x);
    rz = (int64_t)mulhi_u64(((uint64_t)qz.b << 32) | qz.a, (uint64_t)m.n_z);
  } else {
    rx = rows_x ? rows_x[(int64_t)s * kx + ax] : ax;
    rz = rows_z ? rows_z[(int64_t)s * kz + az] : az;
  }
}

// Wide rows (32 < d <= 512): a wave holds one pair's two rows, 8 columns per lane.
constexpr int kWideCols = 8;                     // columns per lane
constexpr int kWideMaxD = kWideCols * kWave;     // 512
constexpr int kIdxPhase = 1024;                  // pairs whose rows are resolved per phase
constexpr int kStreamCH = kWideBlock / kWave;    // 16 pairs per streaming chunk

// csrc/complete_grad.hip: A @ w, one wave per row (lane-strided partial dot + fixed butterfly)
int launch_row_scores(const double* A, int64_t d, int64_t n, const double* w, double* out,
                      hipStream_t st);

}  // namespace tw
