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

// Wide rows (32 < d <= 512): a wave holds one pair's two rows, 8 columns per lane.
constexpr int kWideCols = 8;                     // columns per lane
constexpr int kWideMaxD = kWideCols * kWave;     // 512
constexpr int kIdxPhase = 1024;                  // pairs whose rows are resolved per phase
constexpr int kStreamCH = kWideBlock / kWave;    // 16 pairs per streaming chunk

// csrc/complete_grad.hip: A @ w, one wave per row (lane-strided partial dot + fixed butterfly)
int launch_row_scores(const double* A, int64_t d, int64_t n, const double* w, double* out,
                      hipStream_t st);

}  // namespace tw
