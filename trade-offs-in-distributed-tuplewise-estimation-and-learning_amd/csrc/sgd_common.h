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

// ---- inter-block hand-offs of the persistent / fused SGD kernels (sgdseg.hip, hinge.hip)
constexpr uint64_t kSegSpinTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ double ld_agent(const double* p) {
  const uint64_t v = __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store((uint64_t*)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// ctl[0]: arrivals (monotonic within a launch, zeroed before it); ctl[1]: abort word, sticky
// (zeroed once by the caller: a later launch that finds it set exits at its first wait).
// Memory-model contract of the grid barrier: every published word is an agent-scope atomic
// store (st_agent); each storing wave waits for its own stores (s_waitcnt vmcnt(0) — the
// block barrier's workgroup-scope release does not wait for another wave's vector stores to
// reach the agent-coherent level), the block barrier orders them before thread 0's arrival,
// and the arrival is an agent-scope RELEASE add (gfx950: buffer_wbl2 sc1 before the atomic).
// The poller spins on RELAXED loads of the counter and, once it has seen the target, issues
// ONE agent-scope ACQUIRE fence (buffer_inv sc1) — acquire loads in the spin itself would
// invalidate the L2 on every iteration; the fence after the last relaxed load that read the
// release's value gives the same synchronisation (fence-atomic rule), and s_waitcnt vmcnt(0)
// holds the block barrier after the poll until the invalidate has completed, so every wave's
// loads of the published words (ld_agent) come after it.
// TW_SEG_BARRIER (A/B builds, tools/ab_barrier.py): 0 = relaxed arrival and spin, no fence
// (round 3); 1 = acquire loads in the spin; 2 (default) = as above.
#ifndef TW_SEG_BARRIER
#define TW_SEG_BARRIER 2
#endif
// arriver: the thread that adds the arrival — the release's L2 write-back (~0.6 us on gfx950)
// stalls only its wave, so the narrow kernel hands it to the last wave, which has no pairs in
// the next step's chain when B <= 192 (C4: B = 100): the stall hides behind the other waves'
// draws -> rows -> diff rows (tools/ab_barrier.py)
__device__ __forceinline__ void seg_arrive(uint32_t* ctl, int arriver = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's published stores landed
  __syncthreads();
  if ((int)threadIdx.x == arriver)
    __hip_atomic_fetch_add(ctl, 1u, TW_SEG_BARRIER ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// one lane: spin until the counter reaches target (false: aborted or timed out -> abort word)
__device__ __forceinline__ bool seg_poll(uint32_t* ctl, uint32_t target) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(ctl, TW_SEG_BARRIER == 1 ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
        wall_clock64() - t0 > kSegSpinTicks) {
      __hip_atomic_store(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (TW_SEG_BARRIER == 2) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // the invalidate completes before the block barrier lets any wave load (the consumer
    // recipe of MI355X_MICROARCH.md: relaxed poll -> acquire -> vmcnt(0) -> barrier -> loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  return true;
}

// the whole block waits (thread 0 polls)
__device__ __forceinline__ bool seg_wait(uint32_t* ctl, uint32_t target, int* s_ok) {
  if (threadIdx.x == 0) *s_ok = seg_poll(ctl, target) ? 1 : 0;
  __syncthreads();
  return *s_ok != 0;
}

}  // namespace tw
