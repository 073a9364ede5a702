// peer.h — the peer buffers of the device-resident gradient exchange between ranks (round 5;
// SURVEY.md §8(e) "Learning": the per-step all-gather of the shard partials, done by the GPUs
// themselves over xGMI instead of by a host-enqueued RCCL collective between two launches).
// Shared by csrc/sgdseg.hip (the narrow persistent segment over ranks) and csrc/peer.hip (the
// buffers, their IPC mapping, and the per-step publish / wait-and-update kernels).
//
// One buffer per rank, allocated uncached (no device's cache keeps a line of it), mapped into
// every other rank through an IPC handle.  Layout (bytes):
//   0    u64 segment arrival counter (monotonic; the persistent segments)
//   64   u64 segment epoch: global steps done by this rank's persistent segments
//   128  u64 per-step counters [2] (128, 192), by step parity (the publish / update launches)
//   256  u64 hello words [16]: rank p's token, written by rank p at setup (tw_peer_hello)
//   384  u64 per-step publication counters [2] (384, 448), by step parity (the column-owned
//        step, tw_peer_step_cols: owners' updated columns of w / dw arrived)
//   512  segment gradient slots [2][n_total][d] f64
//   ...  per-step gradient slots [2][n_total][d] f64
//   ...  per-step publication slots [2][2][d] f64: by parity, w then dw (tw_peer_step_cols)
#pragma once
#include "tw_common.h"

namespace tw {

constexpr size_t kPeerSegCtr = 0, kPeerEpoch = 64, kPeerStepCtr = 128, kPeerHello = 256,
                 kPeerPubCtr = 384, kPeerHdr = 512;

__host__ __device__ inline size_t peer_slots_words(int64_t n_total, int64_t d) {
  return 2 * (size_t)n_total * (size_t)d;
}
__host__ __device__ inline size_t peer_buffer_bytes(int64_t n_total, int64_t d) {
  return kPeerHdr + 2 * sizeof(double) * peer_slots_words(n_total, d) +
         4 * sizeof(double) * (size_t)d;
}

constexpr int kPeerMax = 16;
constexpr uint64_t kPeerSpinTicks = 2000000000ull;  // 20 s: ranks' hosts may drift apart

struct PeerSeg {
  double* slot[kPeerMax];                // rank p's slots [2][n_total][d]
  unsigned long long* ctr[kPeerMax];     // rank p's arrival counter
  unsigned long long* my_ctr;            // this rank's counter, epoch word and slots
  unsigned long long* epoch;
  const double* my_slot;
  int G, n_total;
};

__device__ __forceinline__ double ld_sys(const double* p) {
  const uint64_t v = __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void st_sys(double* p, double v) {
  __hip_atomic_store((uint64_t*)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane: spin until *c >= target (false: aborted or timed out -> abort word raised)
__device__ __forceinline__ bool peer_poll(const unsigned long long* c, uint64_t target,
                                          uint32_t* abort_word) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
        wall_clock64() - t0 > kPeerSpinTicks) {
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}

__device__ __forceinline__ bool peer_wait(const unsigned long long* c, uint64_t target,
                                          uint32_t* abort_word, int* s_ok) {
  if (threadIdx.x == 0) *s_ok = peer_poll(c, target, abort_word) ? 1 : 0;
  __syncthreads();
  return *s_ok != 0;
}

}  // namespace tw
