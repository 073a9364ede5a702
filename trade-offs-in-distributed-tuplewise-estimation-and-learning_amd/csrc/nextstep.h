// nextstep.h — the next repartition of est.UnNT's loop carried by spare blocks of a count launch
// (k_count_complete via tw_count_pairs_step): the keyed permutation of both samples as a
// gather and the zeroing of the next step's counters.  (The device-RNG image count carries the
// same gathers in its count threads instead — csrc/imagecount.hip NextSlice — since its LDS
// footprint leaves no room for spare blocks beside its own.)
#pragma once
#include "feistel.h"

namespace tw {

// Carried by `blocks` spare blocks of a count launch: the permutation of both samples as a gather (tw_permute_pair)
// and the zeroing of the next step's counters.  These blocks are memory-latency bound and
// share the CUs with the VALU-bound count blocks, so the repartition costs no separate
// kernel, no launch gap and almost no time.
struct NextStep {
  const uint64_t* x_in;
  uint64_t* x_out;
  int64_t nx;
  const uint64_t* z_in;
  uint64_t* z_out;
  int64_t nz;
  unsigned long long* zero;
  int64_t nzero;
  Feistel fx, fz;
  int blocks;  // a multiple of kXcds
  int every;   // placement of the spare blocks (see k_count_complete)
  int tail;
};

template <int BS>
__device__ __forceinline__ void next_step_part(const NextStep& nx, int b) {
  constexpr int kU = 8;  // independent gathers in flight per thread
  const int64_t stride = (int64_t)nx.blocks * BS;
  for (int64_t i = (int64_t)b * BS + threadIdx.x; i < nx.nzero; i += stride) nx.zero[i] = 0;
  const int64_t tot = nx.nx + nx.nz;
  for (int64_t p0 = (int64_t)b * BS + threadIdx.x; p0 < tot; p0 += stride * kU) {
    uint64_t v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t p = p0 + u * stride;
      if (p < nx.nx)
        v[u] = nx.x_in[feistel_perm_inv(nx.fx, (uint64_t)p, (uint64_t)nx.nx)];
      else if (p < tot)
        v[u] = nx.z_in[feistel_perm_inv(nx.fz, (uint64_t)(p - nx.nx), (uint64_t)nx.nz)];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t p = p0 + u * stride;
      if (p < nx.nx)
        nx.x_out[p] = v[u];
      else if (p < tot)
        nx.z_out[p - nx.nx] = v[u];
    }
  }
}

}  // namespace tw
