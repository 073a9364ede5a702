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

// The next repartition carried by the COUNT threads of a launch whose blocks leave no room for
// spare blocks (LDS-resident shards): thread t of block b owns elements e = b*BS + t + k*stride
// (stride = grid threads), k < kmax, of the next permutation (next_step_part's gather).
// NextSlice keeps ONE gather in flight — issue() stores the previous value and issues the next
// — for kernels with a long loop to spread them over; NextBatch issues up to KB at once and
// stores them at commit(), for kernels whose middle phases are LDS-bound.
template <int BS>
struct NextSlice {
  const NextStep& nx;
  int64_t e0, stride, tot;
  int k = 0, kmax;
  uint64_t v = 0;
  int64_t p = -1;
  __device__ NextSlice(const NextStep& n) : nx(n) {
    e0 = (int64_t)blockIdx.x * BS + threadIdx.x;
    stride = (int64_t)gridDim.x * BS;
    tot = n.nx + n.nz;
    kmax = n.blocks ? (int)((tot + stride - 1) / stride) : 0;
  }
  __device__ __forceinline__ uint64_t gather(int64_t q) const {
    if (q < nx.nx) return nx.x_in[feistel_perm_inv(nx.fx, (uint64_t)q, (uint64_t)nx.nx)];
    if (q < tot) return nx.z_in[feistel_perm_inv(nx.fz, (uint64_t)(q - nx.nx), (uint64_t)nx.nz)];
    return 0;
  }
  __device__ __forceinline__ void store(int64_t q, uint64_t val) const {
    if (q >= 0 && q < nx.nx)
      nx.x_out[q] = val;
    else if (q >= nx.nx && q < tot)
      nx.z_out[q - nx.nx] = val;
  }
  __device__ __forceinline__ void issue() {  // stores the previous gather, issues the next
    store(p, v);
    p = e0 + (int64_t)k * stride;
    ++k;
    v = gather(p);
  }
  __device__ __forceinline__ void finish() {
    while (k < kmax) issue();
    store(p, v);
    p = -1;
  }
};

template <int BS, int KB>
struct NextBatch {
  NextSlice<BS> sl;
  uint64_t v[KB];
  __device__ NextBatch(const NextStep& n) : sl(n) {}
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (k < sl.kmax) v[k] = sl.gather(sl.e0 + (int64_t)k * sl.stride);
  }
  __device__ __forceinline__ void commit() {
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (k < sl.kmax) sl.store(sl.e0 + (int64_t)k * sl.stride, v[k]);
    for (int k = KB; k < sl.kmax; ++k) {  // beyond the batch: one at a time
      const int64_t q = sl.e0 + (int64_t)k * sl.stride;
      sl.store(q, sl.gather(q));
    }
  }
};

// zero the next step's counters (grid-stride over the launch)
template <int BS>
__device__ __forceinline__ void next_step_zero(const NextStep& nx) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nx.nzero;
       i += (int64_t)gridDim.x * BS)
    nx.zero[i] = 0;
}

}  // namespace tw
