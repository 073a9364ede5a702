// sortkeys.h — order-preserving u64 keys, the in-LDS bitonic chunk sort and branchless
// binary searches shared by rankcount.hip (sorted counts, rank codes) and complete_grad.hip
// (hinge pair coefficients by threshold search).
#pragma once
#include "tw_common.h"
#include <algorithm>
#include <type_traits>

namespace tw {

constexpr int kSortThreads = 1024;
constexpr int64_t kMaxChunk = 16384;  // 128 KiB of u64 keys in LDS

template <typename T>
__device__ __forceinline__ uint64_t order_key(T v);

template <>
__device__ __forceinline__ uint64_t order_key<double>(double v) {
  if (v != v) return ~0ull;                     // NaN: above everything
  uint64_t b = (uint64_t)__double_as_longlong(v);
  if (b == 0x8000000000000000ull) b = 0;        // -0.0 == +0.0
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <>
__device__ __forceinline__ uint64_t order_key<long long>(long long v) {
  return (uint64_t)v ^ 0x8000000000000000ull;
}

template <typename T>
__device__ __forceinline__ bool is_nan_score(T v) {
  if constexpr (std::is_floating_point<T>::value) return v != v;
  return false;
}

// Register-blocked bitonic sort of one chunk: thread t owns keys [16t, 16t+16).  For every
// merge size k the passes with partner distance j >= 16 run through LDS (one compare-exchange
// per pair), the last four (j = 8, 4, 2, 1) on the thread's own 16 registers.  C >= 1024.
__device__ __forceinline__ void cex(uint64_t& a, uint64_t& b, bool up) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = up ? lo : hi;
  b = up ? hi : lo;
}

// bitonic levels j = E/2..1 of merge size k on v[0..E) = keys[base .. base+E)
template <int E>
__device__ __forceinline__ void reg_levels(uint64_t (&v)[E], int base, int k, int jmax) {
#pragma unroll
  for (int j = E / 2; j > 0; j >>= 1) {
    if (j > jmax) continue;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if ((e & j) == 0) {
        const bool up = ((base + e) & k) == 0;
        cex(v[e], v[e | j], up);
      }
    }
  }
}

// Keys stay in registers for the whole network: thread t owns keys [E t, E t + E) of the
// chunk (C / E threads; E = max(4, C / 1024) so a block always has >= 256 threads and
// chunks >= 4096 get 16 waves to hide shuffle/LDS latency).  Level (k, j) pairs key i with
// key i ^ j:
//   j <  E          same thread          -> compare-exchange in registers
//   E <= j < 64 E   same wave (lane ^ j/E) -> __shfl_xor, no barrier
//   j >= 64 E       other wave           -> exchange through LDS (one barrier pair)
// Direction: ascending iff (i & k) == 0.  C is a power of two >= 4 E (>= 1024 for the
// callers that sort shard chunks; the ranking's sample sort uses C >= 256).
// The network on C keys already in LDS (`keys`), thread t owning [E t, E t + E); the sorted
// keys written to dst.  Every thread of the block (C / E of them) calls it.
template <int kE>
__device__ __forceinline__ void sort_keys_block(uint64_t* keys, int C, uint64_t* __restrict__ dst,
                                                int n_out = -1) {
  const int nthr = blockDim.x;  // == C / kE
  const int tid = threadIdx.x;
  const int base = tid * kE;
  uint64_t v[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) v[e] = keys[base + e];
  for (int k = 2; k <= kE; k <<= 1) reg_levels<kE>(v, base, k, k >> 1);  // runs of E sorted
  for (int k = 2 * kE; k <= C; k <<= 1) {
    const bool up = ((base & k) == 0);  // (i & k) for every e, since k >= 2E > e
    for (int j = k >> 1; j >= kE; j >>= 1) {
      const int m = j / kE;  // partner thread distance
      const bool keep_min = (((tid & m) == 0) == up);
      if (m >= kWave) {  // across waves: through LDS
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kE; ++e) keys[base + e] = v[e];
        __syncthreads();
        const int pb = (tid ^ m) * kE;
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const uint64_t o = keys[pb + e];
          v[e] = keep_min ? (o < v[e] ? o : v[e]) : (o > v[e] ? o : v[e]);
        }
      } else {  // inside the wave: lane shuffles
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const uint64_t o = __shfl_xor(v[e], m, kWave);
          v[e] = keep_min ? (o < v[e] ? o : v[e]) : (o > v[e] ? o : v[e]);
        }
      }
    }
    reg_levels<kE>(v, base, k, kE >> 1);
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kE; ++e) keys[base + e] = v[e];
  __syncthreads();
  const int n = n_out < 0 ? C : n_out;  // the first n sorted keys (pads sort last)
  for (int i = tid; i < n; i += nthr) dst[i] = keys[i];
}

// The same network on kE * 64 keys held by ONE wave (lane l owning [kE l, kE l + kE)): the
// register levels and the in-wave shuffles only, no barrier, so the waves of a block sort
// different key runs at once (the ranking's long sub-buckets).
template <int kE>
__device__ __forceinline__ void wave_sort_keys(uint64_t (&v)[kE], int lane) {
  constexpr int C = kE * kWave;
  const int base = lane * kE;
  for (int k = 2; k <= kE; k <<= 1) reg_levels<kE>(v, base, k, k >> 1);
  for (int k = 2 * kE; k <= C; k <<= 1) {
    const bool up = ((base & k) == 0);
    for (int j = k >> 1; j >= kE; j >>= 1) {
      const int m = j / kE;
      const bool keep_min = (((lane & m) == 0) == up);
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const uint64_t o = __shfl_xor(v[e], m, kWave);
        v[e] = keep_min ? (o < v[e] ? o : v[e]) : (o > v[e] ? o : v[e]);
      }
    }
    reg_levels<kE>(v, base, k, kE >> 1);
  }
}

template <typename T, int kE>
__global__ __launch_bounds__(kSortThreads) void k_sort_chunks(const T* __restrict__ z,
                                                              const int64_t* __restrict__ z_off,
                                                              int chunks, int C,
                                                              uint64_t* __restrict__ sorted,
                                                              int64_t stride = 0) {
  extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
  const int s = blockIdx.x / chunks;
  const int c = blockIdx.x - s * chunks;
  // shard s is z[z_off[s], z_off[s+1]), or z[s*stride, (s+1)*stride) without offsets
  const int64_t zb = z_off ? z_off[s] : (int64_t)s * stride;
  const int64_t ze = z_off ? z_off[s + 1] : zb + stride;
  const int64_t c0 = zb + (int64_t)c * C;
  const int nthr = blockDim.x;  // == C / kE
  const int tid = threadIdx.x;
  for (int i = tid; i < C; i += nthr) {  // coalesced load + key transform
    const int64_t g = c0 + i;
    keys[i] = (g < ze) ? order_key<T>(z[g]) : ~0ull;
  }
  __syncthreads();
  uint64_t* dst = sorted + (int64_t)blockIdx.x * C;
  if (c0 >= ze) {  // block-uniform: an empty chunk stays all-padding
    for (int i = tid; i < C; i += nthr) dst[i] = ~0ull;
    return;
  }
  sort_keys_block<kE>(keys, C, dst);
}

// #{keys < k} in a sorted power-of-two array (branchless).
__device__ __forceinline__ uint32_t lower_bound_lds(const uint64_t* a, int C, uint64_t k) {
  uint32_t i = 0;
  for (int st = C >> 1; st > 0; st >>= 1) i += (a[i + st - 1] < k) ? st : 0;
  return i + (a[i] < k ? 1 : 0);
}
__device__ __forceinline__ uint32_t upper_bound_lds(const uint64_t* a, int C, uint64_t k) {
  uint32_t i = 0;
  for (int st = C >> 1; st > 0; st >>= 1) i += (a[i + st - 1] <= k) ? st : 0;
  return i + (a[i] <= k ? 1 : 0);
}

// Inverse of order_key<double> (NaN/padding key ~0 decodes to a NaN).
__device__ __forceinline__ double key_to_double(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)b);
}

}  // namespace tw
