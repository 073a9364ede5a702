// feistel.h — the keyed bijection of [0, n) behind every device repartition
// (csrc/permute.hip; restated in oracle/oracle.py feistel_perm / feistel_perm_inv): a 6-round
// balanced Feistel network on the smallest even-bit power-of-two domain >= n, cycle-walked
// into [0, n).
#pragma once
#include "tw_common.h"

namespace tw {

// v / d for the exchange's rank arithmetic (v < G*n_loc < 2^53, d = n_loc >= 1): one f64
// multiply by the reciprocal and an exact integer correction, instead of the ~50-instruction
// 64-bit division sequence — the exchange kernels run beside the VALU-bound count kernel and
// every instruction they issue is taken from it.
struct FastDiv {
  uint64_t d;
  double inv;
};

__host__ __device__ inline FastDiv make_fastdiv(uint64_t d) { return FastDiv{d, 1.0 / (double)d}; }

__host__ __device__ inline uint64_t fast_div(uint64_t v, const FastDiv& f) {
  uint64_t q = (uint64_t)((double)v * f.inv);
  while (q * f.d > v) --q;            // the product is within one of v / d for v < 2^53
  while ((q + 1) * f.d <= v) ++q;
  return q;
}

struct Feistel {
  uint32_t half_bits;
  uint32_t mask;
  uint32_t k[6];
};

__host__ __device__ inline uint32_t mix32(uint32_t v) {  // murmur3 finaliser
  v ^= v >> 16;
  v *= 0x85EBCA6Bu;
  v ^= v >> 13;
  v *= 0xC2B2AE35u;
  v ^= v >> 16;
  return v;
}

__host__ __device__ inline Feistel make_feistel(int64_t n, uint64_t key) {
  Feistel f;
  int bits = 2;
  while (bits < 62 && (1ll << bits) < n) ++bits;
  if (bits & 1) ++bits;
  f.half_bits = bits / 2;
  f.mask = (uint32_t)((1ull << f.half_bits) - 1);
  uint64_t st = key ^ 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 6; ++i) {  // splitmix64 key schedule
    st += 0x9E3779B97F4A7C15ull;
    uint64_t zz = st;
    zz = (zz ^ (zz >> 30)) * 0xBF58476D1CE4E5B9ull;
    zz = (zz ^ (zz >> 27)) * 0x94D049BB133111EBull;
    zz ^= zz >> 31;
    f.k[i] = (uint32_t)zz;
  }
  return f;
}

__host__ __device__ inline uint64_t feistel_once(const Feistel& f, uint64_t v) {
  uint32_t L = (uint32_t)(v >> f.half_bits) & f.mask;
  uint32_t R = (uint32_t)v & f.mask;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint32_t nL = R;
    R = (L ^ mix32(R * 0x9E3779B1u + f.k[i])) & f.mask;
    L = nL;
  }
  return ((uint64_t)L << f.half_bits) | R;
}

__host__ __device__ inline uint64_t feistel_perm(const Feistel& f, uint64_t i, uint64_t n) {
  uint64_t v = feistel_once(f, i);
  while (v >= n) v = feistel_once(f, v);  // cycle walking: terminates (bijection on domain)
  return v;
}

// Inverse network: rounds in reverse order.  Round i maps (L, R) -> (R, L ^ F_i(R)), so its
// inverse maps (L', R') -> (R' ^ F_i(L'), L').  Cycle walking backwards from a position in
// [0, n) retraces the forward walk, so feistel_perm_inv(feistel_perm(i)) == i.
__host__ __device__ inline uint64_t feistel_once_inv(const Feistel& f, uint64_t v) {
  uint32_t L = (uint32_t)(v >> f.half_bits) & f.mask;
  uint32_t R = (uint32_t)v & f.mask;
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    const uint32_t pR = L;
    L = (R ^ mix32(pR * 0x9E3779B1u + f.k[i])) & f.mask;
    R = pR;
  }
  return ((uint64_t)L << f.half_bits) | R;
}

__host__ __device__ inline uint64_t feistel_perm_inv(const Feistel& f, uint64_t p, uint64_t n) {
  uint64_t v = feistel_once_inv(f, p);
  while (v >= n) v = feistel_once_inv(f, v);
  return v;
}

// The same rounds on 32-bit words, for domains of at most 2^32 (half_bits <= 16): the step
// chains (csrc/chain.hip) keep positions in u32 and evaluate these per element and step.
__device__ __forceinline__ uint32_t feistel_once32(const Feistel& f, uint32_t v) {
  uint32_t L = (v >> f.half_bits) & f.mask;
  uint32_t R = v & f.mask;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint32_t nL = R;
    R = (L ^ mix32(R * 0x9E3779B1u + f.k[i])) & f.mask;
    L = nL;
  }
  return (L << f.half_bits) | R;
}
__device__ __forceinline__ uint32_t feistel_once_inv32(const Feistel& f, uint32_t v) {
  uint32_t L = (v >> f.half_bits) & f.mask;
  uint32_t R = v & f.mask;
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    const uint32_t pR = L;
    L = (R ^ mix32(pR * 0x9E3779B1u + f.k[i])) & f.mask;
    R = pR;
  }
  return (L << f.half_bits) | R;
}

// v / d for v < 2^32, d < 2^32: one f64 multiply by the reciprocal (within one of the quotient)
// and one exact correction each way
__device__ __forceinline__ uint32_t fast_div32(uint32_t v, const FastDiv& f) {
  uint32_t q = (uint32_t)((double)v * f.inv);
  if ((uint64_t)q * f.d > v) --q;
  else if ((uint64_t)(q + 1) * f.d <= v) ++q;
  return q;
}

}  // namespace tw
