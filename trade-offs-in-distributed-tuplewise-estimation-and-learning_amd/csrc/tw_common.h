// tw_common.h — shared helpers for libtuplewise.so (gfx950 only).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <cstdio>
#include <cstdarg>
#include "../../include/tuplewise.h"

namespace tw {

// Thread-local error message behind tw_last_error().
void set_error(const char* fmt, ...);

#define TW_ARG_CHECK(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::tw::set_error(__VA_ARGS__);      \
      return TW_ERR_ARG;                 \
    }                                    \
  } while (0)

#define TW_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::tw::set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__,    \
                      __LINE__, #expr);                                                 \
      return TW_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

#define TW_LAUNCH_CHECK() TW_HIP_CHECK(hipGetLastError())

constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Zeroing of device buffers by a kernel rather than hipMemsetAsync: every entry point may be
// captured into a hipGraph, and a captured memset node was seen not to take effect in one
// graph-replay sequence; a kernel node is an ordinary launch.
static __global__ __launch_bounds__(256) void k_zero_fill(unsigned char* __restrict__ p,
                                                          size_t n) {
  const size_t tid = blockIdx.x * (size_t)256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
  if ((((uintptr_t)p | n) & 7) == 0) {
    unsigned long long* q = (unsigned long long*)p;
    for (size_t i = tid; i < n / 8; i += stride) q[i] = 0ull;
  } else {
    for (size_t i = tid; i < n; i += stride) p[i] = 0;
  }
}

// same signature as hipMemsetAsync; value must be 0
static inline hipError_t tw_zero_async(void* p, int value, size_t bytes, hipStream_t st) {
  if (value != 0) return hipErrorInvalidValue;
  if (bytes == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>(1024, (bytes + 256 * 8 * 4 - 1) / (256 * 8 * 4));
  hipLaunchKernelGGL(k_zero_fill, dim3((unsigned)std::max<size_t>(blocks, 1)), dim3(256), 0, st,
                     (unsigned char*)p, bytes);
  return hipGetLastError();
}

// XCD-aware block order.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (blocks b and b+8 share one XCD and its 4 MiB L2; MI355X_MICROARCH.md "Workgroup dispatch").
// xcd_block() maps the hardware block id to a logical id so that each XCD receives one
// CONTIGUOUS range of logical ids: with shard-major logical order an XCD works on whole
// shards, and a shard's scores are fetched into one L2 instead of all eight.  Bijective for
// any grid size; placement affects speed only, never results.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_block(int b, int nblocks) {
  const int q = nblocks / kXcds, r = nblocks - q * kXcds;
  const int x = b % kXcds, i = b / kXcds;
  return x * q + (x < r ? x : r) + i;
}

// Wave-level sum of a 64-bit value (DPP/ds_swizzle lowering of __shfl_xor on gfx950).
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Wave sum of a double in a FIXED butterfly order (deterministic for a given lane layout).
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// One DPP move of a double (both 32-bit halves).  Lanes outside row_mask receive an undefined
// value (no "old" operand to materialise): callers only use lanes the pattern defines.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROW_MASK, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Wave sum of a double through DPP lane moves (no LDS round trip, unlike __shfl_xor's
// ds_bpermute): quad xor 1, quad xor 2, half-row mirror, row mirror, then row_bcast15 /
// row_bcast31 fold the four rows into lane 63 (other lanes end with partial or undefined
// sums), which is broadcast.  Fixed order (deterministic).
__device__ __forceinline__ double wave_sum_dpp_f64(double v) {
  v += dpp_f64<0xB1>(v);        // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);        // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);       // row_half_mirror: sums of 8
  v += dpp_f64<0x140>(v);       // row_mirror: sums of 16
  v += dpp_f64<0x142, 0xA>(v);  // row_bcast15 into rows 1, 3
  v += dpp_f64<0x143, 0xC>(v);  // row_bcast31 into rows 2, 3: lane 63 holds the total
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Pair weights of the gradient sum.  TW_LOSS_HINGE: grad_inc_block's filter 1{S > 0}
// (compute_stats.py:158-161), applied as a branch so unfiltered rows are skipped exactly as
// diff[filt] skips them.  TW_LOSS_LOGISTIC (extension, SURVEY.md §8 row L3 — not in the
// reference): the gradient of softplus(S) = log(1 + e^S), weight sigma(S) = 1 / (1 + e^-S).
template <int LOSS>
__device__ __forceinline__ double pair_weight(double S) {
  if constexpr (LOSS == TW_LOSS_HINGE) return S > 0.0 ? 1.0 : 0.0;
  else return 1.0 / (1.0 + exp(-S));
}
template <int LOSS>
__device__ __forceinline__ double weighted(double wgt, double v) {
  if constexpr (LOSS == TW_LOSS_HINGE) return wgt != 0.0 ? v : -0.0;  // -0.0 leaves sums as is
  else return wgt * v;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based RNG for the device-RNG modes.
struct u32x4 {
  uint32_t a, b, c, d;
};
__device__ __forceinline__ u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) gives both halves
    const uint64_t p0 = (uint64_t)M0 * ctr.a, p1 = (uint64_t)M1 * ctr.c;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    // a ^ b ^ c in ONE gfx950 three-input bitwise op (v_bitop3_b32, truth table 0x96; the
    // compiler emits two v_xor_b32 for the plain expression): 20 instead of 40 xors per block
    ctr = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, ctr.b, k0, 0x96), lo1,
                (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, ctr.d, k1, 0x96), lo0};
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}
__device__ __forceinline__ uint64_t mulhi_u64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// Device-RNG pair draws (tw_count_pairs_rng, include/tuplewise.h): word w of the Philox block
// (q lo, q hi, shard, att), and Lemire's exactly uniform map of a word to [0, n).
__device__ __forceinline__ uint32_t philox_word(uint64_t q, uint32_t sid, uint32_t att, int w,
                                                uint32_t k0, uint32_t k1) {
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), sid, att}, k0, k1);
  return w == 0 ? r.a : w == 1 ? r.b : w == 2 ? r.c : r.d;
}

__device__ __forceinline__ uint32_t lemire_index(uint32_t r, uint32_t n, uint64_t q, uint32_t sid,
                                                 int w, uint32_t k0, uint32_t k1) {
  uint64_t m = (uint64_t)r * n;
  if ((uint32_t)m < n) {  // rare: only then can the draw fall in the biased zone
    const uint32_t t = (0u - n) % n;
    for (uint32_t att = 1; (uint32_t)m < t; ++att)
      m = (uint64_t)philox_word(q, sid, att, w, k0, k1) * n;
  }
  return (uint32_t)(m >> 32);
}

}  // namespace tw
