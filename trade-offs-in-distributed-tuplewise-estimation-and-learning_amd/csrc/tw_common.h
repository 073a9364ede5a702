// tw_common.h — shared helpers for libtuplewise.so (gfx950 only).
#pragma once
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

}  // namespace tw
