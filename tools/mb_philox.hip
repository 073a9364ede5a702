// Microbenchmark (issue model of k_count_rng_img): the issue rate of
// v_mad_u64_u32 (the 32x32->64 multiply of every Philox round) against plain VOP2 ops, and the
// throughput of the product's Philox4x32-10 (tw_common.h) alone.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../trade-offs-in-distributed-tuplewise-estimation-and-learning_amd/csrc mb_philox.hip -o mb_philox
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include "tw_common.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// 8 independent chains of one op each per iteration, 32 iterations unrolled by the asm block
#define REP4(s) s s s s
#define MAD8 asm volatile(REP4( \
  "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n" \
  "v_mad_u64_u32 %2, vcc, %8, %9, %2\n v_mad_u64_u32 %3, vcc, %8, %9, %3\n" \
  "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n" \
  "v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7\n") \
  : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) \
  : "v"(b), "v"(c) : "vcc")
#define MULHI8 asm volatile(REP4( \
  "v_mul_hi_u32 %0, %8, %0\n v_mul_hi_u32 %1, %8, %1\n v_mul_hi_u32 %2, %8, %2\n v_mul_hi_u32 %3, %8, %3\n" \
  "v_mul_hi_u32 %4, %8, %4\n v_mul_hi_u32 %5, %8, %5\n v_mul_hi_u32 %6, %8, %6\n v_mul_hi_u32 %7, %8, %7\n") \
  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(b))
#define MULLO8 asm volatile(REP4( \
  "v_mul_lo_u32 %0, %8, %0\n v_mul_lo_u32 %1, %8, %1\n v_mul_lo_u32 %2, %8, %2\n v_mul_lo_u32 %3, %8, %3\n" \
  "v_mul_lo_u32 %4, %8, %4\n v_mul_lo_u32 %5, %8, %5\n v_mul_lo_u32 %6, %8, %6\n v_mul_lo_u32 %7, %8, %7\n") \
  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(b))
#define BITOP8 asm volatile(REP4( \
  "v_bitop3_b32 %0, %8, %0, %9 bitop3:0x96\n v_bitop3_b32 %1, %8, %1, %9 bitop3:0x96\n" \
  "v_bitop3_b32 %2, %8, %2, %9 bitop3:0x96\n v_bitop3_b32 %3, %8, %3, %9 bitop3:0x96\n" \
  "v_bitop3_b32 %4, %8, %4, %9 bitop3:0x96\n v_bitop3_b32 %5, %8, %5, %9 bitop3:0x96\n" \
  "v_bitop3_b32 %6, %8, %6, %9 bitop3:0x96\n v_bitop3_b32 %7, %8, %7, %9 bitop3:0x96\n") \
  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) \
  : "v"(b), "v"(c))
#define XOR8 asm volatile(REP4( \
  "v_xor_b32 %0, %8, %0\n v_xor_b32 %1, %8, %1\n v_xor_b32 %2, %8, %2\n v_xor_b32 %3, %8, %3\n" \
  "v_xor_b32 %4, %8, %4\n v_xor_b32 %5, %8, %5\n v_xor_b32 %6, %8, %6\n v_xor_b32 %7, %8, %7\n") \
  : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]), "+v"(u[7]) : "v"(b))

template <int K>
__global__ __launch_bounds__(256) void probe(int iters, unsigned* out, unsigned seed) {
  uint64_t a[8];
  unsigned u[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7ull + i + seed;
    u[i] = threadIdx.x * 5 + i + seed;
  }
  unsigned b = threadIdx.x ^ seed, c = b * 3;
  for (int i = 0; i < iters; ++i) {
    if constexpr (K == 0) MAD8;
    if constexpr (K == 1) MULHI8;
    if constexpr (K == 2) MULLO8;
    if constexpr (K == 3) XOR8;
    if constexpr (K == 4) { MAD8; XOR8; XOR8; }  // Philox's 1 multiply : 2 xor
    if constexpr (K == 5) BITOP8;
    if constexpr (K == 6) { MAD8; BITOP8; }  // 1 multiply : 1 three-input xor
  }
  unsigned s = 0;
  for (int i = 0; i < 8; ++i) s += (unsigned)a[i] + (unsigned)(a[i] >> 32) + u[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Philox4x32-10 with two-input xors (the round-2 form of tw_common.h), for the A/B
__device__ __forceinline__ tw::u32x4 philox_xor2(tw::u32x4 ctr, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)M0 * ctr.a, p1 = (uint64_t)M1 * ctr.c;
    ctr = tw::u32x4{(uint32_t)(p1 >> 32) ^ ctr.b ^ k0, (uint32_t)p1,
                    (uint32_t)(p0 >> 32) ^ ctr.d ^ k1, (uint32_t)p0};
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// the product's Philox4x32-10 (F = 1) or the two-input-xor form (F = 0) on distinct counters,
// two independent blocks per iteration
template <int F>
__global__ __launch_bounds__(256) void philox_only(int iters, unsigned* out, uint32_t k0,
                                                   uint32_t k1) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const tw::u32x4 c0{t, (uint32_t)i, 7u, 0u}, c1{t, (uint32_t)i, 8u, 0u};
    const tw::u32x4 r0 = F ? tw::philox4x32_10(c0, k0, k1) : philox_xor2(c0, k0, k1);
    const tw::u32x4 r1 = F ? tw::philox4x32_10(c1, k0, k1) : philox_xor2(c1, k0, k1);
    acc += r0.a ^ r0.b ^ r0.c ^ r0.d ^ r1.a ^ r1.b ^ r1.c ^ r1.d;
  }
  out[t] = acc;
}

int main() {
  const char* names[] = {"v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_xor_b32",
                         "mad_u64 + 2 xor", "v_bitop3_b32", "mad_u64 + bitop3"};
  void (*ks[])(int, unsigned*, unsigned) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>,
                                            probe<5>, probe<6>};
  const int ops_per_iter[] = {32, 32, 32, 32, 96, 32, 64};
  const int blocks = 256 * 8, iters = 2048;
  unsigned* out;
  CK(hipMalloc(&out, blocks * 256 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int k = 0; k < 7; ++k) {
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1u);
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1u);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double wave_ops = (double)blocks * 4 * iters * ops_per_iter[k];
    printf("%-18s %8.3f ms  %.3f wave-instr/cycle/CU @2.4GHz\n", names[k], best,
           wave_ops / (best * 1e-3) / 256 / 2.4e9);
  }
  const int piters = 512;
  void (*pk[])(int, unsigned*, uint32_t, uint32_t) = {philox_only<0>, philox_only<1>};
  const char* pn[] = {"philox 2-input xor", "philox bitop3"};
  for (int f = 0; f < 2; ++f) {
    hipLaunchKernelGGL(pk[f], dim3(blocks), dim3(256), 0, 0, piters, out, 11u, 13u);
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(pk[f], dim3(blocks), dim3(256), 0, 0, piters, out, 11u, 13u);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double pblocks = (double)blocks * 256 * piters * 2;
    printf("%-18s %8.3f ms  %.3e blocks/s = %.3e pairs/s (2 pairs per block)\n", pn[f], best,
           pblocks / (best * 1e-3), 2 * pblocks / (best * 1e-3));
  }
  return 0;
}
