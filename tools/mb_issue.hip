// Microbenchmark: raw VALU issue rates on gfx950 (design probe, not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
#define REP8(s) s s s s s s s s
// each kernel: ITER iterations x 32 instructions of one kind
template <int KIND>
__global__ __launch_bounds__(256) void probe(int iters, unsigned* out, double seed) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  double d0 = seed + threadIdx.x, d1 = d0 * 2, d2 = d0 * 3, d3 = d0 * 5;
  float f0 = d0, f1 = d1, f2 = d2, f3 = d3;
  for (int i = 0; i < iters; ++i) {
    if (KIND == 0) {  // v_add_u32 x32
      asm volatile(REP8("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a0));
    } else if (KIND == 1) {  // v_fma_f32 x32
      asm volatile(REP8("v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4\n")
                   : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(f0));
    } else if (KIND == 2) {  // v_cmp_lt_f64 -> vcc x32
      asm volatile(REP8("v_cmp_lt_f64 vcc, %0, %1\n v_cmp_lt_f64 vcc, %1, %2\n v_cmp_lt_f64 vcc, %2, %3\n v_cmp_lt_f64 vcc, %3, %0\n")
                   :: "v"(d0), "v"(d1), "v"(d2), "v"(d3) : "vcc");
    } else if (KIND == 3) {  // v_cmp_lt_f64 -> sgpr pair x32 (VOP3)
      asm volatile(REP8("v_cmp_lt_f64_e64 s[40:41], %0, %1\n v_cmp_lt_f64_e64 s[42:43], %1, %2\n v_cmp_lt_f64_e64 s[44:45], %2, %3\n v_cmp_lt_f64_e64 s[46:47], %3, %0\n")
                   :: "v"(d0), "v"(d1), "v"(d2), "v"(d3) : "s40","s41","s42","s43","s44","s45","s46","s47");
    } else if (KIND == 4) {  // v_addc with vcc carry x32
      asm volatile(REP8("v_addc_co_u32 %0, vcc, 0, %0, vcc\n v_addc_co_u32 %1, vcc, 0, %1, vcc\n v_addc_co_u32 %2, vcc, 0, %2, vcc\n v_addc_co_u32 %3, vcc, 0, %3, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) :: "vcc");
    } else if (KIND == 5) {  // v_cmp_lt_f32 -> vcc x32
      asm volatile(REP8("v_cmp_lt_f32 vcc, %0, %1\n v_cmp_lt_f32 vcc, %1, %2\n v_cmp_lt_f32 vcc, %2, %3\n v_cmp_lt_f32 vcc, %3, %0\n")
                   :: "v"(f0), "v"(f1), "v"(f2), "v"(f3) : "vcc");
    } else if (KIND == 6) {  // v_pk_add_u16 x32
      asm volatile(REP8("v_pk_add_u16 %0, %0, %4\n v_pk_add_u16 %1, %1, %4\n v_pk_add_u16 %2, %2, %4\n v_pk_add_u16 %3, %3, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a0));
    } else if (KIND == 7) {  // v_cmp_lt_u32 -> vcc x32
      asm volatile(REP8("v_cmp_lt_u32 vcc, %0, %1\n v_cmp_lt_u32 vcc, %1, %2\n v_cmp_lt_u32 vcc, %2, %3\n v_cmp_lt_u32 vcc, %3, %0\n")
                   :: "v"(a0), "v"(a1), "v"(a2), "v"(a3) : "vcc");
    } else if (KIND == 8) {  // v_sub_co_u32 (carry out to vcc) x32
      asm volatile(REP8("v_sub_co_u32 %0, vcc, %0, %4\n v_sub_co_u32 %1, vcc, %1, %4\n v_sub_co_u32 %2, vcc, %2, %4\n v_sub_co_u32 %3, vcc, %3, %4\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a0) : "vcc");
    } else if (KIND == 9) {  // v_pk_fma_f32 x32
      asm volatile(REP8("v_pk_fma_f32 %0, %0, %2, %2\n v_pk_fma_f32 %1, %1, %2, %2\n v_pk_fma_f32 %0, %0, %2, %2\n v_pk_fma_f32 %1, %1, %2, %2\n")
                   : "+v"(d0), "+v"(d1) : "v"(d2));
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + (unsigned)(f0 + f1 + f2 + f3) + (unsigned)(d0 + d1);
}
int main() {
  const char* names[] = {"v_add_u32", "v_fma_f32", "v_cmp_lt_f64 vcc", "v_cmp_lt_f64 sgpr", "v_addc vcc",
                         "v_cmp_lt_f32 vcc", "v_pk_add_u16", "v_cmp_lt_u32 vcc", "v_sub_co_u32", "v_pk_fma_f32"};
  void (*ks[])(int, unsigned*, double) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>, probe<8>, probe<9>};
  int blocks = 256 * 8, iters = 4096;
  unsigned* out; CK(hipMalloc(&out, blocks * 256 * 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep)
  for (int k = 0; k < 10; ++k) {
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1.0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1.0);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    double wave_ops = (double)blocks * 4 * iters * 32;
    double per_cu_cycle = wave_ops / (ms * 1e-3) / 256 / 2.4e9;
    printf("%-20s %7.3f ms  %.3e wave-ops/s  %.3f wave-ops/cycle/CU @2.4GHz  lane-ops/s %.3e\n", names[k], ms,
           wave_ops / (ms * 1e-3), per_cu_cycle, wave_ops * 64 / (ms * 1e-3));
  }
  return 0;
}
