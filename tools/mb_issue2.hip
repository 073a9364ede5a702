// Microbenchmark: which gfx950 VALU ops issue faster than 1 per 4 cycles per SIMD (design probe).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
#define REP4(s) s s s s
#define BODY(OP) asm volatile(REP4(OP " %0, %8, %0\n " OP " %1, %8, %1\n " OP " %2, %8, %2\n " OP " %3, %8, %3\n " OP " %4, %8, %4\n " OP " %5, %8, %5\n " OP " %6, %8, %6\n " OP " %7, %8, %7\n") \
   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b) : "vcc")
#define BODY3(OP) asm volatile(REP4(OP " %0, %8, %0, %9\n " OP " %1, %8, %1, %9\n " OP " %2, %8, %2, %9\n " OP " %3, %8, %3, %9\n " OP " %4, %8, %4, %9\n " OP " %5, %8, %5, %9\n " OP " %6, %8, %6, %9\n " OP " %7, %8, %7, %9\n") \
   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c) : "vcc")
#define BODYCMP(OP) asm volatile(REP4(OP " vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n" OP " vcc, %2, %8\n v_cndmask_b32 %3, %3, %8, vcc\n" OP " vcc, %4, %8\n v_cndmask_b32 %5, %5, %8, vcc\n" OP " vcc, %6, %8\n v_cndmask_b32 %7, %7, %8, vcc\n") \
   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b) : "vcc")
template <int K>
__global__ __launch_bounds__(256) void probe(int iters, unsigned* out, unsigned seed) {
  unsigned a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + seed;
  unsigned b = threadIdx.x ^ seed, c = b * 3;
  for (int i = 0; i < iters; ++i) {
    switch (K) {
      case 0: BODY("v_add_u32"); break;
      case 1: BODY("v_sub_u32"); break;
      case 2: BODY("v_xor_b32"); break;
      case 3: BODY("v_and_b32"); break;
      case 4: BODY("v_lshrrev_b32"); break;
      case 5: BODY("v_max_u32"); break;
      case 6: BODY("v_add_f32"); break;
      case 7: BODY("v_mul_f32"); break;
      case 8: BODY3("v_add3_u32"); break;
      case 9: BODY3("v_sad_u32"); break;
      case 10: BODY3("v_sad_u16"); break;
      case 11: BODY3("v_sad_u8"); break;
      case 12: BODY("v_add_co_u32"); break;
      case 13: BODY("v_pk_add_u16"); break;
      case 14: BODY3("v_lshl_add_u32"); break;
      case 15: BODYCMP("v_cmp_lt_u32"); break;
      case 16: BODY3("v_bfe_u32"); break;
      case 17: BODY3("v_med3_u32"); break;
      case 18: BODY("v_cvt_f32_u32" " %0, %8 ; "); break;
    }
  }
  unsigned s = 0; for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  const char* names[] = {"v_add_u32", "v_sub_u32", "v_xor_b32", "v_and_b32", "v_lshrrev_b32", "v_max_u32", "v_add_f32",
                         "v_mul_f32", "v_add3_u32", "v_sad_u32", "v_sad_u16", "v_sad_u8", "v_add_co_u32", "v_pk_add_u16",
                         "v_lshl_add_u32", "cmp_u32+cndmask", "v_bfe_u32", "v_med3_u32", "(skip)"};
  void (*ks[])(int, unsigned*, unsigned) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>, probe<8>, probe<9>,
                                            probe<10>, probe<11>, probe<12>, probe<13>, probe<14>, probe<15>, probe<16>, probe<17>};
  int blocks = 256 * 8, iters = 4096;
  unsigned* out; CK(hipMalloc(&out, blocks * 256 * 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int k = 0; k < 18; ++k) {
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1u);
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(256), 0, 0, iters, out, 1u);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
    }
    double wave_ops = (double)blocks * 4 * iters * 32;
    printf("%-18s %7.3f ms  %.3f wave-ops/cycle/CU @2.4GHz  lane-ops/s %.3e\n", names[k], best,
           wave_ops / (best * 1e-3) / 256 / 2.4e9, wave_ops * 64 / (best * 1e-3));
  }
  return 0;
}
