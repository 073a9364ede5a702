// Microbenchmark (design probe for csrc/count.hip, not product code): can the scalar unit
// carry part of the compare-count accumulation?  Each wave compares its lanes' x-values with
// a wave-uniform z (scalar-loaded, 8 per s_load_dwordx16).  For NS of the R x-values per lane
// the 64 compare bits go to an SGPR pair (v_cmp ... s[a:b]) and are counted by the SCALAR unit
// (s_bcnt1_i32_b64 + s_add_u32, wave-uniform 32-bit accumulator); the other R-NS use the VALU
// carry-add.  Per pair: VALU 2 - f instructions, SALU 2f (f = NS/R).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

template <int R, int NS, int U = 8>
__global__ __launch_bounds__(256) void cnt_mix(const double* __restrict__ x,
                                               const double* __restrict__ z, int nz,
                                               unsigned long long* out) {
  double xv[R];
  unsigned acc[R];
  unsigned sacc[NS > 0 ? NS : 1];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    xv[r] = x[(size_t)blockIdx.x * 256 * R + r * 256 + threadIdx.x];
    acc[r] = 0;
  }
#pragma unroll
  for (int r = 0; r < (NS > 0 ? NS : 1); ++r) sacc[r] = 0;
  const double* zz = z + (size_t)blockIdx.y * nz;
  for (int j0 = 0; j0 < nz; j0 += U) {
    double zv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) zv[u] = zz[j0 + u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < NS)
          sacc[r] += (unsigned)__builtin_popcountll(__ballot(xv[r] > zv[u]));
        else
          acc[r] += (xv[r] > zv[u]);
      }
    }
  }
  unsigned long long s = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r >= NS) s += acc[r];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  unsigned long long ss = 0;
#pragma unroll
  for (int r = 0; r < (NS > 0 ? NS : 1); ++r) ss += (NS > 0 ? sacc[r] : 0u);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s + ss);
}

typedef void (*Kern)(const double*, const double*, int, unsigned long long*);

static void run(const char* name, Kern kern, const double* x, const double* z, int nxb, int nzc,
                int nz, int R, unsigned long long* d_out, unsigned long long expect) {
  dim3 g(nxb, nzc);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out);
  CK(hipDeviceSynchronize());
  CK(hipMemset(d_out, 0, 8));
  const int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h;
  CK(hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost));
  const double pairs = (double)nxb * 256 * R * (double)nz * nzc;
  printf("%-24s %8.3f ms/launch  %.3e pairs/s  frac(3.93e13)=%.3f  %s\n", name, ms / it,
         pairs * it / (ms * 1e-3), pairs * it / (ms * 1e-3) / 3.93e13,
         (expect == 0 || h / it == expect) ? "count ok" : "COUNT MISMATCH");
}

int main() {
  // same pair volume for every R: 2^22 x-values against 8 chunks of 4096 z
  const int nzc = 8, nz = 4096, nx = 1 << 22;
  std::vector<double> hx(nx), hz((size_t)nzc * nz);
  srand(1);
  for (auto& v : hx) v = rand() / (double)RAND_MAX;
  for (auto& v : hz) v = rand() / (double)RAND_MAX;
  double *dx, *dz;
  unsigned long long* d_out;
  CK(hipMalloc(&dx, nx * 8));
  CK(hipMalloc(&dz, hz.size() * 8));
  CK(hipMalloc(&d_out, 8));
  CK(hipMemcpy(dx, hx.data(), nx * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, hz.data(), hz.size() * 8, hipMemcpyHostToDevice));
  // reference count from the pure-VALU variant
  run("valu R2", cnt_mix<2, 0>, dx, dz, nx / 512, nzc, nz, 2, d_out, 0);
  unsigned long long expect;
  CK(hipMemset(d_out, 0, 8));
  hipLaunchKernelGGL((cnt_mix<2, 0>), dim3(nx / 512, nzc), dim3(256), 0, 0, dx, dz, nz, d_out);
  CK(hipMemcpy(&expect, d_out, 8, hipMemcpyDeviceToHost));
  for (int rep = 0; rep < 2; ++rep) {
    run("valu R2", cnt_mix<2, 0>, dx, dz, nx / 512, nzc, nz, 2, d_out, expect);
    run("mix R4 NS2", cnt_mix<4, 2>, dx, dz, nx / 1024, nzc, nz, 4, d_out, expect);
    // the same pairs in blocks of 512 z (8x more, shorter blocks: the bench's shape)
    run("valu R2 nz512", cnt_mix<2, 0>, dx, dz, nx / 512, nzc * 8, nz / 8, 2, d_out, expect);
    run("mix R4 NS2 nz512", cnt_mix<4, 2>, dx, dz, nx / 1024, nzc * 8, nz / 8, 4, d_out, expect);
    run("mix R4 NS2 nz1024", cnt_mix<4, 2>, dx, dz, nx / 1024, nzc * 4, nz / 4, 4, d_out, expect);
    run("mix R2 NS1 nz512", cnt_mix<2, 1, 16>, dx, dz, nx / 512, nzc * 8, nz / 8, 2, d_out, expect);
  }
  return 0;
}
