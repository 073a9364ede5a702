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
#include <cmath>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

template <int R, int NS, int U = 8, bool ZF = false, bool XCD = false>
__global__ __launch_bounds__(256) void cnt_mix(const double* __restrict__ x,
                                               const double* __restrict__ z, int nz,
                                               unsigned long long* out, int nxb) {
  // ZF: z-chunk index fastest, so co-resident blocks of a CU stream DIFFERENT z chunks
  // (the production kernel's pattern) instead of all sharing one (scalar-cache friendly).
  // XCD: 1-D grid, block id remapped so each XCD gets a contiguous range (as production).
  int bx = blockIdx.x, by = blockIdx.y;
  if (XCD) {
    const int nb = gridDim.x, q = nb / 8, rr = nb % 8, xx = blockIdx.x % 8, ii = blockIdx.x / 8;
    const int lb = xx * q + (xx < rr ? xx : rr) + ii;
    bx = lb % nxb;
    by = lb / nxb;
  }
  double xv[R];
  unsigned acc[R];
  unsigned sacc[NS > 0 ? NS : 1];
  const size_t xt = ZF ? by : bx;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    xv[r] = x[xt * 256 * R + r * 256 + threadIdx.x];
    acc[r] = 0;
  }
#pragma unroll
  for (int r = 0; r < (NS > 0 ? NS : 1); ++r) sacc[r] = 0;
  const double* zz = z + (size_t)(ZF ? bx : by) * nz;
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
  // spread over 1024 counters: one address for every wave serialises the atomics and made
  // short-block shapes look 2-4x slower than they are (mb_mix3.log's nz512 rows)
  if ((threadIdx.x & 63) == 0) atomicAdd(out + ((blockIdx.y * gridDim.x + blockIdx.x) & 1023), s + ss);
}

typedef void (*Kern)(const double*, const double*, int, unsigned long long*, int);

static void run(const char* name, Kern kern, const double* x, const double* z, int nxb, int nzc,
                int nz, int R, unsigned long long* d_out, unsigned long long expect,
                bool zf = false, bool xcd = false) {
  dim3 g = xcd ? dim3(nzc * nxb) : zf ? dim3(nzc, nxb) : dim3(nxb, nzc);
  const int nxa = zf ? nzc : nxb;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out, nxa);
  CK(hipDeviceSynchronize());
  CK(hipMemset(d_out, 0, 8 * 1024));
  const int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out, nxa);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h = 0, hv[1024];
  CK(hipMemcpy(hv, d_out, 8 * 1024, hipMemcpyDeviceToHost));
  for (int i = 0; i < 1024; ++i) h += hv[i];
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
  CK(hipMalloc(&d_out, 8 * 1024));
  CK(hipMemcpy(dx, hx.data(), nx * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, hz.data(), hz.size() * 8, hipMemcpyHostToDevice));
  // reference count from the pure-VALU variant
  run("valu R2", cnt_mix<2, 0>, dx, dz, nx / 512, nzc, nz, 2, d_out, 0);
  unsigned long long expect = 0, hv[1024];
  CK(hipMemset(d_out, 0, 8 * 1024));
  hipLaunchKernelGGL((cnt_mix<2, 0>), dim3(nx / 512, nzc), dim3(256), 0, 0, dx, dz, nz, d_out, nx / 512);
  CK(hipMemcpy(hv, d_out, 8 * 1024, hipMemcpyDeviceToHost));
  for (int i = 0; i < 1024; ++i) expect += hv[i];
  // x-values per lane R, NS of them counted on the scalar unit: per pair VALU 2 - NS/R,
  // SALU 2 NS/R; balanced at NS/R = 2/3 (1.33 issue slots each, bound 0.75 of the lane-op peak)
  for (int rep = 0; rep < 2; ++rep) {
    run("valu R2", cnt_mix<2, 0>, dx, dz, nx / 512, nzc, nz, 2, d_out, expect);
    run("mix R4 NS2", cnt_mix<4, 2>, dx, dz, nx / 1024, nzc, nz, 4, d_out, expect);
    run("mix R8 NS4", cnt_mix<8, 4>, dx, dz, nx / 2048, nzc, nz, 8, d_out, expect);
    run("mix R3 NS2", cnt_mix<3, 2>, dx, dz, nx / 768, nzc, nz, 3, d_out, 0);  // count unchecked
    run("mix R6 NS4", cnt_mix<6, 4>, dx, dz, nx / 1536, nzc, nz, 6, d_out, 0);
    run("mix R8 NS5", cnt_mix<8, 5>, dx, dz, nx / 2048, nzc, nz, 8, d_out, expect);
    run("mix R8 NS6", cnt_mix<8, 6>, dx, dz, nx / 2048, nzc, nz, 8, d_out, expect);
    run("mix R4 NS3", cnt_mix<4, 3>, dx, dz, nx / 1024, nzc, nz, 4, d_out, expect);
    run("valu R2 nz512", cnt_mix<2, 0>, dx, dz, nx / 512, nzc * 8, nz / 8, 2, d_out, expect);
    run("mix R4 NS2 nz512", cnt_mix<4, 2>, dx, dz, nx / 1024, nzc * 8, nz / 8, 4, d_out, expect);
    run("mix R8 NS4 nz512", cnt_mix<8, 4>, dx, dz, nx / 2048, nzc * 8, nz / 8, 8, d_out, expect);
    // z-chunk-fastest block order
    run("zf valu R2 nz512", cnt_mix<2, 0, 8, true>, dx, dz, nx / 512, nzc * 8, nz / 8, 2, d_out, expect, true);
    run("zf mix R4 NS2 nz512", cnt_mix<4, 2, 8, true>, dx, dz, nx / 1024, nzc * 8, nz / 8, 4, d_out, expect, true);
    run("zf mix R8 NS4 nz512", cnt_mix<8, 4, 8, true>, dx, dz, nx / 2048, nzc * 8, nz / 8, 8, d_out, expect, true);
    run("zf mix R8 NS4", cnt_mix<8, 4, 8, true>, dx, dz, nx / 2048, nzc, nz, 8, d_out, expect, true);
    // the production launch's size: 2^21 x-values against 15 chunks of 512 z = 1.6e10 pairs,
    // 15360 blocks (~0.75 ms): start-up and tail are no longer amortised
    run("short R8 NS4", cnt_mix<8, 4>, dx, dz, 1024, 15, 512, 8, d_out, 0);
    run("short R4 NS2", cnt_mix<4, 2>, dx, dz, 2048, 15, 512, 4, d_out, 0);
    run("short R4 NS2 z1024", cnt_mix<4, 2>, dx, dz, 2048, 8, 1024, 4, d_out, 0);
    run("short R8 NS4 z1024", cnt_mix<8, 4>, dx, dz, 1024, 8, 1024, 8, d_out, 0);
    run("short x2 R4 NS2", cnt_mix<4, 2>, dx, dz, 4096, 15, 512, 4, d_out, 0);
    run("short R4 NS2 xcd", cnt_mix<4, 2, 8, false, true>, dx, dz, 2048, 15, 512, 4, d_out, 0, false, true);
    run("short R4 NS2 zf xcd", cnt_mix<4, 2, 8, true, true>, dx, dz, 2048, 15, 512, 4, d_out, 0, true, true);
    run("short R8 NS4 zf xcd", cnt_mix<8, 4, 8, true, true>, dx, dz, 1024, 15, 512, 8, d_out, 0, true, true);
  }
  // production-like data: X ~ N(0.5, 1), Z ~ N(0, 1) (Box-Muller)
  auto normal = [] {
    const double u1 = (rand() + 1.0) / ((double)RAND_MAX + 2.0), u2 = rand() / (double)RAND_MAX;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  };
  for (auto& v : hx) v = normal() + 0.5;
  for (auto& v : hz) v = normal();
  CK(hipMemcpy(dx, hx.data(), nx * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, hz.data(), hz.size() * 8, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    run("normal short R4 NS2", cnt_mix<4, 2>, dx, dz, 2048, 15, 512, 4, d_out, 0);
    run("normal short R8 NS4", cnt_mix<8, 4>, dx, dz, 1024, 15, 512, 8, d_out, 0);
    run("normal short valu R2", cnt_mix<2, 0>, dx, dz, 4096, 15, 512, 2, d_out, 0);
  }
  return 0;
}
