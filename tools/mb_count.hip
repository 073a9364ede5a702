// Microbenchmark: accumulation variants for the all-pairs compare kernel
// (design probe for csrc/count.hip; not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

// V: 0 = VALU accumulate, 1 = SALU ballot+popcount, 2 = mixed (NS of R via SALU), 3 = f32 cmp probe
template <int R, int V, int NS>
__global__ __launch_bounds__(256) void cnt(const double* __restrict__ x, const double* __restrict__ z,
                                           int nz, unsigned long long* out) {
  double xv[R]; unsigned acc[R]; unsigned long long sacc = 0;
  for (int r = 0; r < R; ++r) { xv[r] = x[blockIdx.x * 256 * R + r * 256 + threadIdx.x]; acc[r] = 0; }
  const double* zz = z + (blockIdx.y * (size_t)nz);
#pragma unroll 8
  for (int j = 0; j < nz; ++j) {
    double zv = zz[j];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (V == 0 || (V == 2 && r >= NS)) acc[r] += (xv[r] > zv);
      else sacc += __popcll(__ballot(xv[r] > zv));
    }
  }
  unsigned long long s = 0;
  for (int r = 0; r < R; ++r) s += acc[r];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s + sacc);
}
template <int R>
__global__ __launch_bounds__(256) void cnt32(const float* __restrict__ x, const float* __restrict__ z,
                                             int nz, unsigned long long* out) {
  float xv[R]; unsigned acc[R];
  for (int r = 0; r < R; ++r) { xv[r] = x[blockIdx.x * 256 * R + r * 256 + threadIdx.x]; acc[r] = 0; }
  const float* zz = z + (blockIdx.y * (size_t)nz);
#pragma unroll 8
  for (int j = 0; j < nz; ++j) {
    float zv = zz[j];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += (xv[r] > zv);
  }
  unsigned long long s = 0;
  for (int r = 0; r < R; ++r) s += acc[r];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

template <typename T>
void run(const char* name, void (*kern)(const T*, const T*, int, unsigned long long*), const T* x, const T* z, int nxb, int nzc, int nz, int R,
         unsigned long long* d_out) {
  dim3 g(nxb, nzc);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out);
  CK(hipDeviceSynchronize());
  CK(hipMemset(d_out, 0, 8));
  int it = 10;
  CK(hipEventRecord(a));
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, x, z, nz, d_out);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h; CK(hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost));
  double pairs = (double)nxb * 256 * R * (double)nz * nzc;
  printf("%-28s %8.3f ms/launch  %.3e pairs/s  frac(3.93e13)=%.3f  count/it=%llu\n", name, ms / it,
         pairs * it / (ms * 1e-3), pairs * it / (ms * 1e-3) / 3.93e13, h / it);
}

int main() {
  const int R = 8, nxb = 512, nzc = 8, nz = 4096;
  size_t nx = (size_t)nxb * 256 * R, nzt = (size_t)nzc * nz;
  std::vector<double> hx(nx), hz(nzt);
  std::vector<float> fx(nx), fz(nzt);
  srand(1);
  for (auto& v : hx) v = rand() / (double)RAND_MAX;
  for (auto& v : hz) v = rand() / (double)RAND_MAX;
  for (size_t i = 0; i < nx; ++i) fx[i] = hx[i];
  for (size_t i = 0; i < nzt; ++i) fz[i] = hz[i];
  double *dx, *dz; float *fdx, *fdz; unsigned long long* d_out;
  CK(hipMalloc(&dx, nx * 8)); CK(hipMalloc(&dz, nzt * 8)); CK(hipMalloc(&fdx, nx * 4)); CK(hipMalloc(&fdz, nzt * 4));
  CK(hipMalloc(&d_out, 8));
  CK(hipMemcpy(dx, hx.data(), nx * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, hz.data(), nzt * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(fdx, fx.data(), nx * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(fdz, fz.data(), nzt * 4, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    run("valu R8", cnt<8, 0, 0>, dx, dz, nxb, nzc, nz, 8, d_out);
    run("salu R8", cnt<8, 1, 0>, dx, dz, nxb, nzc, nz, 8, d_out);
    run("mix R8 NS2", cnt<8, 2, 2>, dx, dz, nxb, nzc, nz, 8, d_out);
    run("mix R8 NS3", cnt<8, 2, 3>, dx, dz, nxb, nzc, nz, 8, d_out);
    run("mix R8 NS4", cnt<8, 2, 4>, dx, dz, nxb, nzc, nz, 8, d_out);
    run("valu R4 (2x blocks)", cnt<4, 0, 0>, dx, dz, nxb * 2, nzc, nz, 4, d_out);
    run("valu R16 (0.5x blocks)", cnt<16, 0, 0>, dx, dz, nxb / 2, nzc, nz, 16, d_out);
    run("f32 valu R8 (probe)", cnt32<8>, fdx, fdz, nxb, nzc, nz, 8, d_out);
  }
  return 0;
}
