// Microbenchmark (design probe, not product code): does the physical layout of the C5 row
// table change the cost of the gradient kernel's random row gathers?  256 blocks x 16 waves,
// each block gathers 2 x 100 random 4 KiB rows (the C5 B = 100 step: 25600 pairs, 210 MB)
// from a table of `rows` rows, allocated with hipMalloc, or with hipExtMallocWithFlags(
// hipDeviceMallocContiguous) (physically contiguous: the driver can map it with large
// fragments, fewer TLB misses).  Prints us per launch (HIP events over 200 launches, fresh
// random rows each launch).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

// rows of 512 doubles = 256 d2; a wave reads a row as 4 x 16 B per lane
// TPB threads per block, P pairs in flight per wave; a launch covers 25600 pairs whatever the
// grid (blocks = 25600 / pairs per block)
template <int TPB, int P>
__global__ __launch_bounds__(TPB) void k_gather(const d2* __restrict__ X, const d2* __restrict__ Z,
                                                const int* __restrict__ ix,
                                                const int* __restrict__ iz, int B,
                                                double* __restrict__ out) {
  constexpr int W = TPB / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int* bx = ix + blockIdx.x * B;
  const int* bz = iz + blockIdx.x * B;
  d2 acc = {0.0, 0.0};
  for (int p0 = wave; p0 < B; p0 += W * P) {
    d2 v[8 * P];
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int p = p0 + q * W < B ? p0 + q * W : p0;
      const d2* rx = X + (size_t)bx[p] * 256;
      const d2* rz = Z + (size_t)bz[p] * 256;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[8 * q + k] = rx[lane + 64 * k];
        v[8 * q + 4 + k] = rz[lane + 64 * k];
      }
    }
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc += (p0 + q * W < B) ? v[8 * q + 4 + k] - v[8 * q + k] : d2{0, 0};
  }
  if (acc.x + acc.y == 12345.678) out[blockIdx.x] = acc.x;  // keeps the loads live
}

template <int TPB, int P>
static void launch(int blocks, const d2* X, const d2* Z, const int* ix, const int* iz, int B,
                   double* out) {
  k_gather<TPB, P><<<blocks, TPB>>>(X, Z, ix, iz, B, out);
}
typedef void (*LaunchFn)(int, const d2*, const d2*, const int*, const int*, int, double*);
static LaunchFn g_fn = launch<1024, 2>;
static int g_blocks = 256;

__global__ void k_fill(d2* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = d2{(double)(i & 1023), 1.0};
}

static double run(const char* label, size_t rows, bool contiguous) {
  const size_t bytes = rows * 4096;
  d2 *X = nullptr, *Z = nullptr;
  if (contiguous) {
    if (hipExtMallocWithFlags((void**)&X, bytes, hipDeviceMallocContiguous) != hipSuccess ||
        hipExtMallocWithFlags((void**)&Z, bytes, hipDeviceMallocContiguous) != hipSuccess) {
      printf("%-34s rows/class %9zu: contiguous allocation refused\n", label, rows);
      (void)hipGetLastError();
      if (X) CK(hipFree(X));
      return -1;
    }
  } else {
    CK(hipMalloc(&X, bytes));
    CK(hipMalloc(&Z, bytes));
  }
  k_fill<<<4096, 256>>>(X, bytes / 16);
  k_fill<<<4096, 256>>>(Z, bytes / 16);
  const int blocks = g_blocks, B = 25600 / g_blocks, launches = 200;
  std::vector<int> hix((size_t)launches * blocks * B), hiz(hix.size());
  srand(7);
  for (size_t i = 0; i < hix.size(); ++i) {
    hix[i] = (int)(((size_t)rand() * 2654435761u + rand()) % rows);
    hiz[i] = (int)(((size_t)rand() * 2246822519u + rand()) % rows);
  }
  int *ix, *iz;
  double* out;
  CK(hipMalloc(&ix, hix.size() * 4));
  CK(hipMalloc(&iz, hiz.size() * 4));
  CK(hipMalloc(&out, blocks * 8));
  CK(hipMemcpy(ix, hix.data(), hix.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(iz, hiz.data(), hiz.size() * 4, hipMemcpyHostToDevice));
  for (int l = 0; l < 20; ++l)
    g_fn(blocks, X, Z, ix + (size_t)l * blocks * B, iz + (size_t)l * blocks * B, B, out);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int l = 0; l < launches; ++l)
    g_fn(blocks, X, Z, ix + (size_t)l * blocks * B, iz + (size_t)l * blocks * B, B, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / launches;
  printf("%-34s rows/class %9zu (%6.1f GB): %7.2f us/launch, %5.2f TB/s of rows\n", label, rows,
         2.0 * bytes / 1e9, us, 2.0 * blocks * B * 4096 / (us * 1e-6) / 1e12);
  CK(hipFree(X));
  CK(hipFree(Z));
  CK(hipFree(ix));
  CK(hipFree(iz));
  CK(hipFree(out));
  return us;
}

int main(int argc, char** argv) {
  const size_t sizes[] = {5000000, 100000};
  if (argc > 1 && !strcmp(argv[1], "alloc")) {
    for (int rep = 0; rep < 2; ++rep)
      for (size_t rows : sizes) {
        run("hipMalloc", rows, false);
        run("hipExtMallocWithFlags contiguous", rows, true);
      }
    return 0;
  }
  struct V { const char* name; LaunchFn fn; int blocks; };
  const V vs[] = {{"256 x 1024 thr, 2 pairs/wave", launch<1024, 2>, 256},
                  {"256 x 1024 thr, 4 pairs/wave", launch<1024, 4>, 256},
                  {"512 x 512 thr, 2 pairs/wave", launch<512, 2>, 512},
                  {"512 x 512 thr, 4 pairs/wave", launch<512, 4>, 512},
                  {"1024 x 256 thr, 2 pairs/wave", launch<256, 2>, 1024},
                  {"1024 x 256 thr, 4 pairs/wave", launch<256, 4>, 1024},
                  {"2560 x 256 thr, 1 pair/wave", launch<256, 1>, 2560},
                  {"6400 x 256 thr, 1 pair/wave", launch<256, 1>, 6400}};
  for (size_t rows : sizes)
    for (const V& v : vs) {
      g_fn = v.fn;
      g_blocks = v.blocks;
      run(v.name, rows, false);
    }
  return 0;
}
