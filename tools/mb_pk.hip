// Microbenchmark (design probe for the rank-image count kernel, not product code): can the
// all-pairs compare-count run on PACKED f32 ops?  Scores are replaced by integer-valued f32
// images (global ranks, < 2^24) so that, per pair, clamp(gx - gz) is exactly 1 when x > z and
// 0 otherwise.  Per x-pair of a lane and one wave-uniform z:
//     v_pk_add_f32 t, x01, nz op_sel_hi:[1,0] clamp     (nz = -gz from an SGPR, both halves)
//     v_pk_add_f32 acc, acc, t
// = 2 VALU wave-instructions per 128 pairs (1 per 64) against 1.5 VALU + 1 SALU per 64 for the
// f64 compare kernel (csrc/count.hip).  The shape is the bench's: 64 shards of 15625 x 15625,
// R x-images per lane, z chunks of ZC images streamed through the scalar cache.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_pk tools/mb_pk.hip && tools/mb_pk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kWave = 64, kBlock = 256;

// nz2 holds two negated z images (SGPR pair); HI selects which one both halves use
template <int HI>
__device__ __forceinline__ f2 gt_clamp(f2 x, unsigned long long nz2) {
  f2 t;
  if (HI)
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1] clamp" : "=v"(t) : "v"(x), "s"(nz2));
  else
    asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] clamp" : "=v"(t) : "v"(x), "s"(nz2));
  return t;
}
__device__ __forceinline__ void acc_add(f2& a, f2 t) {
  asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(t));
}

template <int R>
__global__ __launch_bounds__(kBlock) void k_pk(const float* __restrict__ gx, const float* __restrict__ nzs,
                                               int n_shards, int k, int tiles_x, int zchunks, int zc,
                                               unsigned long long* __restrict__ out) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int item = blockIdx.x * (kBlock / kWave) + wid;
  const int per_shard = tiles_x * zchunks;
  const int s = item / per_shard;
  if (s >= n_shards) return;
  const int rem = item - s * per_shard, cz = rem / tiles_x, tx = rem - cz * tiles_x;
  const int x0 = s * k + tx * kWave * R, xe = (s + 1) * k;
  const int kp = (k + 15) & ~15;  // z images: shard stride padded to 16 (aligned scalar loads)
  const int z0 = s * kp + cz * zc, z1 = min(z0 + zc, s * kp + k);
  f2 xv[R / 2], acc[R / 2];
#pragma unroll
  for (int p = 0; p < R / 2; ++p) {
    const int i0 = x0 + (2 * p) * kWave + lane, i1 = i0 + kWave;
    xv[p].x = i0 < xe ? gx[i0] : -3.0e7f;  // padded lanes: never greater
    xv[p].y = i1 < xe ? gx[i1] : -3.0e7f;
    acc[p] = f2{0.f, 0.f};
  }
  const unsigned long long* __restrict__ zp = (const unsigned long long*)(nzs + z0);  // z0 even
  const int nz = z1 - z0;
  int j = 0;
  for (; j + 16 <= nz; j += 16) {
    unsigned long long zz[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) zz[u] = zp[j / 2 + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f2 t[R / 2];  // all compares of one z first, then the adds: no adjacent dependence
#pragma unroll
      for (int p = 0; p < R / 2; ++p) t[p] = gt_clamp<0>(xv[p], zz[u]);
#pragma unroll
      for (int p = 0; p < R / 2; ++p) acc_add(acc[p], t[p]);
#pragma unroll
      for (int p = 0; p < R / 2; ++p) t[p] = gt_clamp<1>(xv[p], zz[u]);
#pragma unroll
      for (int p = 0; p < R / 2; ++p) acc_add(acc[p], t[p]);
    }
  }
  for (; j < nz; ++j) {  // odd tail: one z, both halves from the low word
    const unsigned long long zu = (unsigned long long)__float_as_uint(nzs[z0 + j]);
#pragma unroll
    for (int p = 0; p < R / 2; ++p) acc_add(acc[p], gt_clamp<0>(xv[p], zu));
  }
  unsigned long long tot = 0;
#pragma unroll
  for (int p = 0; p < R / 2; ++p) tot += (unsigned)acc[p].x + (unsigned)acc[p].y;
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, kWave);
  if (lane == 0 && tot) atomicAdd(out + s, tot);
}

// the same loop as a pure issue probe: no loads, z from a loop-carried SGPR
__global__ __launch_bounds__(kBlock) void k_issue(int iters, float seed, float* out) {
  f2 x0 = {seed + threadIdx.x, seed}, x1 = x0 * 2.f, x2 = x0 * 3.f, x3 = x0 * 5.f;
  f2 a0 = {0, 0}, a1 = a0, a2 = a0, a3 = a0;
  unsigned long long z = (unsigned long long)__builtin_amdgcn_readfirstlane((int)seed) * 0x100000001ull;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc_add(a0, gt_clamp<0>(x0, z)); acc_add(a1, gt_clamp<1>(x1, z));
      acc_add(a2, gt_clamp<0>(x2, z)); acc_add(a3, gt_clamp<1>(x3, z));
    }
  }
  out[blockIdx.x * kBlock + threadIdx.x] = a0.x + a1.y + a2.x + a3.y;
}

template <int R>
void run(const char* name, const float* dx, const float* dz, int S, int k, int zc, unsigned long long* dout,
         const std::vector<unsigned long long>& want) {
  const int tiles_x = (k + kWave * R - 1) / (kWave * R), zchunks = (k + zc - 1) / zc;
  const long items = (long)S * tiles_x * zchunks, blocks = (items + 3) / 4;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  std::vector<unsigned long long> got(S);
  float best = 1e9, sum = 0; int reps = 20;
  for (int r = -3; r < reps; ++r) {
    CK(hipMemset(dout, 0, S * 8));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_pk<R>, dim3(blocks), dim3(kBlock), 0, 0, dx, dz, S, k, tiles_x, zchunks, zc, dout);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 0) { best = std::min(best, ms); sum += ms; }
  }
  CK(hipMemcpy(got.data(), dout, S * 8, hipMemcpyDeviceToHost));
  const bool ok = got == want;
  const double pairs = (double)S * k * k, mean = sum / reps;
  printf("%-10s R=%d zc=%4d blocks=%6ld  mean %.4f ms  best %.4f ms  %.3e pairs/s  frac(3.93e13) %.3f  %s\n",
         name, R, zc, blocks, mean, best, pairs / (mean * 1e-3), pairs / (mean * 1e-3) / 3.93216e13,
         ok ? "counts OK" : "COUNTS DIFFER");
}

int main() {
  {  // issue probe
    const int blocks = 256 * 8, iters = 2048;
    float* o; CK(hipMalloc(&o, blocks * kBlock * 4));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_issue, dim3(blocks), dim3(kBlock), 0, 0, iters, 3.0f, o);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      const double wi = (double)blocks * 4 * iters * 8 * 8;  // wave-instructions
      printf("issue probe: %.3f ms  %.3f wave-instr/cycle/CU @2.4GHz  -> %.3e pairs/s (128 per 2 instr)\n", ms,
             wi / (ms * 1e-3) / 256 / 2.4e9, wi * 64 / (ms * 1e-3));
    }
    CK(hipFree(o));
  }
  const int S = 64, k = 15625, n = S * k;
  const int kp = (k + 15) & ~15;
  std::vector<float> gx(n), nz((size_t)S * kp, 0.f);
  srand(7);
  for (int i = 0; i < n; ++i) gx[i] = (float)(rand() % 2000000);
  for (int s = 0; s < S; ++s)
    for (int i = 0; i < k; ++i) nz[(size_t)s * kp + i] = -(float)(rand() % 2000000);
  gx[5] = -2.0e7f;  // a NaN-like sentinel on the x side
  nz[7] = -3.0e7f;  // and on the z side (never less than any x)
  std::vector<unsigned long long> want(S, 0);
  for (int s = 0; s < S; ++s) {
    std::vector<float> zs(nz.begin() + (size_t)s * kp, nz.begin() + (size_t)s * kp + k);
    for (auto& v : zs) v = -v;
    std::sort(zs.begin(), zs.end());
    for (int i = 0; i < k; ++i)
      want[s] += std::lower_bound(zs.begin(), zs.end(), gx[s * k + i]) - zs.begin();
  }
  float *dx, *dz; unsigned long long* dout;
  CK(hipMalloc(&dx, n * 4)); CK(hipMalloc(&dz, (size_t)S * kp * 4)); CK(hipMalloc(&dout, S * 8));
  CK(hipMemcpy(dx, gx.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dz, nz.data(), (size_t)S * kp * 4, hipMemcpyHostToDevice));
  for (int zc : {528, 1056, 2048, 4000}) {
    run<8>("pk", dx, dz, S, k, zc, dout, want);
    run<16>("pk", dx, dz, S, k, zc, dout, want);
  }
  run<4>("pk", dx, dz, S, k, 528, dout, want);
  return 0;
}
