// permute.hip — device-side repartition.
//
// The reference repartitions by shuffling the caller's arrays in place with NumPy's global
// RNG (compute_stats.py:66-67, estimation-experiment/main.py:43-44) and slicing consecutive
// blocks.  Bit-exact drop-in calls keep doing exactly that on the host.  The device-resident
// path (bench.py, tuplewise.device) instead draws a keyed pseudo-random bijection of [0, n)
// on the GPU: a 6-round balanced Feistel network on the smallest even-bit power-of-two domain
// >= n, with cycle walking to stay inside [0, n).  Every rank of a multi-GPU job evaluates the
// same bijection for its own global indices, so the permuted global array — and therefore
// every shard's count — is identical at 1, 2, 4 and 8 GPUs.
#include "tw_common.h"
#include <algorithm>

namespace tw {

struct Feistel {
  uint32_t half_bits;
  uint32_t mask;
  uint32_t k[6];
};

__host__ __device__ inline uint32_t mix32(uint32_t v) {  // murmur3 finaliser
  v ^= v >> 16;
  v *= 0x85EBCA6Bu;
  v ^= v >> 13;
  v *= 0xC2B2AE35u;
  v ^= v >> 16;
  return v;
}

inline Feistel make_feistel(int64_t n, uint64_t key) {
  Feistel f;
  int bits = 2;
  while (bits < 62 && (1ll << bits) < n) ++bits;
  if (bits & 1) ++bits;
  f.half_bits = bits / 2;
  f.mask = (uint32_t)((1ull << f.half_bits) - 1);
  uint64_t st = key ^ 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 6; ++i) {  // splitmix64 key schedule
    st += 0x9E3779B97F4A7C15ull;
    uint64_t zz = st;
    zz = (zz ^ (zz >> 30)) * 0xBF58476D1CE4E5B9ull;
    zz = (zz ^ (zz >> 27)) * 0x94D049BB133111EBull;
    zz ^= zz >> 31;
    f.k[i] = (uint32_t)zz;
  }
  return f;
}

__host__ __device__ inline uint64_t feistel_once(const Feistel& f, uint64_t v) {
  uint32_t L = (uint32_t)(v >> f.half_bits) & f.mask;
  uint32_t R = (uint32_t)v & f.mask;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint32_t nL = R;
    R = (L ^ mix32(R * 0x9E3779B1u + f.k[i])) & f.mask;
    L = nL;
  }
  return ((uint64_t)L << f.half_bits) | R;
}

__host__ __device__ inline uint64_t feistel_perm(const Feistel& f, uint64_t i, uint64_t n) {
  uint64_t v = feistel_once(f, i);
  while (v >= n) v = feistel_once(f, v);  // cycle walking: terminates (bijection on domain)
  return v;
}

__global__ __launch_bounds__(kBlock) void k_permute_scatter(const uint64_t* __restrict__ in,
                                                            uint64_t* __restrict__ out,
                                                            int64_t n, Feistel f) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    out[feistel_perm(f, (uint64_t)i, (uint64_t)n)] = in[i];
}

__global__ __launch_bounds__(kBlock) void k_perm_index(int64_t* __restrict__ perm, int64_t n,
                                                       int64_t base, int64_t n_total, Feistel f) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    perm[i] = (int64_t)feistel_perm(f, (uint64_t)(base + i), (uint64_t)n_total);
}


// ---- multi-rank exchange: element g of rank r moves to global position
// perm(g); its destination rank is perm(g) / n_loc.  Counting sort by destination rank:
// a histogram pass, an exclusive scan on the host side of the collective, then a scatter that
// packs {value bits, destination-local position} records per destination (order inside a
// destination bucket is irrelevant: the position travels with the value).
__global__ __launch_bounds__(kBlock) void k_rank_histogram(const int64_t* __restrict__ perm,
                                                           int64_t n, int64_t n_loc, int G,
                                                           unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[64];
  for (int i = threadIdx.x; i < G; i += kBlock) h[i] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    atomicAdd(&h[(int)(perm[i] / n_loc)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (h[i]) atomicAdd(counts + i, (unsigned long long)h[i]);
}

__global__ __launch_bounds__(kBlock) void k_bucket_scatter(const int64_t* __restrict__ perm,
                                                           const uint64_t* __restrict__ vals,
                                                           int64_t n, int64_t n_loc,
                                                           const int64_t* __restrict__ start,
                                                           unsigned long long* __restrict__ cursor,
                                                           uint64_t* __restrict__ send) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t pg = perm[i];
    const int dst = (int)(pg / n_loc);
    const unsigned long long slot = atomicAdd(cursor + dst, 1ull);
    const int64_t o = start[dst] + (int64_t)slot;
    send[2 * o] = vals[i];
    send[2 * o + 1] = (uint64_t)(pg - (int64_t)dst * n_loc);
  }
}

__global__ __launch_bounds__(kBlock) void k_scatter_records(const uint64_t* __restrict__ rec,
                                                            int64_t m, uint64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * kBlock)
    out[rec[2 * i + 1]] = rec[2 * i];
}

}  // namespace tw

using namespace tw;

extern "C" int tw_permute_scatter(const void* d_in, void* d_out, int64_t n, uint64_t key,
                                  void* stream) {
  TW_ARG_CHECK(n >= 0 && n < (1ll << 60), "tw_permute_scatter: bad n");
  TW_ARG_CHECK(n == 0 || d_in != d_out, "tw_permute_scatter: in-place not supported");
  if (n == 0) return TW_OK;
  const Feistel f = make_feistel(n, key);
  const int blocks = (int)std::min<int64_t>(256 * 8, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_permute_scatter, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_in, (uint64_t*)d_out, n, f);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_perm_index(int64_t* d_perm, int64_t n, int64_t base, int64_t n_total,
                             uint64_t key, void* stream) {
  TW_ARG_CHECK(n >= 0 && base >= 0 && base + n <= n_total && n_total < (1ll << 60),
               "tw_perm_index: bad range");
  if (n == 0) return TW_OK;
  const Feistel f = make_feistel(n_total, key);
  const int blocks = (int)std::min<int64_t>(256 * 8, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_perm_index, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, d_perm,
                     n, base, n_total, f);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_rank_histogram(const int64_t* d_perm, int64_t n, int64_t n_loc, int32_t G,
                                 uint64_t* d_counts, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= 64 && n >= 0 && n_loc >= 1, "tw_rank_histogram: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(uint64_t) * G, st));
  if (n == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 4, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_rank_histogram, dim3(blocks), dim3(kBlock), 0, st, d_perm, n, n_loc, (int)G,
                     (unsigned long long*)d_counts);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_bucket_scatter(const int64_t* d_perm, const void* d_vals, int64_t n,
                                 int64_t n_loc, int32_t G, const int64_t* d_start,
                                 uint64_t* d_cursor, void* d_send, void* stream) {
  TW_ARG_CHECK(G >= 1 && n >= 0 && n_loc >= 1, "tw_bucket_scatter: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(hipMemsetAsync(d_cursor, 0, sizeof(uint64_t) * G, st));
  if (n == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 8, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_bucket_scatter, dim3(blocks), dim3(kBlock), 0, st, d_perm,
                     (const uint64_t*)d_vals, n, n_loc, d_start, (unsigned long long*)d_cursor,
                     (uint64_t*)d_send);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_scatter_records(const void* d_rec, int64_t m, void* d_out, void* stream) {
  TW_ARG_CHECK(m >= 0, "tw_scatter_records: bad size");
  if (m == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 8, ceil_div(m, kBlock));
  hipLaunchKernelGGL(k_scatter_records, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_rec, m, (uint64_t*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
