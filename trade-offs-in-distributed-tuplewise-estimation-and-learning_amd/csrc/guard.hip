// guard.hip — the carried rank images' validity check.
//
// ShardedSample.UnN_many carries the rank-image records of its final arrays to the next call
// (device.py CARRY_IMAGES): a repartition only permutes a sample, never changes its values
// (estimation-experiment/main.py:43-44, the in-place shuffles), so the images stay valid while
// nobody writes the arrays.  torch's version counter misses writes through `.data`, DLPack
// aliases or a foreign kernel.  This entry hashes the arrays' words, position-keyed, into one
// 64-bit sum when the images are saved and again when they are about to be reused, and writes
// a verdict word (`good` when the sums agree, `bad` otherwise) that the host reads after the
// call's counts — the call is redone from a fresh ranking when it reads `bad`.
//
// HBM-bound: 8 B read per score, one pass; a 64-bit add per word; one atomic per wave.
#include "tw_common.h"

namespace tw {
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64's finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// sum over words i of mix64(word_i ^ i * golden): a value change at any position, or two
// positions exchanging unequal values, changes the sum (but for a 2^-64 collision).  One
// partial per block (no atomics: 2000 same-address atomics serialised at one L2 channel cost the
// first build ~0.2 ms per call, profiles/r06s11_chain_probe.log), summed by the verdict block.
constexpr int kHashBlocks = 256;

__global__ __launch_bounds__(256) void k_words_hash(const uint64_t* __restrict__ a, int64_t na,
                                                    const uint64_t* __restrict__ b, int64_t nb,
                                                    uint64_t* __restrict__ partial) {
  const int64_t n = na + nb;
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint64_t s = 0;
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += stride) {
    const uint64_t w = i < na ? __builtin_nontemporal_load(a + i)
                              : __builtin_nontemporal_load(b + (i - na));
    s += mix64(w ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull));
  }
  s = wave_sum_u64(s);
  __shared__ uint64_t ws[4];
  if ((threadIdx.x & (kWave - 1)) == 0) ws[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// acc[0] = the sum of the blocks' partials (acc[1 ..]); with expect: the verdict word
__global__ __launch_bounds__(256) void k_words_verdict(uint64_t* __restrict__ acc, int nparts,
                                                       const uint64_t* __restrict__ expect,
                                                       int64_t* __restrict__ verdict,
                                                       int64_t good, int64_t bad) {
  uint64_t s = (int)threadIdx.x < nparts ? acc[1 + threadIdx.x] : 0ull;
  s = wave_sum_u64(s);
  __shared__ uint64_t ws[4];
  if ((threadIdx.x & (kWave - 1)) == 0) ws[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t tot = ws[0] + ws[1] + ws[2] + ws[3];
    acc[0] = tot;
    if (verdict) verdict[0] = tot == expect[0] ? good : bad;
  }
}

}  // namespace
}  // namespace tw

using namespace tw;

extern "C" int tw_words_checksum(const void* d_a, int64_t na, const void* d_b, int64_t nb,
                                 void* d_acc, const void* d_expect, void* d_verdict,
                                 int64_t good, int64_t bad, void* stream) {
  TW_ARG_CHECK(na >= 0 && nb >= 0 && d_acc != nullptr && (na == 0 || d_a != nullptr) &&
                   (nb == 0 || d_b != nullptr),
               "tw_words_checksum: bad sizes or null buffers");
  TW_ARG_CHECK((d_expect == nullptr) == (d_verdict == nullptr),
               "tw_words_checksum: expect and verdict go together");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = na + nb;
  // one block per CU at most, ~8 words per thread at the chain sizes (2e6 words: 256 blocks)
  const int g = (int)std::min<int64_t>(kHashBlocks, std::max<int64_t>(1, ceil_div(n, 2048)));
  uint64_t* acc = (uint64_t*)d_acc;
  hipLaunchKernelGGL(k_words_hash, dim3(g), dim3(256), 0, st, (const uint64_t*)d_a, na,
                     (const uint64_t*)d_b, nb, acc + 1);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_words_verdict, dim3(1), dim3(256), 0, st, acc, g,
                     (const uint64_t*)d_expect, (int64_t*)d_verdict, good, bad);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int64_t tw_words_checksum_acc_words(void) { return 1 + kHashBlocks; }
