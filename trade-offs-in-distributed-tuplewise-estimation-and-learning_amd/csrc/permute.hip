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
#include "feistel.h"
#include <algorithm>

namespace tw {

// out[perm(i)] = in[i], evaluated as a GATHER out[p] = in[perm^-1(p)]: the writes are
// coalesced and the random 8-byte reads hit the L2 / Infinity Cache (the input was just read
// by the previous count), where a scatter would pay a partial-line write per element.
// Two arrays (the X and Z samples of one repartition) share one launch.
__global__ __launch_bounds__(kBlock) void k_permute_gather2(
    const uint64_t* __restrict__ a_in, uint64_t* __restrict__ a_out, int64_t na, Feistel fa,
    const uint64_t* __restrict__ b_in, uint64_t* __restrict__ b_out, int64_t nb, Feistel fb) {
  for (int64_t p = blockIdx.x * (int64_t)kBlock + threadIdx.x; p < na + nb;
       p += (int64_t)gridDim.x * kBlock) {
    if (p < na)
      a_out[p] = a_in[feistel_perm_inv(fa, (uint64_t)p, (uint64_t)na)];
    else
      b_out[p - na] = b_in[feistel_perm_inv(fb, (uint64_t)(p - na), (uint64_t)nb)];
  }
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
// The receive side needs no message to size its buffers: position p of rank r is filled from
// global source perm^-1(p), so k_source_histogram counts, per source rank, what r will receive.
constexpr int kMaxG = 64;
__global__ __launch_bounds__(kBlock) void k_rank_histogram(const int64_t* __restrict__ perm,
                                                           int64_t n, int64_t n_loc, int G,
                                                           unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[kMaxG];
  for (int i = threadIdx.x; i < G; i += kBlock) h[i] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    atomicAdd(&h[(int)(perm[i] / n_loc)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (h[i]) atomicAdd(counts + i, (unsigned long long)h[i]);
}

__global__ __launch_bounds__(kBlock) void k_source_histogram(int64_t n, int64_t base,
                                                             uint64_t n_total, int64_t n_loc,
                                                             int G, Feistel f,
                                                             unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[kMaxG];
  for (int i = threadIdx.x; i < G; i += kBlock) h[i] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    atomicAdd(&h[(int)((int64_t)feistel_perm_inv(f, (uint64_t)(base + i), n_total) / n_loc)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (h[i]) atomicAdd(counts + i, (unsigned long long)h[i]);
}

// Records of a chunk of kScatChunk consecutive elements are placed with ONE global
// reservation per (block, destination): LDS counters give each element its rank inside the
// block's share of a bucket.  (A global atomic per element would serialise ~n/G returning
// atomics on each of G cursor words.)
constexpr int kScatPer = 8;
constexpr int kScatChunk = kBlock * kScatPer;
__global__ __launch_bounds__(kBlock) void k_bucket_scatter(const int64_t* __restrict__ perm,
                                                           const uint64_t* __restrict__ vals,
                                                           int64_t n, int64_t n_loc, int G,
                                                           const int64_t* __restrict__ start,
                                                           unsigned long long* __restrict__ cursor,
                                                           int64_t pos_base,
                                                           uint64_t* __restrict__ send) {
  __shared__ unsigned int lcnt[kMaxG];
  __shared__ int64_t lbase[kMaxG];
  for (int64_t c0 = (int64_t)blockIdx.x * kScatChunk; c0 < n;
       c0 += (int64_t)gridDim.x * kScatChunk) {
    for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
    __syncthreads();
    int dst[kScatPer];
    unsigned slot[kScatPer];
    int64_t pos[kScatPer];
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      const int64_t i = c0 + k * kBlock + threadIdx.x;
      dst[k] = -1;
      if (i < n) {
        const int64_t pg = perm[i];
        dst[k] = (int)(pg / n_loc);
        pos[k] = pg - (int64_t)dst[k] * n_loc;
        slot[k] = atomicAdd(&lcnt[dst[k]], 1u);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += kBlock)
      if (lcnt[i]) lbase[i] = start[i] + (int64_t)atomicAdd(cursor + i, (unsigned long long)lcnt[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      if (dst[k] >= 0) {
        const int64_t o = lbase[dst[k]] + slot[k];
        send[2 * o] = vals[c0 + k * kBlock + threadIdx.x];
        send[2 * o + 1] = (uint64_t)(pos[k] + pos_base);
      }
    }
    __syncthreads();  // lcnt / lbase are reset by the next chunk
  }
}

// ---- the fused exchange of ONE repartition of both samples (what ShardedSample runs): two
// launches instead of perm_index/histogram/scan/scatter per array, and no permutation array.
//   k_exchange_counts: per element of the X and Z slices owned here, the destination rank
//     (forward permutation) and, per local position, the source rank (inverse permutation);
//     counts[0..G) send X, [G..2G) receive X, [2G..3G) send Z, [3G..4G) receive Z.  Also
//     zeroes the 2G pack cursors.
//   k_exchange_pack: records {value, position} bucketed by destination rank, each bucket
//     [X records | Z records], Z positions offset by n_loc; bucket starts are prefix sums of
//     the send counts, computed by every block (G <= 64).
__global__ __launch_bounds__(kBlock) void k_exchange_counts(int64_t n_loc, int64_t m_loc,
                                                            int64_t xbase, int64_t zbase, int G,
                                                            Feistel fx, Feistel fz,
                                                            unsigned long long* __restrict__ counts,
                                                            unsigned long long* __restrict__ cursor) {
  __shared__ unsigned int h[4 * kMaxG];
  for (int i = threadIdx.x; i < 4 * G; i += kBlock) h[i] = 0;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < 2 * G; i += kBlock) cursor[i] = 0;
  __syncthreads();
  const uint64_t NX = (uint64_t)n_loc * G, NZ = (uint64_t)m_loc * G;
  const FastDiv dx = make_fastdiv((uint64_t)n_loc), dz = make_fastdiv((uint64_t)m_loc);
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < n_loc + m_loc;
       e += (int64_t)gridDim.x * kBlock) {
    if (e < n_loc) {
      const uint64_t g = (uint64_t)(xbase + e);
      atomicAdd(&h[(int)fast_div(feistel_perm(fx, g, NX), dx)], 1u);
      atomicAdd(&h[G + (int)fast_div(feistel_perm_inv(fx, g, NX), dx)], 1u);
    } else {
      const uint64_t g = (uint64_t)(zbase + e - n_loc);
      atomicAdd(&h[2 * G + (int)fast_div(feistel_perm(fz, g, NZ), dz)], 1u);
      atomicAdd(&h[3 * G + (int)fast_div(feistel_perm_inv(fz, g, NZ), dz)], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * G; i += kBlock)
    if (h[i]) atomicAdd(counts + i, (unsigned long long)h[i]);
}

__global__ __launch_bounds__(kBlock) void k_exchange_pack(
    const uint64_t* __restrict__ xv, int64_t n_loc, const uint64_t* __restrict__ zv,
    int64_t m_loc, int64_t xbase, int64_t zbase, int G, Feistel fx, Feistel fz,
    const unsigned long long* __restrict__ counts, unsigned long long* __restrict__ cursor,
    uint64_t* __restrict__ send) {
  __shared__ int64_t start[2 * kMaxG];  // bucket start of X (g) and Z (G + g) records
  __shared__ unsigned int lcnt[2 * kMaxG];
  __shared__ int64_t lbase[2 * kMaxG];
  if (threadIdx.x == 0) {
    int64_t o = 0;
    for (int g = 0; g < G; ++g) {
      start[g] = o;
      start[G + g] = o + (int64_t)counts[g];
      o += (int64_t)counts[g] + (int64_t)counts[2 * G + g];
    }
  }
  const uint64_t NX = (uint64_t)n_loc * G, NZ = (uint64_t)m_loc * G;
  const FastDiv dx = make_fastdiv((uint64_t)n_loc), dz = make_fastdiv((uint64_t)m_loc);
  const int64_t tot = n_loc + m_loc;
  for (int64_t c0 = (int64_t)blockIdx.x * kScatChunk; c0 < tot;
       c0 += (int64_t)gridDim.x * kScatChunk) {
    for (int i = threadIdx.x; i < 2 * G; i += kBlock) lcnt[i] = 0;
    __syncthreads();
    int bucket[kScatPer];
    unsigned slot[kScatPer];
    int64_t pos[kScatPer];
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      const int64_t e = c0 + k * kBlock + threadIdx.x;
      bucket[k] = -1;
      if (e < n_loc) {
        const int64_t p = (int64_t)feistel_perm(fx, (uint64_t)(xbase + e), NX);
        const int dst = (int)fast_div((uint64_t)p, dx);
        bucket[k] = dst;
        pos[k] = p - (int64_t)dst * n_loc;
      } else if (e < tot) {
        const int64_t p = (int64_t)feistel_perm(fz, (uint64_t)(zbase + e - n_loc), NZ);
        const int dst = (int)fast_div((uint64_t)p, dz);
        bucket[k] = G + dst;
        pos[k] = p - (int64_t)dst * m_loc + n_loc;  // Z follows X in the receive buffer
      }
      if (bucket[k] >= 0) slot[k] = atomicAdd(&lcnt[bucket[k]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * G; i += kBlock)
      if (lcnt[i]) lbase[i] = start[i] + (int64_t)atomicAdd(cursor + i, (unsigned long long)lcnt[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      if (bucket[k] >= 0) {
        const int64_t e = c0 + k * kBlock + threadIdx.x;
        const int64_t o = lbase[bucket[k]] + slot[k];
        send[2 * o] = e < n_loc ? xv[e] : zv[e - n_loc];
        send[2 * o + 1] = (uint64_t)pos[k];
      }
    }
    __syncthreads();
  }
}

// ---- fixed-capacity exchange: no split sizes on the host, ONE Feistel pass per element.
// The send buffer is G buckets of (1 + cap) 16-byte records; bucket g = [header {count, 0} |
// up to cap records {value bits, position at g}], X and Z records mixed (Z positions offset by
// n_loc).  Equal-size buckets make the all-to-all a plain equal-split one whose sizes every rank
// knows, so a repartition needs no count pass, no inverse permutation and no host round trip.
// cap is the expected bucket size (n_loc + m_loc) / G plus a margin of dozens of standard
// deviations; a bucket that would overflow sets *flag (records past cap are dropped) and the
// host refuses the result.
__global__ __launch_bounds__(kBlock) void k_exchange_pack_fixed(
    const uint64_t* __restrict__ xv, int64_t n_loc, const uint64_t* __restrict__ zv,
    int64_t m_loc, int64_t xbase, int64_t zbase, int G, Feistel fx, Feistel fz, int64_t cap,
    unsigned long long* __restrict__ cursor, uint64_t* __restrict__ send, int* __restrict__ flag) {
  __shared__ unsigned int lcnt[kMaxG];
  __shared__ int64_t lbase[kMaxG];
  const uint64_t NX = (uint64_t)n_loc * G, NZ = (uint64_t)m_loc * G;
  const FastDiv dx = make_fastdiv((uint64_t)n_loc), dz = make_fastdiv((uint64_t)m_loc);
  const int64_t tot = n_loc + m_loc, bsz = cap + 1;
  for (int64_t c0 = (int64_t)blockIdx.x * kScatChunk; c0 < tot;
       c0 += (int64_t)gridDim.x * kScatChunk) {
    for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
    __syncthreads();
    int dst[kScatPer];
    unsigned slot[kScatPer];
    int64_t pos[kScatPer];
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      const int64_t e = c0 + k * kBlock + threadIdx.x;
      dst[k] = -1;
      if (e < n_loc) {
        const uint64_t p = feistel_perm(fx, (uint64_t)(xbase + e), NX);
        dst[k] = (int)fast_div(p, dx);
        pos[k] = (int64_t)p - (int64_t)dst[k] * n_loc;
      } else if (e < tot) {
        const uint64_t p = feistel_perm(fz, (uint64_t)(zbase + e - n_loc), NZ);
        dst[k] = (int)fast_div(p, dz);
        pos[k] = (int64_t)p - (int64_t)dst[k] * m_loc + n_loc;
      }
      if (dst[k] >= 0) slot[k] = atomicAdd(&lcnt[dst[k]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += kBlock)
      if (lcnt[i]) lbase[i] = (int64_t)atomicAdd(cursor + i, (unsigned long long)lcnt[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScatPer; ++k) {
      if (dst[k] >= 0) {
        const int64_t o = lbase[dst[k]] + slot[k];
        if (o < cap) {
          const int64_t e = c0 + k * kBlock + threadIdx.x;
          uint64_t* r = send + 2 * (dst[k] * bsz + 1 + o);
          r[0] = e < n_loc ? xv[e] : zv[e - n_loc];
          r[1] = (uint64_t)pos[k];
        } else {
          *flag = 1;
        }
      }
    }
    __syncthreads();
  }
}

// Bucket headers from the cursors (then zeroed for the next repartition).
__global__ void k_exchange_seal(int G, int64_t cap, unsigned long long* __restrict__ cursor,
                                uint64_t* __restrict__ send, int* __restrict__ flag) {
  const int g = threadIdx.x;
  if (g < G) {
    const unsigned long long c = cursor[g];
    send[2 * (g * (cap + 1))] = c;
    send[2 * (g * (cap + 1)) + 1] = 0;
    cursor[g] = 0;
    if (c > (unsigned long long)cap) *flag = 1;
  }
}

// Receive side: bucket g's first min(header, cap) records, out[pos] = value.  A header past cap
// or a position outside [0, n_out) flags the exchange instead of writing.
__global__ __launch_bounds__(kBlock) void k_scatter_buckets(const uint64_t* __restrict__ recv,
                                                            int G, int64_t cap,
                                                            uint64_t* __restrict__ out,
                                                            int64_t n_out, int* __restrict__ flag) {
  const int64_t bsz = cap + 1, tot = (int64_t)G * cap;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t g = i / cap, r = i - g * cap;
    const uint64_t c = recv[2 * (g * bsz)];
    if (c > (uint64_t)cap) *flag = 1;
    if ((uint64_t)r < c && r < cap) {
      const uint64_t* q = recv + 2 * (g * bsz + 1 + r);
      const uint64_t p = q[1];
      if (p < (uint64_t)n_out)
        out[p] = q[0];
      else
        *flag = 1;
    }
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

static int launch_permute2(const void* a_in, void* a_out, int64_t na, uint64_t ka,
                           const void* b_in, void* b_out, int64_t nb, uint64_t kb,
                           hipStream_t st) {
  const Feistel fa = make_feistel(std::max<int64_t>(na, 1), ka);
  const Feistel fb = make_feistel(std::max<int64_t>(nb, 1), kb);
  const int blocks = (int)std::min<int64_t>(256 * 16, ceil_div(na + nb, kBlock));
  hipLaunchKernelGGL(k_permute_gather2, dim3(blocks), dim3(kBlock), 0, st,
                     (const uint64_t*)a_in, (uint64_t*)a_out, na, fa, (const uint64_t*)b_in,
                     (uint64_t*)b_out, nb, fb);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_permute_scatter(const void* d_in, void* d_out, int64_t n, uint64_t key,
                                  void* stream) {
  TW_ARG_CHECK(n >= 0 && n < (1ll << 60), "tw_permute_scatter: bad n");
  TW_ARG_CHECK(n == 0 || d_in != d_out, "tw_permute_scatter: in-place not supported");
  if (n == 0) return TW_OK;
  return launch_permute2(d_in, d_out, n, key, nullptr, nullptr, 0, 0, (hipStream_t)stream);
}

extern "C" int tw_permute_pair(const void* d_x_in, void* d_x_out, int64_t n, uint64_t key_x,
                               const void* d_z_in, void* d_z_out, int64_t m, uint64_t key_z,
                               void* stream) {
  TW_ARG_CHECK(n >= 0 && m >= 0 && n < (1ll << 60) && m < (1ll << 60),
               "tw_permute_pair: bad sizes");
  TW_ARG_CHECK((n == 0 || d_x_in != d_x_out) && (m == 0 || d_z_in != d_z_out),
               "tw_permute_pair: in-place not supported");
  if (n + m == 0) return TW_OK;
  return launch_permute2(d_x_in, d_x_out, n, key_x, d_z_in, d_z_out, m, key_z,
                         (hipStream_t)stream);
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
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && n >= 0 && n_loc >= 1, "tw_rank_histogram: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_counts, 0, sizeof(uint64_t) * G, st));
  if (n == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 4, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_rank_histogram, dim3(blocks), dim3(kBlock), 0, st, d_perm, n, n_loc, (int)G,
                     (unsigned long long*)d_counts);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_source_histogram(int64_t n, int64_t base, int64_t n_total, uint64_t key,
                                   int64_t n_loc, int32_t G, uint64_t* d_counts, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && n >= 0 && n_loc >= 1 && base >= 0 &&
                   base + n <= n_total && n_total <= n_loc * (int64_t)G && n_total < (1ll << 60),
               "tw_source_histogram: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_counts, 0, sizeof(uint64_t) * G, st));
  if (n == 0) return TW_OK;
  const Feistel f = make_feistel(n_total, key);
  const int blocks = (int)std::min<int64_t>(256 * 4, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_source_histogram, dim3(blocks), dim3(kBlock), 0, st, n, base,
                     (uint64_t)n_total, n_loc, (int)G, f, (unsigned long long*)d_counts);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_bucket_scatter(const int64_t* d_perm, const void* d_vals, int64_t n,
                                 int64_t n_loc, int32_t G, const int64_t* d_start,
                                 uint64_t* d_cursor, int64_t pos_base, void* d_send,
                                 void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && n >= 0 && n_loc >= 1 && pos_base >= 0,
               "tw_bucket_scatter: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_cursor, 0, sizeof(uint64_t) * G, st));
  if (n == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(256 * 4, ceil_div(n, kScatChunk));
  hipLaunchKernelGGL(k_bucket_scatter, dim3(blocks), dim3(kBlock), 0, st, d_perm,
                     (const uint64_t*)d_vals, n, n_loc, (int)G, d_start,
                     (unsigned long long*)d_cursor, pos_base, (uint64_t*)d_send);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// Grid cap for the exchange kernels, which run beside the previous step's count kernel:
// fewer blocks take fewer of its CU slots.  World-size-1 probe (tools/multi_path_probe.py,
// profiles/r01_multi_path_probe.log): 1024-2048 blocks 1.00 ms/step, 128-256 blocks 0.925,
// 32-64 blocks 1.00-1.04 (the exchange then outlasts the count); one-GPU path 0.87.
// Tuning hook tw_exchange_set_grid (0 = this default).
constexpr int kExchangeGrid = 128;
static int g_exchange_grid = 0;
static int exchange_grid(int) { return g_exchange_grid > 0 ? g_exchange_grid : kExchangeGrid; }

extern "C" int tw_exchange_set_grid(int32_t blocks) {
  TW_ARG_CHECK(blocks >= 0, "tw_exchange_set_grid: blocks >= 0");
  g_exchange_grid = blocks;
  return TW_OK;
}

extern "C" int tw_exchange_counts(int64_t n_loc, int64_t m_loc, int32_t rank, int32_t G,
                                  uint64_t key_x, uint64_t key_z, uint64_t* d_counts,
                                  uint64_t* d_cursor, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && rank >= 0 && rank < G && n_loc >= 1 && m_loc >= 1 &&
                   n_loc * (int64_t)G < (1ll << 60) && m_loc * (int64_t)G < (1ll << 60),
               "tw_exchange_counts: bad sizes");
  TW_ARG_CHECK(d_counts && d_cursor, "tw_exchange_counts: null pointer");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_counts, 0, sizeof(uint64_t) * 4 * G, st));
  const Feistel fx = make_feistel(n_loc * (int64_t)G, key_x);
  const Feistel fz = make_feistel(m_loc * (int64_t)G, key_z);
  const int blocks = (int)std::min<int64_t>(exchange_grid(256 * 4), ceil_div(n_loc + m_loc, kBlock));
  hipLaunchKernelGGL(k_exchange_counts, dim3(blocks), dim3(kBlock), 0, st, n_loc, m_loc,
                     (int64_t)rank * n_loc, (int64_t)rank * m_loc, (int)G, fx, fz,
                     (unsigned long long*)d_counts, (unsigned long long*)d_cursor);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_exchange_pack(const void* d_x, int64_t n_loc, const void* d_z, int64_t m_loc,
                                int32_t rank, int32_t G, uint64_t key_x, uint64_t key_z,
                                const uint64_t* d_counts, uint64_t* d_cursor, void* d_send,
                                void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && rank >= 0 && rank < G && n_loc >= 1 && m_loc >= 1 &&
                   n_loc * (int64_t)G < (1ll << 60) && m_loc * (int64_t)G < (1ll << 60),
               "tw_exchange_pack: bad sizes");
  TW_ARG_CHECK(d_x && d_z && d_counts && d_cursor && d_send, "tw_exchange_pack: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const Feistel fx = make_feistel(n_loc * (int64_t)G, key_x);
  const Feistel fz = make_feistel(m_loc * (int64_t)G, key_z);
  const int blocks = (int)std::min<int64_t>(exchange_grid(256 * 4), ceil_div(n_loc + m_loc, kScatChunk));
  hipLaunchKernelGGL(k_exchange_pack, dim3(blocks), dim3(kBlock), 0, st, (const uint64_t*)d_x,
                     n_loc, (const uint64_t*)d_z, m_loc, (int64_t)rank * n_loc,
                     (int64_t)rank * m_loc, (int)G, fx, fz, (const unsigned long long*)d_counts,
                     (unsigned long long*)d_cursor, (uint64_t*)d_send);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_exchange_pack_fixed(const void* d_x, int64_t n_loc, const void* d_z,
                                      int64_t m_loc, int32_t rank, int32_t G, uint64_t key_x,
                                      uint64_t key_z, int64_t cap, uint64_t* d_cursor,
                                      void* d_send, int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && rank >= 0 && rank < G && n_loc >= 1 && m_loc >= 1 &&
                   n_loc * (int64_t)G < (1ll << 52) && m_loc * (int64_t)G < (1ll << 52) &&
                   cap >= 1 && cap <= n_loc + m_loc,
               "tw_exchange_pack_fixed: bad sizes");
  TW_ARG_CHECK(d_x && d_z && d_cursor && d_send && d_flag, "tw_exchange_pack_fixed: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const Feistel fx = make_feistel(n_loc * (int64_t)G, key_x);
  const Feistel fz = make_feistel(m_loc * (int64_t)G, key_z);
  const int blocks = (int)std::min<int64_t>(exchange_grid(256 * 4), ceil_div(n_loc + m_loc, kScatChunk));
  hipLaunchKernelGGL(k_exchange_pack_fixed, dim3(blocks), dim3(kBlock), 0, st,
                     (const uint64_t*)d_x, n_loc, (const uint64_t*)d_z, m_loc,
                     (int64_t)rank * n_loc, (int64_t)rank * m_loc, (int)G, fx, fz, cap,
                     (unsigned long long*)d_cursor, (uint64_t*)d_send, (int*)d_flag);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_exchange_seal, dim3(1), dim3(kMaxG), 0, st, (int)G, cap,
                     (unsigned long long*)d_cursor, (uint64_t*)d_send, (int*)d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_scatter_buckets(const void* d_recv, int32_t G, int64_t cap, void* d_out,
                                  int64_t n_out, int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxG && cap >= 1 && n_out >= 0 && d_recv && d_out && d_flag,
               "tw_scatter_buckets: bad arguments");
  const int blocks = (int)std::min<int64_t>(exchange_grid(256 * 8), ceil_div((int64_t)G * cap, kBlock));
  hipLaunchKernelGGL(k_scatter_buckets, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_recv, (int)G, cap, (uint64_t*)d_out, n_out, (int*)d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_scatter_records(const void* d_rec, int64_t m, void* d_out, void* stream) {
  TW_ARG_CHECK(m >= 0, "tw_scatter_records: bad size");
  if (m == 0) return TW_OK;
  const int blocks = (int)std::min<int64_t>(exchange_grid(256 * 8), ceil_div(m, kBlock));
  hipLaunchKernelGGL(k_scatter_records, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_rec, m, (uint64_t*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
