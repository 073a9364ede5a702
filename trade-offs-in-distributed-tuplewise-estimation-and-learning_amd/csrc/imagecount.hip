// imagecount.hip — incomplete counts on float32 images of the scores held in LDS (rows A5/A8:
// cs.UB / UnNB / UnNBT, compute_stats.py:37-42, :104-123, in replay and device-RNG mode).
//
// The explicit-index (replay) and device-drawn pairs of a shard compare x[i] > z[j] at random
// positions.  A 15625 + 15625-value shard pair is 250 KB of doubles, too much for a CU's
// 160 KB of LDS, but its float32 images are 125 KB: one block per CU stages its shard's images
// once and every pair then reads two LDS words instead of two random L2 lines.  The compare is
// exact:
//   f(v) = (float)v rounds to nearest, a monotone non-decreasing map (for doubles and for int64),
//   so f(x) > f(z) implies x > z and f(x) < f(z) implies x < z;
//   only f(x) == f(z) is undecided — ties, -0 vs +0, values within half a float ulp of each
//   other, both beyond the float range, subnormals — and those pairs are decided on the scores
//   themselves (two gathers), only in the waves where they occur;
//   NaN images are NaN: every compare is false and they are never "equal", so a pair with a NaN
//   counts nothing, as in NumPy.
// Half-ties (TW_PRED_HALF) add x >= z: f(x) > f(z) gives 2, f(x) < f(z) gives 0.
// No precomputed rank codes (the codes kernel of the 16-bit path cost 28 us of a 130 us replay
// call at the bench shape), no workspace.  Scores with many exact ties between the samples
// (small integers) take the gather for every tied pair: correct, slower.
#include "imagecount.h"
#include "nextstep.h"
#include <algorithm>

namespace tw {

constexpr int kImgThreads = 1024;

// the shard's images into LDS: eight loads in flight per thread, then the conversions
template <typename T>
__device__ __forceinline__ void stage_images(float* __restrict__ dst, const T* __restrict__ src,
                                             int64_t n) {
  constexpr int U = 8;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)U * kImgThreads) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * kImgThreads;
      v[u] = i < n ? src[i] : (T)0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * kImgThreads;
      if (i < n) dst[i] = (float)v[u];
    }
  }
}

__device__ __forceinline__ int64_t al4(int64_t n) { return (n + 3) & ~(int64_t)3; }

// pair outcome from the images: r = the count to add when decided, und = undecided (equal
// images: the scores decide)
template <int PRED>
__device__ __forceinline__ unsigned image_cmp(float xf, float zf, bool& und) {
  und = xf == zf;
  return (xf > zf) ? (PRED == TW_PRED_HALF ? 2u : 1u) : 0u;
}

template <typename T, int PRED>
__device__ __forceinline__ unsigned exact_cmp(T xv, T zv) {
  return (unsigned)(xv > zv) + (PRED == TW_PRED_HALF ? (unsigned)(xv >= zv) : 0u);
}

template <typename I> struct ImgVec;
typedef int32_t img_i32x4 __attribute__((ext_vector_type(4)));
typedef int64_t img_i64x2 __attribute__((ext_vector_type(2)));
template <> struct ImgVec<int32_t> {
  using V = int4;
  using NVec = img_i32x4;  // the same 16 bytes as a clang vector (nontemporal builtin operand)
  static constexpr int N = 4;
  __device__ static __forceinline__ int32_t at(const V& v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
  }
};
template <> struct ImgVec<int64_t> {
  using V = longlong2;
  using NVec = img_i64x2;
  static constexpr int N = 2;
  __device__ static __forceinline__ int64_t at(const V& v, int e) { return e == 0 ? v.x : v.y; }
};

// Replay: explicit absolute index pairs (as tw_count_pairs_idx); an index outside its shard's
// span compares the scores.  Index streams as 16-B vectors (VEC: aligned base pointers), U per
// stream and batch, two register buffers used in turn (batch k+1 in flight while batch k is
// compared; the first batch is issued before the images are staged).  Loads are unconditional
// (clamped to the last vector) so the compiler's wait counts stay exact.
template <typename T, int PRED, typename I, bool VEC, int U, bool NT>
__global__ __launch_bounds__(kImgThreads) void k_count_idx_img(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, const I* __restrict__ ix, const I* __restrict__ iz,
    const int64_t* __restrict__ pair_off, int parts, unsigned long long* __restrict__ out) {
  using IV = ImgVec<I>;
  using V = typename IV::V;
  constexpr int NV = VEC ? IV::N : 1;
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // a shard's parts share one L2
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int tid = threadIdx.x;
  const int64_t xb = x_off[s], zb = z_off[s];
  const int64_t nx = x_off[s + 1] - xb, nz = z_off[s + 1] - zb;
  float* lx = img;
  float* lz = img + al4(nx);
  const int64_t pb = pair_off[s], pe = pair_off[s + 1];
  const int64_t per = (pe - pb + parts - 1) / parts;
  const int64_t q0 = std::min<int64_t>(pe, pb + (int64_t)part * per);
  const int64_t q1 = std::min<int64_t>(pe, q0 + per);
  const int64_t a0 = std::min<int64_t>(q1, (q0 + NV - 1) / NV * NV);
  const int64_t a1 = std::max<int64_t>(a0, q1 / NV * NV);
  const int nv = (int)((a1 - a0) / NV);
  auto local = [&](I a, I b, uint32_t& i, uint32_t& j) -> bool {
    if constexpr (sizeof(I) == 4) {  // 32-bit offsets: the arrays hold < 2^31 elements
      i = (uint32_t)(a - (int32_t)xb);
      j = (uint32_t)(b - (int32_t)zb);
      return i < (uint32_t)nx && j < (uint32_t)nz;
    } else {
      const uint64_t i64 = (uint64_t)(a - xb), j64 = (uint64_t)(b - zb);
      i = (uint32_t)i64;
      j = (uint32_t)j64;
      return i64 < (uint64_t)nx && j64 < (uint64_t)nz;
    }
  };
  auto one = [&](I a, I b) -> unsigned {  // scalar heads / tails
    uint32_t i, j;
    bool und = true;
    unsigned r = 0;
    if (local(a, b, i, j)) r = image_cmp<PRED>(lx[i], lz[j], und);
    return und ? exact_cmp<T, PRED>(x[a], z[b]) : r;
  };
  const I* __restrict__ px = ix + a0;
  const I* __restrict__ pzi = iz + a0;
  auto load = [&](const I* p, int v) -> V {
    if constexpr (VEC && NT) {  // streamed once: nontemporal
      return __builtin_bit_cast(
          V, __builtin_nontemporal_load(((const typename IV::NVec*)p) + v));
    } else if constexpr (VEC) {
      return ((const V*)p)[v];
    } else {
      V r;
      r.x = p[v];
      return r;
    }
  };
  // a batch without branches; pairs whose images tie or that leave the shard's span are
  // counted from the scores, in the waves that have one
  auto compare = [&](const V (&A)[U], const V (&Bv)[U], int base) -> unsigned {
    unsigned c = 0;
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = base + tid + u * kImgThreads < nv;
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        uint32_t i, j;
        const bool in = local(IV::at(A[u], e), IV::at(Bv[u], e), i, j) && live;
        bool und;
        const unsigned r = image_cmp<PRED>(lx[in ? i : 0u], lz[in ? j : 0u], und);
        bad |= live && (!in || und);
        c += (in && !und) ? r : 0u;
      }
    }
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool live = base + tid + u * kImgThreads < nv;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          uint32_t i, j;
          const I a = IV::at(A[u], e), b = IV::at(Bv[u], e);
          bool und = true;
          if (live && local(a, b, i, j)) image_cmp<PRED>(lx[i], lz[j], und);
          if (live && und) c += exact_cmp<T, PRED>(x[a], z[b]);
        }
      }
    }
    return c;
  };
  auto load_batch = [&](V (&A)[U], V (&Bv)[U], int base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = min(base + tid + u * kImgThreads, nv - 1);
      A[u] = load(px, v);
      Bv[u] = load(pzi, v);
    }
  };
  constexpr int step = U * kImgThreads;
  const int nb = (nv + step - 1) / step;
  V A[U], Bv[U], A2[U], B2[U];
  if (nb > 0) load_batch(A, Bv, 0);  // in flight while the images are staged
  stage_images<T>(lx, x + xb, nx);
  stage_images<T>(lz, z + zb, nz);
  __syncthreads();
  unsigned acc = 0;
  if (tid < a0 - q0) acc += one(ix[q0 + tid], iz[q0 + tid]);
  if (tid < q1 - a1) acc += one(ix[a1 + tid], iz[a1 + tid]);
  for (int k = 0; k < nb; k += 2) {
    load_batch(A2, B2, (k + 1) * step);
    acc += compare(A, Bv, k * step);
    load_batch(A, Bv, (k + 2) * step);
    acc += compare(A2, B2, (k + 1) * step);
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kImgThreads / kWave];
  const int lane = tid & (kWave - 1), wid = tid / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (tid == 0) {
    unsigned long long sum = 0;
    for (int w = 0; w < kImgThreads / kWave; ++w) sum += part_sum[w];
    if (sum) atomicAdd(out + s, sum);
  }
}

// Attribution builds of the device-RNG count's inner loop (make
// ab-rngimg, tools/ab_rng_img.py): 0 = the product; 1 = Philox + Lemire only (no LDS, no
// compare); 2 = + the two LDS image reads and the compare (no equal-image fallback); 3 = 2 with
// the LDS reads at conflict-free addresses (lane-consecutive: what the random gathers' bank
// conflicts cost); 4 = the product with the Lemire maps' four per-draw rejection branches
// (tw_common.h lemire_index) in place of lemire4's one wave-uniform test.  Measured (round 5,
// profiles/r05s8_rng_img_attribution.json): product 0.0848 ms per 64 x 1e6 pairs, 1: 0.0752,
// 2: 0.0781, 3: 0.0797, 4: 0.1010 — the round-4 gap was the per-draw branches.
#ifndef TW_RNG_IMG_VARIANT
#define TW_RNG_IMG_VARIANT 0
#endif

// The four Lemire maps of one Philox block (pairs 2q and 2q+1) with ONE wave-uniform test for
// the biased zone (probability n / 2^32 per draw, ~4e-6 at C3): the common case is four
// multiplies; any lane in the zone sends the whole wave through lemire_index's rejection
// loop, which returns the same index for every lane not in the zone — the same draws, bit for
// bit, without four divergent branches (and their exec-mask bookkeeping) per block.
__device__ __forceinline__ void lemire4(const u32x4& r, uint32_t nx, uint32_t nz, uint64_t q,
                                        uint32_t ss, uint32_t k0, uint32_t k1, uint32_t& i0,
                                        uint32_t& j0, uint32_t& i1, uint32_t& j1) {
  const uint64_t m0 = (uint64_t)r.a * nx, m1 = (uint64_t)r.b * nz;
  const uint64_t m2 = (uint64_t)r.c * nx, m3 = (uint64_t)r.d * nz;
  const bool zone = ((uint32_t)m0 < nx) | ((uint32_t)m1 < nz) | ((uint32_t)m2 < nx) |
                    ((uint32_t)m3 < nz);
  if (__builtin_expect(__ballot(zone) != 0, 0)) {
    i0 = lemire_index(r.a, nx, q, ss, 0, k0, k1);
    j0 = lemire_index(r.b, nz, q, ss, 1, k0, k1);
    i1 = lemire_index(r.c, nx, q, ss, 2, k0, k1);
    j1 = lemire_index(r.d, nz, q, ss, 3, k0, k1);
  } else {
    i0 = (uint32_t)(m0 >> 32);
    j0 = (uint32_t)(m1 >> 32);
    i1 = (uint32_t)(m2 >> 32);
    j1 = (uint32_t)(m3 >> 32);
  }
}

// Device RNG: the draws of tw_count_pairs_rng (Philox block q -> pairs 2q and 2q+1, Lemire
// maps; csrc/count.hip k_count_rng) compared on the images.
template <typename T, int PRED, int QU>
__global__ __launch_bounds__(kImgThreads) void k_count_rng_img(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, int64_t B, int parts, uint32_t k0, uint32_t k1,
    uint32_t sid, unsigned long long* __restrict__ out, NextStep nxt) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int s = lb / parts;
  const int part = lb - s * parts;
  const int64_t xb = x_off[s], zb = z_off[s];
  const int64_t nx = x_off[s + 1] - xb, nz = z_off[s + 1] - zb;
  // the next repartition riding in the count threads (tw_count_pairs_rng_step): a block's
  // LDS holds its shard's images, so no spare block of the same launch could share a CU with
  // it; each thread carries ~8 of the next permutation's gathers, one issued every `every`
  // iterations of its Philox loop, so the random reads' latency hides behind the draws
  NextSlice<kImgThreads> ns(nxt);
  next_step_zero<kImgThreads>(nxt);
  if (ns.kmax > 0) ns.issue();  // in flight while the images are staged
  unsigned acc = 0;
  if (nx > 0 && nz > 0) {
    float* lx = img;
    float* lz = img + al4(nx);
    stage_images<T>(lx, x + xb, nx);
    stage_images<T>(lz, z + zb, nz);
    __syncthreads();
    const uint32_t ss = (uint32_t)s + sid;
    const int64_t nq = (B + 1) / 2;
    const int64_t per = (nq + parts - 1) / parts;
    const int64_t q0 = (int64_t)part * per, q1 = std::min<int64_t>(nq, q0 + per);
    // next-step gathers: one every `every` iterations (block-uniform)
    const int64_t nit = (q1 - q0 + (int64_t)QU * kImgThreads - 1) / ((int64_t)QU * kImgThreads);
    const int every = ns.kmax > 1 ? (int)std::max<int64_t>(1, nit / ns.kmax) : 0;
    int it = 0;
    // trip count uniform over the block (q1 - q0 is), so the ballot below is wave-uniform.
    // QU Philox blocks per thread and iteration, computed unconditionally (a dead lane's draw
    // is discarded): independent chains the scheduler interleaves (16 waves per CU only).
    for (int64_t qb = q0; qb < q1; qb += (int64_t)QU * kImgThreads) {
      if (every && ++it == every) {
        it = 0;
        if (ns.k < ns.kmax) ns.issue();
      }
      u32x4 r[QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int64_t q = qb + (int64_t)u * kImgThreads + threadIdx.x;
        r[u] = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), ss, 0u}, k0, k1);
      }
      // the iteration's undecided pairs (equal images), settled on the scores after ONE
      // wave-uniform test for all QU blocks (one ballot per iteration, not per block)
      uint32_t ui[QU][2], uj[QU][2];
      bool ud[QU][2];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int64_t q = qb + (int64_t)u * kImgThreads + threadIdx.x;
        const bool live = q < q1;
        const bool two = live && 2 * q + 1 < B;
        uint32_t i0 = 0, j0 = 0, i1 = 0, j1 = 0;
#if TW_RNG_IMG_VARIANT == 4
        if (live) {
          i0 = lemire_index(r[u].a, (uint32_t)nx, q, ss, 0, k0, k1);
          j0 = lemire_index(r[u].b, (uint32_t)nz, q, ss, 1, k0, k1);
          if (two) {
            i1 = lemire_index(r[u].c, (uint32_t)nx, q, ss, 2, k0, k1);
            j1 = lemire_index(r[u].d, (uint32_t)nz, q, ss, 3, k0, k1);
          }
        }
#else
        // a dead lane's indices are in range too (its reads are discarded)
        lemire4(r[u], (uint32_t)nx, (uint32_t)nz, q, ss, k0, k1, i0, j0, i1, j1);
#endif
#if TW_RNG_IMG_VARIANT == 1
        acc += (live ? ((i0 ^ j0) & 1u) : 0u) + (two ? ((i1 ^ j1) & 1u) : 0u);
#elif TW_RNG_IMG_VARIANT == 2 || TW_RNG_IMG_VARIANT == 3
#if TW_RNG_IMG_VARIANT == 3
        // (shards of >= 4096 values: the bench shape; the images at lane-consecutive slots,
        // the draws kept live by the added low bits — two extra VALU per pair)
        const uint32_t a0 = (threadIdx.x + 64u * u) & 4095u, b0 = a0;
        const uint32_t a1 = (threadIdx.x + 64u * u + 32u) & 4095u, b1 = a1;
        (void)j0;
        (void)j1;
        bool u0, u1;
        const unsigned r0 = image_cmp<PRED>(lx[a0] + (float)((i0 ^ j0) & 1u), lz[b0], u0);
        const unsigned r1 = image_cmp<PRED>(lx[a1] + (float)((i1 ^ j1) & 1u), lz[b1], u1);
#else
        bool u0, u1;
        const unsigned r0 = image_cmp<PRED>(lx[i0], lz[j0], u0);
        const unsigned r1 = image_cmp<PRED>(lx[i1], lz[j1], u1);
#endif
        (void)u0;
        (void)u1;
        acc += (live ? r0 : 0u) + (two ? r1 : 0u);
#else
        bool u0, u1;
        const unsigned r0 = image_cmp<PRED>(lx[i0], lz[j0], u0);
        const unsigned r1 = image_cmp<PRED>(lx[i1], lz[j1], u1);
        u0 = u0 && live;
        u1 = u1 && two;
        acc += (live && !u0 ? r0 : 0u) + (two && !u1 ? r1 : 0u);
        ui[u][0] = i0;
        uj[u][0] = j0;
        ui[u][1] = i1;
        uj[u][1] = j1;
        ud[u][0] = u0;
        ud[u][1] = u1;
#endif
      }
#if TW_RNG_IMG_VARIANT == 0 || TW_RNG_IMG_VARIANT == 4
      bool any = false;
#pragma unroll
      for (int u = 0; u < QU; ++u) any = any || ud[u][0] || ud[u][1];
      if (__builtin_expect(__ballot(any) != 0, 0)) {
#pragma unroll
        for (int u = 0; u < QU; ++u)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            if (ud[u][h]) acc += exact_cmp<T, PRED>(x[xb + ui[u][h]], z[zb + uj[u][h]]);
      }
#else
      (void)ui;
      (void)uj;
      (void)ud;
#endif
    }
  }
  ns.finish();
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kImgThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < kImgThreads / kWave; ++w) b += part_sum[w];
    if (b) atomicAdd(out + s, b);
  }
}

// Device RNG on the step chains' bags (tw_count_pairs_chain_rng; cs.UnNBT over ranks,
// compute_stats.py:119-123): the chunk's (step, shard) bags hold, at the exact positions of the
// step's permuted arrays, integer rank images — x: g(x) = #{z : z < x}, z: -g(z) (csrc/pkcount.h)
// — so x > z <=> g(x) + (-g(z)) >= 1 decides every pair, ties included, with no score gathers.
// The draws are k_count_rng_img's (Philox block q -> pairs 2q and 2q+1 of shard `sid + s`, key
// seed + c for step c, lemire4): the same pair indices, hence the same integers as the score
// path's count of the same permuted arrays.  Grid: steps x shards x parts blocks, logical
// order step-major (one step's bags meet in one XCD's L2).
template <int QU>
__global__ __launch_bounds__(kImgThreads) void k_count_rng_chain(
    const float* __restrict__ xbag, const int64_t* __restrict__ x_off, int64_t x_stride,
    const float* __restrict__ zbag, const int64_t* __restrict__ z_off, int64_t z_stride,
    int n_shards, int64_t B, int parts, uint64_t seed, uint32_t sid,
    unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int v = lb / parts;
  const int part = lb - v * parts;
  const int c = v / n_shards, s = v - c * n_shards;
  const int64_t xb = x_off[s], zb = z_off[s];
  const int64_t nx = x_off[s + 1] - xb, nz = z_off[s + 1] - zb;
  unsigned acc = 0;
  if (nx > 0 && nz > 0) {
    float* lx = img;
    float* lz = img + al4(nx);
    stage_images<float>(lx, xbag + (int64_t)c * x_stride + xb, nx);
    stage_images<float>(lz, zbag + (int64_t)c * z_stride + zb, nz);
    __syncthreads();
    const uint64_t sd = seed + (uint64_t)c;
    const uint32_t k0 = (uint32_t)sd, k1 = (uint32_t)(sd >> 32);
    const uint32_t ss = (uint32_t)s + sid;
    const int64_t nq = (B + 1) / 2;
    const int64_t per = (nq + parts - 1) / parts;
    const int64_t q0 = (int64_t)part * per, q1 = std::min<int64_t>(nq, q0 + per);
    for (int64_t qb = q0; qb < q1; qb += (int64_t)QU * kImgThreads) {
      u32x4 r[QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int64_t q = qb + (int64_t)u * kImgThreads + threadIdx.x;
        r[u] = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), ss, 0u}, k0, k1);
      }
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int64_t q = qb + (int64_t)u * kImgThreads + threadIdx.x;
        const bool live = q < q1;
        const bool two = live && 2 * q + 1 < B;
        uint32_t i0, j0, i1, j1;
        lemire4(r[u], (uint32_t)nx, (uint32_t)nz, q, ss, k0, k1, i0, j0, i1, j1);
        acc += (live && lx[i0] + lz[j0] >= 1.0f ? 1u : 0u) +
               (two && lx[i1] + lz[j1] >= 1.0f ? 1u : 0u);
      }
    }
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part_sum[kImgThreads / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part_sum[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < kImgThreads / kWave; ++w) b += part_sum[w];
    if (b) atomicAdd(out + v, b);
  }
}

static int g_img_parts = 0;  // tuning: blocks per shard (0 = plan)
static int g_img_u = 1;      // tuning: index vectors per stream and batch (1, 2, 4)
static int g_img_nt = 1;     // tuning: nontemporal index loads (default on: streamed once)

ImgPlan plan_images(int32_t n_shards, int64_t max_nx, int64_t max_nz, int32_t pred,
                    int64_t pairs) {
  ImgPlan p{};
  p.lds = (size_t)(al4h(max_nx) + max_nz) * sizeof(float);
  p.ok = n_shards > 0 && max_nx > 0 && max_nz > 0 &&
         (pred == TW_PRED_GT || pred == TW_PRED_HALF) && p.lds <= 160 * 1024 - 1024;
  // one 1024-thread block per CU (up to 125 KB of images each): ~256 blocks over the grid,
  // at least 16384 pairs per block
  p.parts = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(256, n_shards),
                                                        ceil_div(std::max<int64_t>(pairs, 1),
                                                                 16384)));
  if (g_img_parts > 0) p.parts = g_img_parts;
  p.ok = p.ok && (int64_t)n_shards * p.parts < (1ll << 31);
  return p;
}

template <typename T, int PRED, typename I, bool VEC, int U, bool NT>
static int launch_idx_img_v(const void* x, const int64_t* x_off, const void* z,
                            const int64_t* z_off, int32_t n_shards, const I* ix, const I* iz,
                            const int64_t* pair_off, const ImgPlan& p, uint64_t* out,
                            hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_count_idx_img<T, PRED, I, VEC, U, NT>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - 1024));
    attr = true;
  }
  hipLaunchKernelGGL((k_count_idx_img<T, PRED, I, VEC, U, NT>), dim3(n_shards * p.parts),
                     dim3(kImgThreads), p.lds, st, (const T*)x, x_off, (const T*)z, z_off, ix, iz,
                     pair_off, p.parts, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T, int PRED, typename I>
static int launch_idx_img_t(const void* x, const int64_t* x_off, const void* z,
                            const int64_t* z_off, int32_t n_shards, const I* ix, const I* iz,
                            const int64_t* pair_off, const ImgPlan& p, uint64_t* out,
                            hipStream_t st) {
  if ((((uintptr_t)ix | (uintptr_t)iz) & 15) != 0)
    return launch_idx_img_v<T, PRED, I, false, 4, false>(x, x_off, z, z_off, n_shards, ix, iz,
                                                         pair_off, p, out, st);
#define TW_IMG(U, NT) return launch_idx_img_v<T, PRED, I, true, U, NT>(x, x_off, z, z_off, n_shards, ix, iz, pair_off, p, out, st)
  if (g_img_nt) {
    if (g_img_u == 2) TW_IMG(2, true);
    if (g_img_u == 4) TW_IMG(4, true);
    TW_IMG(1, true);
  }
  if (g_img_u == 2) TW_IMG(2, false);
  if (g_img_u == 4) TW_IMG(4, false);
  TW_IMG(1, false);
#undef TW_IMG
}

template <typename I>
int launch_idx_images(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, const I* ix, const I* iz, const int64_t* pair_off,
                      int32_t dtype, int32_t pred, const ImgPlan& p, uint64_t* out,
                      hipStream_t st) {
  if (dtype == TW_F64) {
    if (pred == TW_PRED_HALF)
      return launch_idx_img_t<double, TW_PRED_HALF, I>(x, x_off, z, z_off, n_shards, ix, iz, pair_off, p, out, st);
    return launch_idx_img_t<double, TW_PRED_GT, I>(x, x_off, z, z_off, n_shards, ix, iz, pair_off, p, out, st);
  }
  if (pred == TW_PRED_HALF)
    return launch_idx_img_t<long long, TW_PRED_HALF, I>(x, x_off, z, z_off, n_shards, ix, iz, pair_off, p, out, st);
  return launch_idx_img_t<long long, TW_PRED_GT, I>(x, x_off, z, z_off, n_shards, ix, iz, pair_off, p, out, st);
}
template int launch_idx_images<int32_t>(const void*, const int64_t*, const void*, const int64_t*,
                                        int32_t, const int32_t*, const int32_t*, const int64_t*,
                                        int32_t, int32_t, const ImgPlan&, uint64_t*, hipStream_t);
template int launch_idx_images<int64_t>(const void*, const int64_t*, const void*, const int64_t*,
                                        int32_t, const int64_t*, const int64_t*, const int64_t*,
                                        int32_t, int32_t, const ImgPlan&, uint64_t*, hipStream_t);

template <typename T, int PRED, int QU>
static int launch_rng_img_q(const void* x, const int64_t* x_off, const void* z,
                            const int64_t* z_off, int32_t n_shards, int64_t B, uint64_t seed,
                            uint64_t sid, const ImgPlan& p, uint64_t* out, const NextStep& nxt,
                            hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_count_rng_img<T, PRED, QU>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - 1024));
    attr = true;
  }
  hipLaunchKernelGGL((k_count_rng_img<T, PRED, QU>), dim3(n_shards * p.parts),
                     dim3(kImgThreads), p.lds, st, (const T*)x, x_off, (const T*)z, z_off, B,
                     p.parts, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)sid,
                     (unsigned long long*)out, nxt);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

static int g_img_rng_qu = 2;  // tuning: Philox blocks per thread and iteration (1, 2, 4)

template <typename T, int PRED>
static int launch_rng_img_t(const void* x, const int64_t* x_off, const void* z,
                            const int64_t* z_off, int32_t n_shards, int64_t B, uint64_t seed,
                            uint64_t sid, const ImgPlan& p, uint64_t* out, const NextStep& nxt,
                            hipStream_t st) {
  if (g_img_rng_qu == 4)
    return launch_rng_img_q<T, PRED, 4>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
  if (g_img_rng_qu == 2)
    return launch_rng_img_q<T, PRED, 2>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
  return launch_rng_img_q<T, PRED, 1>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
}

int launch_rng_images(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, int64_t B, uint64_t seed, uint64_t sid, int32_t dtype,
                      int32_t pred, const ImgPlan& p, uint64_t* out, const NextStep& nxt,
                      hipStream_t st) {
  if (dtype == TW_F64) {
    if (pred == TW_PRED_HALF)
      return launch_rng_img_t<double, TW_PRED_HALF>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
    return launch_rng_img_t<double, TW_PRED_GT>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
  }
  if (pred == TW_PRED_HALF)
    return launch_rng_img_t<long long, TW_PRED_HALF>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
  return launch_rng_img_t<long long, TW_PRED_GT>(x, x_off, z, z_off, n_shards, B, seed, sid, p, out, nxt, st);
}

}  // namespace tw

extern "C" int tw_count_pairs_chain_rng(const float* d_x_bag, const int64_t* d_x_off,
                                        int64_t x_stride, const float* d_z_bag,
                                        const int64_t* d_z_off, int64_t z_stride,
                                        int32_t n_shards, int32_t steps, int64_t max_nx,
                                        int64_t max_nz, int64_t B, uint64_t seed,
                                        uint64_t stream_id, uint64_t* d_out, void* stream) {
  using namespace tw;
  TW_ARG_CHECK(n_shards >= 0 && steps >= 0 && B >= 0 && max_nx >= 0 && max_nz >= 0 &&
                   x_stride >= 0 && z_stride >= 0,
               "tw_count_pairs_chain_rng: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nbags = (int64_t)n_shards * steps;
  if (nbags == 0) return TW_OK;
  TW_ARG_CHECK(d_out != nullptr, "tw_count_pairs_chain_rng: out");
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * (size_t)nbags, st));
  if (B == 0 || max_nx == 0 || max_nz == 0) return TW_OK;
  TW_ARG_CHECK(d_x_bag && d_z_bag && d_x_off && d_z_off, "tw_count_pairs_chain_rng: buffers");
  // the plan spreads the chunk's (step, shard) bags over the CUs: with 8 shards a rank (G = 8)
  // and 4 steps, 8 blocks a bag rather than one step's 32 — every block stages its bag's
  // 125 KB of images once, so a grid of steps x (256 / shards) blocks staged each bag 4x over
  ImgPlan p = plan_images((int32_t)std::min<int64_t>(nbags, 1 << 30), max_nx, max_nz,
                          TW_PRED_GT, (B + 1) / 2);
  TW_ARG_CHECK(p.ok, "tw_count_pairs_chain_rng: a shard's images exceed the LDS (%lld + %lld)",
               (long long)max_nx, (long long)max_nz);
  // blocks per bag: one 1024-thread block per CU holds a bag's images, so the grid runs in
  // waves of ~256 blocks; pick the split that minimises waves x (a block's draws + its staging,
  // ~5k draws' worth) — 160 bags (G = 8, T = 20): 8 blocks a bag (5 full waves) rather than 2
  // (a second wave of 64 blocks as long as the first)
  {
    const int64_t nq = (B + 1) / 2;
    double best = -1.0;
    for (int parts = 1; parts <= 64; ++parts) {
      if (parts > 1 && nq / parts < 4096) break;
      const double waves = (double)ceil_div(nbags * parts, 256);
      const double cost = waves * ((double)ceil_div(nq, parts) + 2500.0);
      if (best < 0 || cost < best) {
        best = cost;
        p.parts = parts;
      }
    }
  }
  TW_ARG_CHECK(nbags * p.parts < (1ll << 31), "tw_count_pairs_chain_rng: grid too large");
  static bool attr = false;
  if (!attr) {
    TW_HIP_CHECK(hipFuncSetAttribute((const void*)k_count_rng_chain<2>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - 1024));
    attr = true;
  }
  hipLaunchKernelGGL(k_count_rng_chain<2>, dim3((unsigned)(nbags * p.parts)), dim3(kImgThreads),
                     p.lds, st, d_x_bag, d_x_off, x_stride, d_z_bag, d_z_off, z_stride,
                     (int)n_shards, B, p.parts, seed, (uint32_t)stream_id,
                     (unsigned long long*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_count_rng_img_set_unroll(int32_t qu) {
  TW_ARG_CHECK(qu == 1 || qu == 2 || qu == 4, "tw_count_rng_img_set_unroll: 1, 2 or 4");
  tw::g_img_rng_qu = qu;
  return TW_OK;
}

extern "C" int tw_count_img_set_plan(int32_t parts, int32_t u) {
  // u: 1, 2 or 4 index vectors per stream and batch; + 8: nontemporal index loads
  TW_ARG_CHECK(parts >= 0 && parts <= 4096 && ((u & 7) == 1 || (u & 7) == 2 || (u & 7) == 4) &&
                   u < 16,
               "tw_count_img_set_plan: parts 0..4096, u in {1, 2, 4} (+ 8: nontemporal)");
  tw::g_img_parts = parts;
  tw::g_img_u = u & 7;
  tw::g_img_nt = u >> 3;
  return TW_OK;
}
