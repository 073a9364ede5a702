// chain.hip — the T repartitions of one est.UnNT call as per-element CHAINS of positions, and
// the all-pairs counts of all T steps in ONE launch (round 4).
//
// Reference: est.UnN / UnNT  estimation-experiment/main.py:72-79 (repartition, count, repeat)
//            est.Un          estimation-experiment/main.py:29-31 (the strict predicate)
//
// The step structure of csrc/rankimage.hip (count step i, permute ALL records for step i+1 in
// the same launch) makes every step depend on the previous one through the whole array.  But a
// repartition is a keyed bijection of POSITIONS (csrc/feistel.h), so element e sits at step t
// at position P_t(e) = pi_t(P_{t-1}(e)), P_0(e) = e — a chain that depends on e alone.  And a
// step's count needs each shard's MULTISET of images, not their order.  So for a chunk of
// C <= 32 steps:
//  * k_chain_emit: every element walks its chain once (C forward Feistel evaluations, its
//    image in registers) and, per step, appends its image to the bag of the shard that holds
//    its position — an LDS histogram per block and round of steps, one cursor reservation per
//    (step, shard) and block, runs written coalesced (records.h's staging).  Over several ranks a
//    rank walks only ITS OWN elements and appends {image, local position} records to one
//    fixed-capacity bucket per (destination rank, step); ONE equal-split all-to-all per chunk
//    moves them and k_chain_unpack appends them to the receiver's (step, shard) bags (runs
//    reserved per block: a bag's multiset is what the count needs, not positions).
//  * k_count_chain: the C x N (step, shard) bags counted in one launch (k_count_rank's packed
//    f32 compare-and-count, its work items, XCD order and epilogue), counts [C][N].
//  * at the end of the call the scores in their final order: one scatter by the chains' last
//    positions (one process), or, over ranks, the inverse chain of each of the rank's own
//    final positions (k_chain_inverse) and a gather from the all-gathered sample.
// Work per element and step: one forward Feistel and a 4-B append, by exactly one rank — the
// repartitions no longer cost every rank the whole array.  The count launch has no random
// gathers, so its HBM traffic is the images themselves.  Same permutations (the keyed Feistel
// chain of est.UnNT's loop on the device), same counts, same final arrays as the step path.
//
// Half ties (tie_mode = "half"): an x image is the pair {g(x), h(x)}, h(x) = #{z : z <= x}
// (tw_rank_images_query with half = 1), and ONE clamped packed add gives [x > z] and [x >= z]
// for a z: clamp(h(x) - g(z)) == 1 <=> x >= z.  Half units = the sum of both lanes.
#include "feistel.h"
#include "pkcount.h"
#include "records.h"

namespace tw {

constexpr int kChainMax = 32;            // steps per emission launch (keys in kernel args)
constexpr int kEmThreads = 256;
// tuning hooks (tw_chain_set_emit): elements per thread, steps per round; 0 = automatic
static int g_emit_epr = 0, g_emit_s = 0;
constexpr int kEmMaxB = 2 * kEmThreads;  // staged buckets (block_scan_excl's range)
constexpr int kEmMaxBig = 8192;          // buckets of the unstaged variant (LDS counters)

struct ChainKeys {
  uint64_t kx[kChainMax], kz[kChainMax];
};

struct ChainEmit {
  const uint64_t* xr;  // the emitting rank's X records (low word image; high word h when half)
  const uint64_t* zr;  // its Z records (low word: negated image)
  int64_t nx, nz;      // its element counts (every rank's local sizes)
  uint32_t* xpos;      // chain state: global position of each element at the last step done
  uint32_t* zpos;
  int first;           // no state yet: the position before step 0 is base + e
  int64_t xbase, zbase;
  int64_t NX, NZ;      // global sizes (the permutations' domains)
  int steps, half;
  // every rank's local prop-SWOR layout: shard s = [min(s k, n), min((s+1) k, n)), then the
  // tail that belongs to no shard
  int64_t kx, kz;
  FastDiv dkx, dkz;
  int nsh;
  // one process: bags [steps][nx] (4 B, or 8 B per x when half) and [steps][nz]; cursors
  // [steps][2][nsh + 1], zero on entry
  void* xbag;
  uint32_t* zbag;
  unsigned* cur;
  // the exchange (several ranks, or one rank forced through its collectives): per destination
  // g, steps buckets of 1 + cap records of W words (slot 0: the count), records {image
  // word(s), local position (z: nx + position)}
  int xchg, world, W;
  FastDiv dnx, dnz;
  uint64_t* send;
  int64_t cap;
  int* flag;
  int bx;  // blocks of X tiles; the rest are Z tiles
};

__device__ __forceinline__ int64_t em_region(int b, uint32_t k, int64_t n) {
  const int64_t o = (int64_t)b * k;
  return o < n ? o : n;
}

// next position of every element slot: one forward round set for all, then the cycle walks
// (4.6 % of the slots at n = 1e6 on a 2^20 domain) lane by lane — each lane takes ITS next
// walking slot, so a wave re-evaluates max-over-lanes times instead of once per slot with a
// walker anywhere in the wave (~0.95 of the slots)
template <int EPR>
__device__ __forceinline__ void chain_next(const Feistel& F, uint32_t Ntot, uint32_t (&pos)[EPR],
                                           unsigned valid) {
  unsigned walk = 0;
#pragma unroll
  for (int r = 0; r < EPR; ++r) {
    pos[r] = feistel_once32(F, pos[r]);
    if (((valid >> r) & 1u) && pos[r] >= Ntot) walk |= 1u << r;
  }
  while (__any(walk != 0)) {
    if (walk) {
      const int r = __builtin_ctz(walk);
      uint32_t v = pos[0];
#pragma unroll
      for (int i = 1; i < EPR; ++i) v = i == r ? pos[i] : v;
      v = feistel_once32(F, v);
#pragma unroll
      for (int i = 0; i < EPR; ++i) pos[i] = i == r ? v : pos[i];
      if (v < Ntot) walk &= ~(1u << r);
    }
  }
}

// The emission: each block walks its tile's chains through the chunk's steps, S steps per
// round: the positions of S steps (registers), ONE LDS histogram over the S x NB (step, bucket)
// counters, ONE reservation round of global adds and one staged write pass for all S steps.
// The per-round hand-offs (barriers, the cursor round trip) are a latency every block pays in
// sequence, so small problems (few blocks per CU) take several steps per round; large ones
// one (their blocks are issue-bound, and wider staging only costs occupancy).  A position walk
// kept in memory and placed by a second, fully parallel pass measured slower in both regimes
// (2e6 elements x 20 steps: 308 against 254 us; 250k: 59 against 52 us;
// profiles/r04_prof_parts3_stats.log) — it re-reads the images once per step.
template <int EPR, int S, bool STAGED>
__global__ __launch_bounds__(kEmThreads) void k_chain_emit(ChainEmit em, ChainKeys keys) {
  constexpr int TILE = kEmThreads * EPR;
  constexpr int MB = STAGED ? kEmMaxB : kEmMaxBig;
  __shared__ Feistel fs[kChainMax];
  __shared__ unsigned hist[MB], base[MB], start[STAGED ? kEmMaxB : 1];
  __shared__ unsigned wave_tot[kEmThreads / kWave];
  __shared__ uint64_t sv[STAGED ? TILE * S : 1];
  __shared__ uint32_t sq[STAGED ? TILE * S : 1];
  __shared__ uint16_t sb[STAGED ? TILE * S : 1];
  const bool isx = (int)blockIdx.x < em.bx;
  const int tile = isx ? (int)blockIdx.x : (int)blockIdx.x - em.bx;
  const int64_t n = isx ? em.nx : em.nz;
  const int64_t Ntot = isx ? em.NX : em.NZ;
  if ((int)threadIdx.x < em.steps)
    fs[threadIdx.x] = make_feistel(Ntot > 1 ? Ntot : 1, isx ? keys.kx[threadIdx.x]
                                                           : keys.kz[threadIdx.x]);
  const uint64_t* rec = isx ? em.xr : em.zr;
  uint32_t* posa = isx ? em.xpos : em.zpos;
  const int64_t gbase = isx ? em.xbase : em.zbase;
  const bool wide = isx && em.half;  // 8-B x images {g, h}
  uint64_t val[EPR];
  uint32_t pos[EPR];
  unsigned valid = 0;
  const int64_t e0 = (int64_t)tile * TILE + threadIdx.x;
#pragma unroll
  for (int r = 0; r < EPR; ++r) {
    const int64_t e = e0 + (int64_t)r * kEmThreads;
    val[r] = 0;
    pos[r] = 0;
    if (e < n) {
      valid |= 1u << r;
      const uint64_t v = rec[e];
      val[r] = wide ? v : (v & 0xFFFFFFFFull);
      pos[r] = em.first ? (uint32_t)(gbase + e) : posa[e];
    }
  }
  const int N = em.nsh;
  const int NB = em.xchg ? em.world : N + 1;
  const uint32_t kb = (uint32_t)(isx ? em.kx : em.kz);
  const FastDiv dk = isx ? em.dkx : em.dkz;
  const FastDiv dn = isx ? em.dnx : em.dnz;
  const int cnt = (int)min<int64_t>(TILE, n - (int64_t)tile * TILE);
  for (int i = threadIdx.x; i < S * NB && i < MB; i += kEmThreads) hist[i] = 0;
  __syncthreads();  // fs, hist
  for (int c0 = 0; c0 < em.steps; c0 += S) {
    const int ns = min(S, em.steps - c0);
    int bk[S][EPR];
    uint32_t aux[S][EPR];
    unsigned slot[S][EPR];
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int r = 0; r < EPR; ++r) {
        bk[s][r] = -1;
        aux[s][r] = 0;
        slot[s][r] = 0;
      }
      if (s < ns) {
        chain_next<EPR>(fs[c0 + s], (uint32_t)Ntot, pos, valid);
#pragma unroll
        for (int r = 0; r < EPR; ++r) {
          if ((valid >> r) & 1u) {
            const uint32_t q = pos[r];
            int b;
            if (em.xchg) {
              const uint32_t g = fast_div32(q, dn);
              const uint32_t ql = q - g * (uint32_t)n;
              b = (int)g;
              aux[s][r] = isx ? ql : (uint32_t)em.nx + ql;
            } else {
              b = kb == 0 ? N : (int)min(fast_div32(q, dk), (uint32_t)N);
            }
            bk[s][r] = s * NB + b;
            slot[s][r] = atomicAdd(&hist[s * NB + b], 1u);
          }
        }
      }
    }
    __syncthreads();
    const int nc = ns * NB;
    for (int i = threadIdx.x; i < nc; i += kEmThreads) {
      const int s = i / NB, b = i - s * NB;
      const int c = c0 + s;
      const unsigned h = hist[i];
      unsigned* cu;
      if (em.xchg)
        cu = (unsigned*)(em.send + ((int64_t)b * em.steps + c) * (em.cap + 1) * em.W);
      else
        cu = em.cur + ((int64_t)c * 2 + (isx ? 0 : 1)) * (N + 1) + b;
      base[i] = h ? atomicAdd(cu, h) : 0u;
      if constexpr (STAGED) start[i] = h;
      hist[i] = 0;  // for the next round (its atomics come after the next barrier)
    }
    __syncthreads();
    // one record: counter i = s * NB + b (step c0 + s, bucket b), slot u in the bucket's run
    auto put = [&](int i, unsigned u, uint64_t v, uint32_t a) {
      const int s = i / NB, b = i - s * NB;
      const int c = c0 + s;
      if (em.xchg) {
        if ((int64_t)u >= em.cap) {
          *em.flag = 1;  // dropped, never written out of place; the host raises
          return;
        }
        uint64_t* d = em.send + (((int64_t)b * em.steps + c) * (em.cap + 1) + 1 + u) * em.W;
        if (em.W == 1) {
          d[0] = v | ((uint64_t)a << 32);
        } else {
          d[0] = v;
          d[1] = a;
        }
      } else {
        const int64_t o = (int64_t)c * n + em_region(b, kb, n) + u;
        if (wide)
          ((uint64_t*)em.xbag)[o] = v;
        else
          (isx ? (uint32_t*)em.xbag : em.zbag)[o] = (uint32_t)v;
      }
    };
    if constexpr (STAGED) {
      block_scan_excl<kEmThreads>(start, nc, wave_tot);
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int r = 0; r < EPR; ++r) {
          if (bk[s][r] < 0) continue;
          const unsigned j = start[bk[s][r]] + slot[s][r];
          sv[j] = val[r];
          sq[j] = aux[s][r];
          sb[j] = (uint16_t)bk[s][r];
        }
      }
      __syncthreads();
      for (int j = threadIdx.x; j < cnt * ns; j += kEmThreads) {
        const int i = sb[j];
        put(i, base[i] + (unsigned)j - start[i], sv[j], sq[j]);
      }
      __syncthreads();  // staging and start[] are reused by the next round
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int r = 0; r < EPR; ++r)
          if (bk[s][r] >= 0) put(bk[s][r], base[bk[s][r]] + slot[s][r], val[r], aux[s][r]);
    }
  }
#pragma unroll
  for (int r = 0; r < EPR; ++r) {
    const int64_t e = e0 + (int64_t)r * kEmThreads;
    if (e < n) posa[e] = pos[r];
  }
}

// the count slots of every (destination, step) bucket of a send buffer
__global__ __launch_bounds__(kBlock) void k_chain_zero_heads(uint64_t* __restrict__ send,
                                                             int64_t buckets, int64_t stride) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < buckets;
       i += (int64_t)gridDim.x * kBlock)
    send[i * stride] = 0;
}

// Receiver side: every record of bucket (source g, step c) appended to its (step, side, shard)
// bag region.  The count needs each bag's multiset, not the positions inside it, so a block
// histograms its records over the step's 2 (nsh + 1) regions in LDS, reserves one run per
// (block, region) with one global atomic on the step's cursors, and writes each record into
// its run — whole lines per run, where one scattered 4-B store per record at its position
// (round 4) made every line a partial write: 0.37 ms per 20 steps at G = 2, whose 4-MB step
// bags overflow an XCD's L2.  Region b of a side starts at min(b k, n) (em_region: shard b,
// and b = nsh the tail that belongs to no shard).  Logical blocks are step-major and dealt to
// the XCDs in contiguous ranges (xcd_block), so one step's runs meet in one L2.
constexpr int kUnpackPer = 4;  // records per thread and round
__global__ __launch_bounds__(kBlock) void k_chain_unpack(
    const uint64_t* __restrict__ recv, int world, int steps, int parts, int64_t cap, int W,
    int half, int64_t nx, int64_t nz, int64_t kx, int64_t kz, int nsh, void* __restrict__ xbag,
    uint32_t* __restrict__ zbag, unsigned* __restrict__ cursors, int* __restrict__ flag) {
  extern __shared__ unsigned un_lds[];  // hist[NB], base[NB]
  const int NB = 2 * (nsh + 1);
  unsigned* hist = un_lds;
  unsigned* base = un_lds + NB;
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int c = lb / (world * parts);
  const int rem = lb - c * world * parts;
  const int g = rem / parts, part = rem - g * parts;
  const uint64_t* b = recv + ((int64_t)g * steps + c) * (cap + 1) * W;
  const int64_t cnt0 = (int64_t)(uint32_t)b[0];
  if (cnt0 > cap && part == 0 && threadIdx.x == 0) *flag = 1;
  const int64_t cnt = cnt0 < cap ? cnt0 : cap;
  unsigned* cur = cursors + (int64_t)c * NB;
  for (int j = threadIdx.x; j < NB; j += kBlock) hist[j] = 0;
  __syncthreads();
  constexpr int64_t kRound = (int64_t)kBlock * kUnpackPer;
  for (int64_t i0 = (int64_t)part * kRound; i0 < cnt; i0 += (int64_t)parts * kRound) {
    uint64_t v[kUnpackPer];
    int bk[kUnpackPer];
    unsigned slot[kUnpackPer];
#pragma unroll
    for (int u = 0; u < kUnpackPer; ++u) {
      const int64_t i = i0 + (int64_t)u * kBlock + threadIdx.x;
      bk[u] = -1;
      v[u] = 0;
      slot[u] = 0;
      if (i < cnt) {
        const uint64_t* r = b + (1 + i) * W;
        v[u] = W == 1 ? (r[0] & 0xFFFFFFFFull) : r[0];
        const int64_t p = W == 1 ? (int64_t)(r[0] >> 32) : (int64_t)r[1];
        if (p < nx) {
          bk[u] = kx > 0 ? (int)min<int64_t>(p / kx, nsh) : nsh;
        } else if (p < nx + nz) {
          const int64_t q = p - nx;
          bk[u] = (nsh + 1) + (kz > 0 ? (int)min<int64_t>(q / kz, nsh) : nsh);
        }
        if (bk[u] >= 0) slot[u] = atomicAdd(&hist[bk[u]], 1u);
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < NB; j += kBlock) {
      const unsigned h = hist[j];
      base[j] = h ? atomicAdd(cur + j, h) : 0u;
      hist[j] = 0;  // for the next round (its atomics come after the next barrier)
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kUnpackPer; ++u) {
      if (bk[u] < 0) continue;
      const bool isx = bk[u] <= nsh;
      const int rb = isx ? bk[u] : bk[u] - (nsh + 1);
      const int64_t o = em_region(rb, (uint32_t)(isx ? kx : kz), isx ? nx : nz) + base[bk[u]] +
                        slot[u];
      if (isx) {
        if (half)
          ((uint64_t*)xbag)[(int64_t)c * nx + o] = v[u];
        else
          ((uint32_t*)xbag)[(int64_t)c * nx + o] = (uint32_t)v[u];
      } else {
        zbag[(int64_t)c * nz + o] = (uint32_t)v[u];
      }
    }
    __syncthreads();  // base[] is rewritten by the next round
  }
}

// ----------------------------------------------------------------------------- the count
// One wave item: 64*R x-images (strict: R/2 packed pairs per lane; half: R {g, h} pairs) of
// one (step, shard) bag against z images [z0, z1) of it, z streamed through the scalar cache
// (16 images per s_load_dwordx16, the next group in flight while one is compared).
template <int R, bool HALF>
__device__ __forceinline__ unsigned long long count_chain_item(const void* __restrict__ xb,
                                                               int64_t x0, int64_t xe,
                                                               const float* __restrict__ zf,
                                                               int64_t z0, int64_t z1, int lane) {
  constexpr int P = HALF ? R : R / 2;
  f2 xv[P], acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    if constexpr (HALF) {
      const int64_t i = x0 + p * kWave + lane;
      xv[p] = i < xe ? ((const f2*)xb)[i] : f2{kImgNever, kImgNever};
    } else {
      const int64_t i0 = x0 + (2 * p) * kWave + lane, i1 = i0 + kWave;
      const float* xf = (const float*)xb;
      xv[p].x = i0 < xe ? xf[i0] : kImgNever;  // padded lanes: never greater
      xv[p].y = i1 < xe ? xf[i1] : kImgNever;
    }
    acc[p] = f2{0.f, 0.f};
  }
  // all compares of one z first, then the accumulations
  auto z_lo = [&](uint64_t zu) {
    f2 t[P];
#pragma unroll
    for (int p = 0; p < P; ++p) t[p] = gt_clamp(xv[p], zu);
#pragma unroll
    for (int p = 0; p < P; ++p) acc_add(acc[p], t[p]);
  };
  auto z_hi = [&](uint64_t zu) {
    f2 t[P];
#pragma unroll
    for (int p = 0; p < P; ++p) t[p] = gt_clamp_hi(xv[p], zu);
#pragma unroll
    for (int p = 0; p < P; ++p) acc_add(acc[p], t[p]);
  };
  auto z_pair = [&](uint64_t zu) {
    z_lo(zu);
    z_hi(zu);
  };
  const float* __restrict__ zp = zf + z0;
  const int nz = (int)(z1 - z0);
  int j = 0;
  if (nz > 0 && ((uintptr_t)zp & 7)) {  // an odd first image: alone, then aligned pairs
    z_lo((uint64_t)__float_as_uint(zp[0]));
    j = 1;
  }
  const uint64_t* __restrict__ q = (const uint64_t*)(zp + j);
  const int np = (nz - j) >> 1;
  int i = 0;
  if (np >= 16) {
    uint64_t za[8], zb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) za[u] = q[u];
    const int last = np - 8;
    for (; i + 16 <= np; i += 16) {
      const uint64_t* qb = q + i + 8;
#pragma unroll
      for (int u = 0; u < 8; ++u) zb[u] = qb[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) z_pair(za[u]);
      const uint64_t* qa = q + (i + 16 <= last ? i + 16 : last);
#pragma unroll
      for (int u = 0; u < 8; ++u) za[u] = qa[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) z_pair(zb[u]);
    }
  }
  for (; i + 8 <= np; i += 8) {
    uint64_t zv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) zv[u] = q[i + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) z_pair(zv[u]);
  }
  for (; i < np; ++i) z_pair(q[i]);
  if ((nz - j) & 1) z_lo((uint64_t)__float_as_uint(zp[nz - 1]));
  unsigned long long tot = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) tot += (unsigned)acc[p].x + (unsigned)acc[p].y;  // exact < 2^24
  return wave_sum_u64(tot);
}

// Work items as k_count_rank (csrc/rankimage.hip): per wave (bag v = step * N + shard, x tile,
// z chunk), shard-major logical order dealt to the XCDs in contiguous ranges, one u64 atomic
// per block and bag.
template <int R, bool HALF>
__global__ __launch_bounds__(kBlock) void k_count_chain(
    const void* __restrict__ xb, const int64_t* __restrict__ x_off, int64_t x_stride,
    const float* __restrict__ zb, const int64_t* __restrict__ z_off, int64_t z_stride,
    int n_shards, int n_bags, int tiles_x, int zchunks, int64_t z_chunk,
    unsigned long long* __restrict__ out) {
  const int per_bag = tiles_x * zchunks;
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int item = lb * (kBlock / kWave) + wid;
  const int v = item / per_bag;
  bool active = v < n_bags;
  int64_t x0 = 0, xe = 0, z0 = 0, z1 = 0;
  if (active) {
    const int c = v / n_shards, s = v - c * n_shards;
    const int rem = item - v * per_bag;
    const int cz = rem / tiles_x;
    const int tx = rem - cz * tiles_x;
    const int64_t xo = (int64_t)c * x_stride, zo = (int64_t)c * z_stride;
    const int64_t xbg = xo + x_off[s], zbg = zo + z_off[s], ze = zo + z_off[s + 1];
    xe = xo + x_off[s + 1];
    x0 = xbg + (int64_t)tx * (kWave * R);
    z0 = zbg + (int64_t)cz * z_chunk;
    z1 = (z0 + z_chunk < ze) ? z0 + z_chunk : ze;
    active = x0 < xe && z0 < ze;
  }
  unsigned long long tot = 0;
  if (active) tot = count_chain_item<R, HALF>(xb, x0, xe, zb, z0, z1, lane);
  __shared__ unsigned long long part[kBlock / kWave];
  __shared__ int part_v[kBlock / kWave];
  if (lane == 0) {
    part[wid] = tot;
    part_v[wid] = active ? v : -1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int cur = part_v[0];
    unsigned long long sum = part[0];
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) {
      if (part_v[w] != cur) {
        if (cur >= 0 && sum) atomicAdd(out + cur, sum);
        cur = part_v[w];
        sum = 0;
      }
      sum += part[w];
    }
    if (cur >= 0 && sum) atomicAdd(out + cur, sum);
  }
}

// ------------------------------------------- the call's final arrays over ranks: one exchange
// (round 6) Every rank walked its own elements to their final global positions (the chains'
// state after the call's last emission); each element's score and rank-image record travel
// ONCE to the rank that holds its final position — 24-B records {score, record, local
// position (z: n + position)} in G fixed-capacity buckets (k_exchange_pack_fixed's layout: a
// header record with the count, then up to cap records) through one equal-split all-to-all —
// and land at their positions: the rank's final arrays and the carried records of the next
// call.  This replaces the all-gathers of both samples and of both record arrays (G x the
// rank's bytes received per call) and the inverse-chain gathers from them.
constexpr int kFinMaxG = 1024, kFinPer = 8, kFinChunk = kBlock * kFinPer;

__global__ __launch_bounds__(kBlock) void k_chain_final_pack(
    const uint64_t* __restrict__ xv, const uint64_t* __restrict__ xr,
    const uint32_t* __restrict__ xpos, int64_t n, const uint64_t* __restrict__ zv,
    const uint64_t* __restrict__ zr, const uint32_t* __restrict__ zpos, int64_t m, int G,
    FastDiv dn, FastDiv dm, int64_t cap, unsigned long long* __restrict__ cursor,
    uint64_t* __restrict__ send, int* __restrict__ flag) {
  __shared__ unsigned lcnt[kFinMaxG];
  __shared__ int64_t lbase[kFinMaxG];
  const int64_t tot = n + m, bsz = cap + 1;
  for (int64_t c0 = (int64_t)blockIdx.x * kFinChunk; c0 < tot;
       c0 += (int64_t)gridDim.x * kFinChunk) {
    for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
    __syncthreads();
    int dst[kFinPer];
    unsigned slot[kFinPer];
    int64_t pos[kFinPer];
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
      const int64_t e = c0 + k * kBlock + threadIdx.x;
      dst[k] = -1;
      slot[k] = 0;
      pos[k] = 0;
      if (e < n) {
        const uint64_t p = xpos[e];
        const uint64_t g = fast_div(p, dn);
        dst[k] = (int)g;
        pos[k] = (int64_t)(p - g * (uint64_t)n);
      } else if (e < tot) {
        const uint64_t p = zpos[e - n];
        const uint64_t g = fast_div(p, dm);
        dst[k] = (int)g;
        pos[k] = (int64_t)(p - g * (uint64_t)m) + n;
      }
      if (dst[k] >= G) {  // a position past the sample (never, for a valid chain state)
        *flag = 1;
        dst[k] = -1;
      }
      if (dst[k] >= 0) slot[k] = atomicAdd(&lcnt[dst[k]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += kBlock)
      if (lcnt[i]) lbase[i] = (int64_t)atomicAdd(cursor + i, (unsigned long long)lcnt[i]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
      if (dst[k] >= 0) {
        const int64_t o = lbase[dst[k]] + slot[k];
        if (o < cap) {
          const int64_t e = c0 + k * kBlock + threadIdx.x;
          uint64_t* r = send + 3 * ((int64_t)dst[k] * bsz + 1 + o);
          r[0] = e < n ? xv[e] : zv[e - n];
          r[1] = e < n ? xr[e] : zr[e - n];
          r[2] = (uint64_t)pos[k];
        } else {
          *flag = 1;  // dropped, never written out of place; the host raises
        }
      }
    }
    __syncthreads();
  }
}

// the bucket headers from the cursors (then zeroed for the next call)
__global__ void k_chain_final_seal(int G, int64_t cap, unsigned long long* __restrict__ cursor,
                                   uint64_t* __restrict__ send, int* __restrict__ flag) {
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    const unsigned long long c = cursor[g];
    uint64_t* h = send + 3 * ((int64_t)g * (cap + 1));
    h[0] = c;
    h[1] = 0;
    h[2] = 0;
    cursor[g] = 0;
    if (c > (unsigned long long)cap) *flag = 1;
  }
}

// receive side: every record of every bucket at its position of the final arrays
__global__ __launch_bounds__(kBlock) void k_chain_final_scatter(
    const uint64_t* __restrict__ recv, int G, int64_t cap, int64_t n, int64_t m,
    uint64_t* __restrict__ xo, uint64_t* __restrict__ xro, uint64_t* __restrict__ zo,
    uint64_t* __restrict__ zro, int* __restrict__ flag) {
  const int64_t bsz = cap + 1, tot = (int64_t)G * cap;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t g = i / cap, r = i - g * cap;
    const uint64_t c = recv[3 * (g * bsz)];
    if (c > (uint64_t)cap && r == 0) *flag = 1;
    if ((uint64_t)r < c && r < cap) {
      const uint64_t* q = recv + 3 * (g * bsz + 1 + r);
      const uint64_t p = q[2];
      if (p < (uint64_t)n) {
        xo[p] = q[0];
        xro[p] = q[1];
      } else if (p < (uint64_t)(n + m)) {
        zo[p - n] = q[0];
        zro[p - n] = q[1];
      } else {
        *flag = 1;
      }
    }
  }
}

// ----------------------------------------------------------------------------- final order
// One process: the scores at the chains' last positions, out[pos[e]] = in[e] (8-B values).
__global__ __launch_bounds__(kBlock) void k_chain_scatter(const uint64_t* __restrict__ xin,
                                                          const uint32_t* __restrict__ xpos,
                                                          int64_t nx,
                                                          const uint64_t* __restrict__ zin,
                                                          const uint32_t* __restrict__ zpos,
                                                          int64_t nz, uint64_t* __restrict__ xout,
                                                          uint64_t* __restrict__ zout) {
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < nx + nz;
       e += (int64_t)gridDim.x * kBlock) {
    if (e < nx)
      xout[xpos[e]] = xin[e];
    else
      zout[zpos[e - nx]] = zin[e - nx];
  }
}

// Over ranks: position i of this rank (global base + i) walked back through steps
// [0, steps) of a chunk (last step first): into pout, or, for the call's first chunk, the
// element found there gathered from the all-gathered sample into out.
__global__ __launch_bounds__(kBlock) void k_chain_inverse(
    int64_t xbase, int64_t nx, int64_t NX, int64_t zbase, int64_t nz, int64_t NZ,
    const uint32_t* __restrict__ pin, uint32_t* __restrict__ pout, ChainKeys keys, int steps,
    int gather, const uint64_t* __restrict__ xall, const uint64_t* __restrict__ zall,
    uint64_t* __restrict__ xout, uint64_t* __restrict__ zout,
    const uint64_t* __restrict__ xall2, const uint64_t* __restrict__ zall2,
    uint64_t* __restrict__ xout2, uint64_t* __restrict__ zout2) {
  __shared__ Feistel fs[2 * kChainMax];
  if ((int)threadIdx.x < 2 * steps) {
    const int t = threadIdx.x;
    fs[t] = t < steps ? make_feistel(NX > 1 ? NX : 1, keys.kx[t])
                      : make_feistel(NZ > 1 ? NZ : 1, keys.kz[t - steps]);
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nx + nz;
       i += (int64_t)gridDim.x * kBlock) {
    const bool isx = i < nx;
    const int64_t Nt = isx ? NX : NZ;
    uint32_t p = pin ? pin[i] : (uint32_t)(isx ? xbase + i : zbase + (i - nx));
    for (int c = steps - 1; c >= 0; --c) {
      const Feistel& F = fs[isx ? c : steps + c];
      p = feistel_once_inv32(F, p);
      while (p >= (uint32_t)Nt) p = feistel_once_inv32(F, p);
    }
    if (gather) {  // (a second pair of arrays, e.g. the carried records, from the same walk)
      if (isx) {
        xout[i] = xall[p];
        if (xall2) xout2[i] = xall2[p];
      } else {
        zout[i - nx] = zall[p];
        if (zall2) zout2[i - nx] = zall2[p];
      }
    } else {
      pout[i] = p;
    }
  }
}

// The forward walk alone: position base + e (pin null) or pin[e] through steps [0, steps) of a
// chunk, cycle-walked exactly as chain_next does — the positions the emission of the same keys
// leaves in its chain state, known before any emission has run (the final exchange forks at
// the call's start, beside the emissions and counts).
__global__ __launch_bounds__(kBlock) void k_chain_walk(int64_t xbase, int64_t nx, int64_t NX,
                                                       int64_t zbase, int64_t nz, int64_t NZ,
                                                       int have, uint32_t* __restrict__ xpos,
                                                       uint32_t* __restrict__ zpos,
                                                       ChainKeys keys, int steps) {
  __shared__ Feistel fs[2 * kChainMax];
  if ((int)threadIdx.x < 2 * steps) {
    const int t = threadIdx.x;
    fs[t] = t < steps ? make_feistel(NX > 1 ? NX : 1, keys.kx[t])
                      : make_feistel(NZ > 1 ? NZ : 1, keys.kz[t - steps]);
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nx + nz;
       i += (int64_t)gridDim.x * kBlock) {
    const bool isx = i < nx;
    const int64_t e = isx ? i : i - nx;
    const uint32_t Nt = (uint32_t)(isx ? NX : NZ);
    uint32_t* pa = isx ? xpos : zpos;
    uint32_t p = have ? pa[e] : (uint32_t)((isx ? xbase : zbase) + e);
    for (int c = 0; c < steps; ++c) {
      const Feistel& F = fs[isx ? c : steps + c];
      p = feistel_once32(F, p);
      while (p >= Nt) p = feistel_once32(F, p);
    }
    pa[e] = p;
  }
}

// ----------------------------------------------------------------------------- plan
struct ChainPlan {
  int R, tiles_x, zchunks;
  int64_t z_chunk, blocks;
};
static int g_chain_R = 0;  // tuning hooks (tw_count_chain_set_plan); 0 = automatic
static int64_t g_chain_zchunk = 0;

// strict: R in {16, 8} x-images per lane, least padded slots (ties to 16); half: R = 8 {g, h}
// pairs (the same 8 packed registers per lane).  z chunks: as many as give ~150 work items per
// SIMD (kChainItems), each of >= 600 images — long items amortise a wave's x loads and
// epilogue, enough of them keep the tail short.  Round 5 (tools/count_plan_ab.py, profiles/
// r05s49_count_plan_ab.log, interleaved A/B): against round 4's fixed 1024-image chunks the
// headline K = 20 launch 8.54 -> 8.31 ms, K = 32 13.68 -> 13.34, half ties 17.02 -> 16.54,
// every per-rank shape of the strong problem 0.3-2.4 % faster, C2 within 1 %
constexpr int64_t kChainItems = 256 * 4 * 150;
// (C2's single 1e5 x 1e5 bag: 600-image chunks 276.9 us, 512 282.3 us, profiles/
// r05s59_c2_plan.log; the large shapes are indifferent between 512 and 1024)
constexpr int64_t kChainMinZ = 600;
static ChainPlan plan_chain(int64_t max_nx, int64_t max_nz, int64_t n_bags, bool half) {
  ChainPlan p{half ? 8 : 16, 1, 1, max_nz, 0};
  if (!half) {
    int64_t best = -1;
    for (int R : {16, 8}) {
      if (g_chain_R && R != g_chain_R) continue;
      const int64_t slots = ceil_div(max_nx, (int64_t)kWave * R) * kWave * R;
      if (best < 0 || slots < best) {
        best = slots;
        p.R = R;
      }
    }
  }
  p.tiles_x = (int)ceil_div(max_nx, (int64_t)kWave * p.R);
  const int64_t base = (int64_t)p.tiles_x * n_bags;
  int64_t zc = g_chain_zchunk;
  if (zc <= 0)
    zc = std::max<int64_t>(
        kChainMinZ,
        ceil_div(max_nz, std::max<int64_t>(1, ceil_div(kChainItems, std::max<int64_t>(1, base)))));
  zc = std::min<int64_t>(zc, (int64_t)1 << 24);  // f32 lane counters stay exact
  p.z_chunk = ceil_div(std::min<int64_t>(zc, max_nz), 8) * 8;
  p.zchunks = (int)ceil_div(max_nz, p.z_chunk);
  p.blocks = ceil_div((int64_t)p.tiles_x * p.zchunks * n_bags, kBlock / kWave);
  return p;
}

static ChainKeys chain_keys(const uint64_t* kx, const uint64_t* kz, int steps) {
  ChainKeys k{};
  for (int i = 0; i < steps; ++i) {
    k.kx[i] = kx[i];
    k.kz[i] = kz[i];
  }
  return k;
}

}  // namespace tw

using namespace tw;

extern "C" int tw_chain_emit(const uint64_t* d_x_rec, int64_t n_x, const uint64_t* d_z_rec,
                             int64_t n_z, int32_t half, uint32_t* d_x_pos, uint32_t* d_z_pos,
                             int32_t first, int32_t rank, int32_t world, const uint64_t* keys_x,
                             const uint64_t* keys_z, int32_t steps, int64_t x_shard,
                             int64_t z_shard, int32_t n_shards, void* d_x_bag, void* d_z_bag,
                             uint32_t* d_cursors, uint64_t* d_send, int64_t cap,
                             int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(n_x >= 0 && n_z >= 0 && world >= 1 && rank >= 0 && rank < world &&
                   steps >= 0 && steps <= kChainMax && n_shards >= 0 && x_shard >= 0 &&
                   z_shard >= 0 && (half == 0 || half == 1) && (first == 0 || first == 1),
               "tw_chain_emit: bad sizes");
  TW_ARG_CHECK((int64_t)world * n_x < (1ll << 32) && (int64_t)world * n_z < (1ll << 32),
               "tw_chain_emit: positions must fit 32 bits");
  // the exchange mode is chosen by the send buffer, not by world > 1: a world-size-1 process
  // group can be forced through the collectives' path (ShardedSample(collectives=True))
  const bool xchg = d_send != nullptr;
  TW_ARG_CHECK((xchg ? world : n_shards + 1) <= kEmMaxBig,
               "tw_chain_emit: at most %d buckets (shards + 1, or ranks)", kEmMaxBig);
  TW_ARG_CHECK(steps == 0 || (keys_x != nullptr && keys_z != nullptr),
               "tw_chain_emit: keys missing");
  if (steps == 0 || n_x + n_z == 0) return TW_OK;
  TW_ARG_CHECK(d_x_pos != nullptr && d_z_pos != nullptr, "tw_chain_emit: position state missing");
  if (xchg)
    TW_ARG_CHECK(d_flag != nullptr && cap >= 1 && world <= 1024,
                 "tw_chain_emit: flag and cap >= 1 needed with a send buffer");
  else
    TW_ARG_CHECK(world == 1 && d_x_bag != nullptr && d_z_bag != nullptr && d_cursors != nullptr,
                 "tw_chain_emit: over ranks a send buffer, in one process bags and cursors");
  hipStream_t st = (hipStream_t)stream;
  ChainEmit em{};
  em.xr = d_x_rec;
  em.zr = d_z_rec;
  em.nx = n_x;
  em.nz = n_z;
  em.xpos = d_x_pos;
  em.zpos = d_z_pos;
  em.first = first;
  em.xbase = (int64_t)rank * n_x;
  em.zbase = (int64_t)rank * n_z;
  em.NX = (int64_t)world * n_x;
  em.NZ = (int64_t)world * n_z;
  em.steps = steps;
  em.half = half;
  em.kx = x_shard;
  em.kz = z_shard;
  em.dkx = make_fastdiv(x_shard > 0 ? x_shard : 1);
  em.dkz = make_fastdiv(z_shard > 0 ? z_shard : 1);
  em.nsh = n_shards;
  em.xbag = d_x_bag;
  em.zbag = (uint32_t*)d_z_bag;
  em.cur = d_cursors;
  em.xchg = xchg ? 1 : 0;
  em.world = world;
  em.W = half ? 2 : 1;
  em.dnx = make_fastdiv(n_x > 0 ? n_x : 1);
  em.dnz = make_fastdiv(n_z > 0 ? n_z : 1);
  em.send = d_send;
  em.cap = cap;
  em.flag = d_flag;
  if (xchg) {
    const int64_t buckets = (int64_t)world * steps;
    hipLaunchKernelGGL(k_chain_zero_heads, dim3((unsigned)ceil_div(buckets, kBlock)),
                       dim3(kBlock), 0, st, d_send, buckets, (cap + 1) * em.W);
  } else {
    TW_HIP_CHECK(tw_zero_async(d_cursors, 0,
                               sizeof(unsigned) * (size_t)steps * 2 * (n_shards + 1), st));
  }
  const ChainKeys k = chain_keys(keys_x, keys_z, steps);
  const int NB = xchg ? world : n_shards + 1;
  auto launch = [&](auto epr, auto spr, auto staged) {
    constexpr int EPR = decltype(epr)::value, S = decltype(spr)::value;
    constexpr bool ST = decltype(staged)::value;
    em.bx = (int)ceil_div(n_x, (int64_t)kEmThreads * EPR);
    const int64_t blocks = em.bx + ceil_div(n_z, (int64_t)kEmThreads * EPR);
    hipLaunchKernelGGL((k_chain_emit<EPR, S, ST>), dim3((unsigned)blocks), dim3(kEmThreads), 0,
                       st, em, k);
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  // (profiles/r04_chain_parts.log: 2e6 elements, 20 steps: EPR 8 / 1 step per round 257 us,
  // 8 / 2 296 us; 250k elements: 2 / 8 57 us, 2 / 1 79 us, 8 / 1 139 us)
  const int64_t elems = n_x + n_z;
  // (round 5, profiles/r05s46_emit_sweep_ranks.log: a G = 4 rank's 500k elements, 4 per
  // thread and 4 steps per round: 30 against 36 us at K = 4, 92 against 100 at K = 20)
  const int epr = g_emit_epr ? g_emit_epr : elems >= 1500000 ? 8 : elems >= 400000 ? 4 : 2;
  int spr = g_emit_s ? g_emit_s : epr == 8 ? 1 : 16 / epr;
  while (spr > 1 && spr * NB > kEmMaxB) spr >>= 1;
  if (NB > kEmMaxB) {
    if (epr == 8) launch(I8(), I1(), F_());
    else if (epr == 4) launch(I4(), I1(), F_());
    else launch(I2(), I1(), F_());
  } else if (epr == 8) {
    if (spr >= 2) launch(I8(), I2(), T_());
    else launch(I8(), I1(), T_());
  } else if (epr == 4) {
    if (spr >= 4) launch(I4(), I4(), T_());
    else launch(I4(), I1(), T_());
  } else {
    if (spr >= 8) launch(I2(), I8(), T_());
    else launch(I2(), I1(), T_());
  }
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_chain_set_emit(int32_t epr, int32_t steps_per_round) {
  TW_ARG_CHECK(epr == 0 || epr == 2 || epr == 4 || epr == 8,
               "tw_chain_set_emit: elements per thread 0, 2, 4 or 8");
  TW_ARG_CHECK(steps_per_round == 0 || steps_per_round == 1 || steps_per_round * epr == 16,
               "tw_chain_set_emit: steps per round 0, 1 or 16 / elements per thread");
  g_emit_epr = epr;
  g_emit_s = steps_per_round;
  return TW_OK;
}

extern "C" int tw_chain_unpack(const uint64_t* d_recv, int32_t world, int32_t steps, int64_t cap,
                               int32_t half, int64_t n_x, int64_t n_z, int64_t x_shard,
                               int64_t z_shard, int32_t n_shards, void* d_x_bag, void* d_z_bag,
                               uint32_t* d_cursors, int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(world >= 1 && steps >= 0 && steps <= kChainMax && cap >= 1 && n_x >= 0 &&
                   n_z >= 0 && (half == 0 || half == 1) && (int64_t)world * steps < 65536 &&
                   x_shard >= 0 && z_shard >= 0 && n_shards >= 0 && n_shards < kEmMaxBig,
               "tw_chain_unpack: bad sizes");
  if (steps == 0 || n_x + n_z == 0) return TW_OK;
  TW_ARG_CHECK(d_cursors != nullptr && d_flag != nullptr, "tw_chain_unpack: cursors and flag");
  hipStream_t st = (hipStream_t)stream;
  const int NB = 2 * (n_shards + 1);
  TW_HIP_CHECK(tw_zero_async(d_cursors, 0, sizeof(uint32_t) * (size_t)NB * steps, st));
  const int parts = (int)std::max<int64_t>(
      1, std::min<int64_t>(ceil_div(cap, (int64_t)kBlock * kUnpackPer), 64));
  hipLaunchKernelGGL(k_chain_unpack, dim3((unsigned)(parts * world * steps)), dim3(kBlock),
                     sizeof(unsigned) * 2 * (size_t)NB, st, d_recv, (int)world, (int)steps, parts,
                     cap, half ? 2 : 1, (int)half, n_x, n_z, x_shard, z_shard, (int)n_shards,
                     d_x_bag, (uint32_t*)d_z_bag, (unsigned*)d_cursors, d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// Receiver side at exact positions (the incomplete statistic over ranks, tw_chain_unpack_exact):
// a device-RNG draw addresses a POSITION of the step's permuted arrays, so every record {image,
// local position} lands at bag[c][position] — the step's permuted image arrays themselves, which
// tw_count_pairs_chain_rng reads.  Strict images only (one 8-B record word).
__global__ __launch_bounds__(kBlock) void k_chain_unpack_exact(
    const uint64_t* __restrict__ recv, int world, int steps, int parts, int64_t cap, int64_t nx,
    int64_t nz, uint32_t* __restrict__ xbag, uint32_t* __restrict__ zbag, int* __restrict__ flag) {
  const int lb = xcd_block(blockIdx.x, gridDim.x);
  const int c = lb / (world * parts);
  const int rem = lb - c * world * parts;
  const int g = rem / parts, part = rem - g * parts;
  const uint64_t* b = recv + ((int64_t)g * steps + c) * (cap + 1);
  const int64_t cnt0 = (int64_t)(uint32_t)b[0];
  if (cnt0 > cap && part == 0 && threadIdx.x == 0) *flag = 1;
  const int64_t cnt = cnt0 < cap ? cnt0 : cap;
  for (int64_t i = (int64_t)part * kBlock + threadIdx.x; i < cnt; i += (int64_t)parts * kBlock) {
    const uint64_t r = __builtin_nontemporal_load(b + 1 + i);
    const int64_t p = (int64_t)(r >> 32);
    const uint32_t v = (uint32_t)r;
    if (p < nx)
      xbag[(int64_t)c * nx + p] = v;
    else if (p < nx + nz)
      zbag[(int64_t)c * nz + (p - nx)] = v;
  }
}

extern "C" int tw_chain_unpack_exact(const uint64_t* d_recv, int32_t world, int32_t steps,
                                     int64_t cap, int64_t n_x, int64_t n_z, void* d_x_bag,
                                     void* d_z_bag, int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(world >= 1 && steps >= 0 && steps <= kChainMax && cap >= 1 && n_x >= 0 &&
                   n_z >= 0 && (int64_t)world * steps < 65536 && n_x + n_z < (1ll << 32),
               "tw_chain_unpack_exact: bad sizes");
  if (steps == 0 || n_x + n_z == 0) return TW_OK;
  TW_ARG_CHECK(d_recv && d_x_bag && d_z_bag && d_flag, "tw_chain_unpack_exact: buffers");
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(cap, (int64_t)kBlock * 4), 64));
  hipLaunchKernelGGL(k_chain_unpack_exact, dim3((unsigned)(parts * world * steps)), dim3(kBlock),
                     0, (hipStream_t)stream, d_recv, (int)world, (int)steps, parts, cap, n_x, n_z,
                     (uint32_t*)d_x_bag, (uint32_t*)d_z_bag, d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

// The call's final arrays over ranks by one exchange (k_chain_final_pack / _seal / _scatter):
// tw_chain_final_pack packs this rank's walked elements (scores d_x / d_z, records d_x_rec /
// d_z_rec, final global positions d_x_pos / d_z_pos, each rank n_x / n_z of them) into world
// buckets of 1 + cap 24-B records (d_send: world * (cap + 1) * 3 u64; d_cursor: world u64,
// zero on entry and left zero); after an equal-split all-to-all, tw_chain_final_scatter writes
// every received record into d_x_out / d_x_rec_out / d_z_out / d_z_rec_out at its position.
extern "C" int tw_chain_final_pack(const void* d_x, const uint64_t* d_x_rec,
                                   const uint32_t* d_x_pos, int64_t n_x, const void* d_z,
                                   const uint64_t* d_z_rec, const uint32_t* d_z_pos, int64_t n_z,
                                   int32_t world, int64_t cap, uint64_t* d_cursor, void* d_send,
                                   int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(world >= 1 && world <= kFinMaxG && n_x >= 1 && n_z >= 1 && cap >= 1 &&
                   (int64_t)world * n_x < (1ll << 32) && (int64_t)world * n_z < (1ll << 32),
               "tw_chain_final_pack: bad sizes");
  TW_ARG_CHECK(d_x && d_x_rec && d_x_pos && d_z && d_z_rec && d_z_pos && d_cursor && d_send &&
                   d_flag,
               "tw_chain_final_pack: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)std::min<int64_t>(2048, ceil_div(n_x + n_z, (int64_t)kFinChunk));
  hipLaunchKernelGGL(k_chain_final_pack, dim3(blocks), dim3(kBlock), 0, st,
                     (const uint64_t*)d_x, d_x_rec, d_x_pos, n_x, (const uint64_t*)d_z, d_z_rec,
                     d_z_pos, n_z, (int)world, make_fastdiv((uint64_t)n_x),
                     make_fastdiv((uint64_t)n_z), cap, (unsigned long long*)d_cursor,
                     (uint64_t*)d_send, (int*)d_flag);
  TW_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_chain_final_seal, dim3(1), dim3(256), 0, st, (int)world, cap,
                     (unsigned long long*)d_cursor, (uint64_t*)d_send, (int*)d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_chain_final_scatter(const void* d_recv, int32_t world, int64_t cap,
                                      int64_t n_x, int64_t n_z, void* d_x_out,
                                      void* d_x_rec_out, void* d_z_out, void* d_z_rec_out,
                                      int32_t* d_flag, void* stream) {
  TW_ARG_CHECK(world >= 1 && world <= kFinMaxG && cap >= 1 && n_x >= 0 && n_z >= 0 && d_recv &&
                   d_x_out && d_x_rec_out && d_z_out && d_z_rec_out && d_flag,
               "tw_chain_final_scatter: bad arguments");
  const int blocks = (int)std::max<int64_t>(
      1, std::min<int64_t>(2048, ceil_div((int64_t)world * cap, kBlock)));
  hipLaunchKernelGGL(k_chain_final_scatter, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_recv, (int)world, cap, n_x, n_z, (uint64_t*)d_x_out,
                     (uint64_t*)d_x_rec_out, (uint64_t*)d_z_out, (uint64_t*)d_z_rec_out,
                     (int*)d_flag);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

namespace tw {
// the count launch of tw_count_pairs_chain on an output already zeroed
static int count_chain_launch(const void* d_x_bag, const int64_t* d_x_off, int64_t x_stride,
                              const void* d_z_bag, const int64_t* d_z_off, int64_t z_stride,
                              int32_t n_shards, int32_t steps, int64_t max_nx, int64_t max_nz,
                              int32_t half, uint64_t* d_out, hipStream_t st);
}  // namespace tw

extern "C" int tw_count_pairs_chain(const void* d_x_bag, const int64_t* d_x_off,
                                    int64_t x_stride, const void* d_z_bag,
                                    const int64_t* d_z_off, int64_t z_stride, int32_t n_shards,
                                    int32_t steps, int64_t max_nx, int64_t max_nz, int32_t half,
                                    uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && steps >= 0 && max_nx >= 0 && max_nz >= 0 && x_stride >= 0 &&
                   z_stride >= 0 && (half == 0 || half == 1),
               "tw_count_pairs_chain: bad sizes");
  TW_ARG_CHECK(max_nz < (1ll << 24), "tw_count_pairs_chain: shards of < 2^24 z-images");
  hipStream_t st = (hipStream_t)stream;
  const int64_t bags = (int64_t)n_shards * steps;
  if (bags == 0) return TW_OK;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * (size_t)bags, st));
  return count_chain_launch(d_x_bag, d_x_off, x_stride, d_z_bag, d_z_off, z_stride, n_shards,
                            steps, max_nx, max_nz, half, d_out, st);
}

// Over ranks, a chunk's receive side in ONE call: the unpack's cursors and the counts zeroed by
// one launch, tw_chain_unpack's kernel, tw_count_pairs_chain's count — three launches
// back to back from the host instead of four from two calls (at G = 8 the chunk's device work
// is short and the host's launch gaps showed, profiles/r06s23_rank_call_timeline_G8_K4.log).
// Arguments: tw_chain_unpack's, then the count's shard offsets, largest shards and out
// [steps][n_shards] (bag strides n_x / n_z).
static __global__ __launch_bounds__(256) void k_zero_two(uint32_t* __restrict__ a, int64_t na,
                                                  uint64_t* __restrict__ b, int64_t nb) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < na + nb;
       i += (int64_t)gridDim.x * 256) {
    if (i < na)
      a[i] = 0u;
    else
      b[i - na] = 0ull;
  }
}

extern "C" int tw_chain_unpack_count(const uint64_t* d_recv, int32_t world, int32_t steps,
                                     int64_t cap, int32_t half, int64_t n_x, int64_t n_z,
                                     int64_t x_shard, int64_t z_shard, int32_t n_shards,
                                     void* d_x_bag, void* d_z_bag, uint32_t* d_cursors,
                                     int32_t* d_flag, const int64_t* d_x_off,
                                     const int64_t* d_z_off, int64_t max_nx, int64_t max_nz,
                                     uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(world >= 1 && steps >= 0 && steps <= kChainMax && cap >= 1 && n_x >= 0 &&
                   n_z >= 0 && (half == 0 || half == 1) && (int64_t)world * steps < 65536 &&
                   x_shard >= 0 && z_shard >= 0 && n_shards >= 0 && n_shards < kEmMaxBig &&
                   max_nx >= 0 && max_nz >= 0,
               "tw_chain_unpack_count: bad sizes");
  TW_ARG_CHECK(max_nz < (1ll << 24), "tw_chain_unpack_count: shards of < 2^24 z-images");
  const int64_t bags = (int64_t)n_shards * steps;
  if (bags == 0) return TW_OK;
  TW_ARG_CHECK(d_cursors != nullptr && d_flag != nullptr && d_out != nullptr,
               "tw_chain_unpack_count: cursors, flag and out");
  hipStream_t st = (hipStream_t)stream;
  const int NB = 2 * (n_shards + 1);
  const int64_t nc = (int64_t)NB * steps;
  hipLaunchKernelGGL(k_zero_two, dim3((unsigned)std::min<int64_t>(64, ceil_div(nc + bags, 256))),
                     dim3(256), 0, st, d_cursors, nc, d_out, bags);
  TW_LAUNCH_CHECK();
  if (n_x + n_z == 0) return TW_OK;
  const int parts = (int)std::max<int64_t>(
      1, std::min<int64_t>(ceil_div(cap, (int64_t)kBlock * kUnpackPer), 64));
  hipLaunchKernelGGL(k_chain_unpack, dim3((unsigned)(parts * world * steps)), dim3(kBlock),
                     sizeof(unsigned) * 2 * (size_t)NB, st, d_recv, (int)world, (int)steps, parts,
                     cap, half ? 2 : 1, (int)half, n_x, n_z, x_shard, z_shard, (int)n_shards,
                     d_x_bag, (uint32_t*)d_z_bag, (unsigned*)d_cursors, d_flag);
  TW_LAUNCH_CHECK();
  return count_chain_launch(d_x_bag, d_x_off, n_x, d_z_bag, d_z_off, n_z, n_shards, steps,
                            max_nx, max_nz, half, d_out, st);
}

namespace tw {
static int count_chain_launch(const void* d_x_bag, const int64_t* d_x_off, int64_t x_stride,
                              const void* d_z_bag, const int64_t* d_z_off, int64_t z_stride,
                              int32_t n_shards, int32_t steps, int64_t max_nx, int64_t max_nz,
                              int32_t half, uint64_t* d_out, hipStream_t st) {
  const int64_t bags = (int64_t)n_shards * steps;
  if (max_nx == 0 || max_nz == 0) return TW_OK;
  const ChainPlan p = plan_chain(max_nx, max_nz, bags, half != 0);
  TW_ARG_CHECK(p.blocks * (kBlock / kWave) < (1ll << 31) && bags < (1ll << 31),
               "tw_count_pairs_chain: grid too large");
  dim3 g((unsigned)p.blocks), b(kBlock);
  auto* o = (unsigned long long*)d_out;
  const float* zb = (const float*)d_z_bag;
  if (half)
    hipLaunchKernelGGL((k_count_chain<8, true>), g, b, 0, st, d_x_bag, d_x_off, x_stride, zb,
                       d_z_off, z_stride, n_shards, (int)bags, p.tiles_x, p.zchunks, p.z_chunk,
                       o);
  else if (p.R == 16)
    hipLaunchKernelGGL((k_count_chain<16, false>), g, b, 0, st, d_x_bag, d_x_off, x_stride, zb,
                       d_z_off, z_stride, n_shards, (int)bags, p.tiles_x, p.zchunks, p.z_chunk,
                       o);
  else
    hipLaunchKernelGGL((k_count_chain<8, false>), g, b, 0, st, d_x_bag, d_x_off, x_stride, zb,
                       d_z_off, z_stride, n_shards, (int)bags, p.tiles_x, p.zchunks, p.z_chunk,
                       o);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
}  // namespace tw

// ----------------------------------------------------------------------------- exact count
// The exact O(n + m) count of the bags (algo="sorted", row f4) on the rank images themselves:
// z images are integers g in [0, z_total], so a bag's z, bucketed by g >> shift into <= 16384
// LDS buckets (a counting sort in LDS), answer #{z : g(z) < t} as the z count of the lower
// buckets + a scan of t's own bucket (~1 z).  Per x: t = g(x) ([x > z] <=> g(z) < g(x)); half
// ties add t = h(x) ([x >= z] <=> g(z) < h(x)).  NaN x (image -2^25) count nothing; NaN z
// (g = #non-NaN z) are below no t.  One block per (step, shard) bag, bags of <= 16384 z.
namespace tw {

constexpr int kCbMaxZ = 16384;
constexpr int kCbBuckets = 16384;
constexpr int kCbThreads = 1024;
constexpr int kCbPer = kCbMaxZ / kCbThreads;  // z per thread

template <bool HALF>
__global__ __launch_bounds__(kCbThreads) void k_count_chain_bucket(
    const void* __restrict__ xbag, const int64_t* __restrict__ x_off, int64_t x_stride,
    const float* __restrict__ zbag, const int64_t* __restrict__ z_off, int64_t z_stride,
    int n_shards, int shift, int nbk, unsigned long long* __restrict__ out) {
  __shared__ uint32_t end[kCbBuckets];  // after the scatter: end of bucket b = start of b + 1
  __shared__ uint32_t zs[kCbMaxZ];
  __shared__ uint32_t wtot[kCbThreads / kWave];
  __shared__ unsigned long long bsum[kCbThreads / kWave];
  const int bag = xcd_block(blockIdx.x, gridDim.x);  // a step's shards on one XCD
  const int c = bag / n_shards, s = bag - c * n_shards;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int64_t z0 = z_off[s], x0 = x_off[s];
  const int nz = (int)(z_off[s + 1] - z0);
  const int64_t nx = x_off[s + 1] - x0;
  const float* zp = zbag + (int64_t)c * z_stride + z0;
  uint32_t zv[kCbPer];
#pragma unroll
  for (int u = 0; u < kCbPer; ++u) {  // all loads in flight before the first LDS atomic
    const int i = tid + u * kCbThreads;
    zv[u] = i < nz ? (uint32_t)(-zp[i]) : 0xFFFFFFFFu;  // z bags hold -g(z)
  }
  for (int b = tid; b < nbk; b += kCbThreads) end[b] = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kCbPer; ++u)
    if (zv[u] != 0xFFFFFFFFu) atomicAdd(&end[zv[u] >> shift], 1u);
  __syncthreads();
  // exclusive prefix of the counts: kCbPer consecutive buckets per thread, wave scans, then
  // the wave totals
  {
    const int b0 = tid * kCbPer;
    uint32_t loc[kCbPer], sum = 0;
#pragma unroll
    for (int u = 0; u < kCbPer; ++u) {
      loc[u] = b0 + u < nbk ? end[b0 + u] : 0u;
      sum += loc[u];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += t;
    }
    if (lane == kWave - 1) wtot[wid] = inc;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += wtot[w];
    uint32_t run = wbase + inc - sum;
#pragma unroll
    for (int u = 0; u < kCbPer; ++u) {
      if (b0 + u < nbk) end[b0 + u] = run;  // start of bucket b0 + u
      run += loc[u];
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kCbPer; ++u)  // counting-sort scatter: start -> end of every bucket
    if (zv[u] != 0xFFFFFFFFu) zs[atomicAdd(&end[zv[u] >> shift], 1u)] = zv[u];
  __syncthreads();
  auto below = [&](float tf) -> uint32_t {  // #{z of the bag : g(z) < t}
    if (!(tf > 0.0f)) return 0u;              // t <= 0 (or the NaN-x sentinel): none below
    const uint32_t t = (uint32_t)tf;
    const uint32_t b = t >> shift;            // < nbk: t <= z_total
    uint32_t lo = b ? end[b - 1] : 0u;
    // shift 0: every z of bucket t has image exactly t — none below it, no scan;
    // shift > 0: a bucket spans 2^shift images and is scanned (tie-heavy bags: long buckets)
    if (shift == 0) return lo;
    const uint32_t hi = end[b];
    uint32_t cnt = lo;
    for (; lo < hi; ++lo) cnt += zs[lo] < t ? 1u : 0u;
    return cnt;
  };
  unsigned long long acc = 0;
  if constexpr (HALF) {
    const uint64_t* xp = (const uint64_t*)xbag + (int64_t)c * x_stride + x0;
    for (int64_t i = tid; i < nx; i += kCbThreads) {
      const uint64_t v = xp[i];
      acc += below(__uint_as_float((uint32_t)v)) + below(__uint_as_float((uint32_t)(v >> 32)));
    }
  } else {
    const float* xp = (const float*)xbag + (int64_t)c * x_stride + x0;
    for (int64_t i = tid; i < nx; i += kCbThreads) acc += below(xp[i]);
  }
  acc = wave_sum_u64(acc);
  if (lane == 0) bsum[wid] = acc;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kCbThreads / kWave; ++w) t += bsum[w];
    out[bag] = t;
  }
}

}  // namespace tw

extern "C" int tw_count_pairs_chain_bucket(const void* d_x_bag, const int64_t* d_x_off,
                                           int64_t x_stride, const void* d_z_bag,
                                           const int64_t* d_z_off, int64_t z_stride,
                                           int32_t n_shards, int32_t steps, int64_t max_nz,
                                           int64_t z_total, int32_t half, uint64_t* d_out,
                                           void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && steps >= 0 && x_stride >= 0 && z_stride >= 0 &&
                   (half == 0 || half == 1) && z_total >= 0 && z_total < (1ll << 24),
               "tw_count_pairs_chain_bucket: bad sizes");
  TW_ARG_CHECK(max_nz >= 0 && max_nz <= kCbMaxZ,
               "tw_count_pairs_chain_bucket: bags of <= %d z (use tw_count_pairs_chain)",
               kCbMaxZ);
  const int64_t bags = (int64_t)n_shards * steps;
  TW_ARG_CHECK(bags < (1ll << 31), "tw_count_pairs_chain_bucket: too many bags");
  if (bags == 0) return TW_OK;
  int shift = 0;
  while ((z_total >> shift) >= kCbBuckets) ++shift;
  const int nbk = (int)(z_total >> shift) + 1;
  hipStream_t st = (hipStream_t)stream;
  auto* o = (unsigned long long*)d_out;
  if (half)
    hipLaunchKernelGGL((k_count_chain_bucket<true>), dim3((unsigned)bags), dim3(kCbThreads), 0,
                       st, d_x_bag, d_x_off, x_stride, (const float*)d_z_bag, d_z_off, z_stride,
                       n_shards, shift, nbk, o);
  else
    hipLaunchKernelGGL((k_count_chain_bucket<false>), dim3((unsigned)bags), dim3(kCbThreads), 0,
                       st, d_x_bag, d_x_off, x_stride, (const float*)d_z_bag, d_z_off, z_stride,
                       n_shards, shift, nbk, o);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_count_chain_set_plan(int32_t R, int64_t z_chunk) {
  TW_ARG_CHECK(R == 0 || R == 8 || R == 16, "tw_count_chain_set_plan: R in {0, 8, 16}");
  TW_ARG_CHECK(z_chunk >= 0 && z_chunk <= (1ll << 24), "tw_count_chain_set_plan: bad z_chunk");
  g_chain_R = R;
  g_chain_zchunk = z_chunk;
  return TW_OK;
}

extern "C" int tw_chain_scatter(const void* d_x, const uint32_t* d_x_pos, int64_t n_x,
                                const void* d_z, const uint32_t* d_z_pos, int64_t n_z,
                                void* d_x_out, void* d_z_out, void* stream) {
  TW_ARG_CHECK(n_x >= 0 && n_z >= 0, "tw_chain_scatter: bad sizes");
  TW_ARG_CHECK((n_x == 0 || d_x != d_x_out) && (n_z == 0 || d_z != d_z_out),
               "tw_chain_scatter: in and out must differ");
  if (n_x + n_z == 0) return TW_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(n_x + n_z, kBlock));
  hipLaunchKernelGGL(k_chain_scatter, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_x, d_x_pos, n_x, (const uint64_t*)d_z, d_z_pos, n_z,
                     (uint64_t*)d_x_out, (uint64_t*)d_z_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

static int chain_gather_impl(const void* d_x_all, const void* d_z_all, int64_t x_base,
                             int64_t n_x, int64_t n_x_all, int64_t z_base, int64_t n_z,
                             int64_t n_z_all, const uint64_t* keys_x, const uint64_t* keys_z,
                             int32_t steps, uint32_t* d_work, void* d_x_out, void* d_z_out,
                             const void* d_x_all2, const void* d_z_all2, void* d_x_out2,
                             void* d_z_out2, void* stream);

extern "C" int tw_chain_gather(const void* d_x_all, const void* d_z_all, int64_t x_base,
                               int64_t n_x, int64_t n_x_all, int64_t z_base, int64_t n_z,
                               int64_t n_z_all, const uint64_t* keys_x, const uint64_t* keys_z,
                               int32_t steps, uint32_t* d_work, void* d_x_out, void* d_z_out,
                               void* stream) {
  return chain_gather_impl(d_x_all, d_z_all, x_base, n_x, n_x_all, z_base, n_z, n_z_all, keys_x,
                           keys_z, steps, d_work, d_x_out, d_z_out, nullptr, nullptr, nullptr,
                           nullptr, stream);
}

// tw_chain_gather of two pairs of arrays laid out alike (the scores and the carried records)
// through ONE walk of the inverse chains
extern "C" int tw_chain_gather2(const void* d_x_all, const void* d_z_all, const void* d_x_all2,
                                const void* d_z_all2, int64_t x_base, int64_t n_x,
                                int64_t n_x_all, int64_t z_base, int64_t n_z, int64_t n_z_all,
                                const uint64_t* keys_x, const uint64_t* keys_z, int32_t steps,
                                uint32_t* d_work, void* d_x_out, void* d_z_out, void* d_x_out2,
                                void* d_z_out2, void* stream) {
  TW_ARG_CHECK(d_x_all2 && d_z_all2 && d_x_out2 && d_z_out2,
               "tw_chain_gather2: the second pair of arrays");
  return chain_gather_impl(d_x_all, d_z_all, x_base, n_x, n_x_all, z_base, n_z, n_z_all, keys_x,
                           keys_z, steps, d_work, d_x_out, d_z_out, d_x_all2, d_z_all2, d_x_out2,
                           d_z_out2, stream);
}

// Final global positions of this rank's elements (x: x_base + e, z: z_base + e) after steps
// chained permutations of the n_x_all / n_z_all domains (keys_x / keys_z): what tw_chain_emit's
// chain state holds after the same steps, computed without emitting.
extern "C" int tw_chain_walk(int64_t x_base, int64_t n_x, int64_t n_x_all, int64_t z_base,
                             int64_t n_z, int64_t n_z_all, const uint64_t* keys_x,
                             const uint64_t* keys_z, int32_t steps, uint32_t* d_x_pos,
                             uint32_t* d_z_pos, void* stream) {
  TW_ARG_CHECK(n_x >= 0 && n_z >= 0 && x_base >= 0 && z_base >= 0 && steps >= 0 &&
                   x_base + n_x <= n_x_all && z_base + n_z <= n_z_all &&
                   n_x_all < (1ll << 32) && n_z_all < (1ll << 32),
               "tw_chain_walk: bad sizes");
  TW_ARG_CHECK(steps == 0 || (keys_x != nullptr && keys_z != nullptr),
               "tw_chain_walk: keys missing");
  TW_ARG_CHECK((n_x == 0 || d_x_pos != nullptr) && (n_z == 0 || d_z_pos != nullptr),
               "tw_chain_walk: null position arrays");
  if (n_x + n_z == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(n_x + n_z, kBlock));
  int lo = 0;
  do {  // chunks of <= 32 steps; a zero-step walk still writes the base positions
    const int hi = std::min<int>(steps, lo + kChainMax);
    const ChainKeys k = hi > lo ? chain_keys(keys_x + lo, keys_z + lo, hi - lo) : ChainKeys{};
    hipLaunchKernelGGL(k_chain_walk, dim3(grid), dim3(kBlock), 0, st, x_base, n_x, n_x_all,
                       z_base, n_z, n_z_all, lo > 0 ? 1 : 0, d_x_pos, d_z_pos, k, hi - lo);
    TW_LAUNCH_CHECK();
    lo = hi;
  } while (lo < steps);
  return TW_OK;
}

static int chain_gather_impl(const void* d_x_all, const void* d_z_all, int64_t x_base,
                             int64_t n_x, int64_t n_x_all, int64_t z_base, int64_t n_z,
                             int64_t n_z_all, const uint64_t* keys_x, const uint64_t* keys_z,
                             int32_t steps, uint32_t* d_work, void* d_x_out, void* d_z_out,
                             const void* d_x_all2, const void* d_z_all2, void* d_x_out2,
                             void* d_z_out2, void* stream) {
  TW_ARG_CHECK(n_x >= 0 && n_z >= 0 && x_base >= 0 && z_base >= 0 && steps >= 0 &&
                   x_base + n_x <= n_x_all && z_base + n_z <= n_z_all &&
                   n_x_all < (1ll << 32) && n_z_all < (1ll << 32),
               "tw_chain_gather: bad sizes");
  TW_ARG_CHECK(steps == 0 || (keys_x != nullptr && keys_z != nullptr),
               "tw_chain_gather: keys missing");
  TW_ARG_CHECK(steps <= kChainMax || d_work != nullptr,
               "tw_chain_gather: more than 32 steps need a (n_x + n_z) u32 work array");
  if (n_x + n_z == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(n_x + n_z, kBlock));
  // chunks of <= 32 steps from the last: positions walked back into d_work, the first chunk
  // (steps [0, 32)) gathers
  int hi = steps;
  bool have = false;
  do {
    const int lo = std::max(0, hi - kChainMax);
    const ChainKeys k = hi > lo ? chain_keys(keys_x + lo, keys_z + lo, hi - lo) : ChainKeys{};
    hipLaunchKernelGGL(k_chain_inverse, dim3(grid), dim3(kBlock), 0, st, x_base, n_x, n_x_all,
                       z_base, n_z, n_z_all, have ? d_work : nullptr, d_work, k, hi - lo,
                       lo == 0 ? 1 : 0, (const uint64_t*)d_x_all, (const uint64_t*)d_z_all,
                       (uint64_t*)d_x_out, (uint64_t*)d_z_out, (const uint64_t*)d_x_all2,
                       (const uint64_t*)d_z_all2, (uint64_t*)d_x_out2, (uint64_t*)d_z_out2);
    TW_LAUNCH_CHECK();
    have = true;
    hi = lo;
  } while (hi > 0);
  return TW_OK;
}
