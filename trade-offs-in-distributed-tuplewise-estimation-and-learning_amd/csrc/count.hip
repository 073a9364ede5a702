// count.hip — exact two-sample pair counting on gfx950.
//
// Reference semantics
//   est.Un      estimation-experiment/main.py:29-31   mean(X[:,None] > Z[None,:])
//   cs.Un AUC   learning-experiment/compute_stats.py:19   mean((X_col - Z_row > 0).astype(int))
//   cs.UB_indices / UB_pairs / UB   compute_stats.py:22-42 (AUC branch at :30)
// Every block value of those functions is count / #pairs, count an exact integer; the kernels
// below produce that integer (uint64 per shard) and the host divides exactly as NumPy does.
//
// Complete kernel (k_count_complete) — VALU-bound, one launch for all shards:
//   * each wave owns a tile of 64*R x-values of one shard (R per lane, in VGPRs) and a chunk
//     of that shard's z-values (a block = 4 consecutive wave items, normally one z chunk);
//   * z is wave-uniform: it streams through the SCALAR cache (s_load_dwordx16 = 8 doubles)
//     straight into SGPR operands of v_cmp_*_f64 — no LDS staging and no VGPR traffic for z;
//   * per pair: one v_cmp (VCC) + one carry-add into a per-(lane, r) u32 counter
//     (the compiler folds two compares into v_cndmask + v_addc); u32 cannot overflow because a
//     counter sees at most 2 * z_chunk increments;
//   * epilogue: valid counters -> u64 -> wave butterfly (DPP) -> block sum per shard (LDS) ->
//     one u64 atomic per block and shard.
//   Measured on MI355X (tools/mb_issue*.hip): v_cmp_*_f64 and v_addc issue at ~0.94
//   wave-instructions/cycle/CU, so 2 such instructions per pair cap this kernel at ~1.9e13
//   pairs/s; see DESIGN.md "count kernel roofline".
#include "feistel.h"
#include "nextstep.h"
#include <algorithm>
#include <type_traits>

namespace tw {

template <typename T, int PRED>
__device__ __forceinline__ unsigned pair_pred(T x, T z) {
  if constexpr (PRED == TW_PRED_GT) {
    return x > z;
  } else if constexpr (PRED == TW_PRED_HALF) {
    return (unsigned)(x > z) + (unsigned)(x >= z);
  } else {  // TW_PRED_SUBGT: literal (x - z) > 0 of cs.Un; int64 wraps like NumPy
    if constexpr (std::is_integral<T>::value) {
      return (long long)((unsigned long long)x - (unsigned long long)z) > 0;
    } else {
      return x > z;  // identical to (x - z) > 0 for IEEE doubles (no FTZ on f64)
    }
  }
}

// Wave count of one compare on the scalar unit: v_cmp to an SGPR pair, s_bcnt1; half-ties
// count the two one-bit masks x > z and x >= z.
template <typename T, int PRED>
__device__ __forceinline__ unsigned scalar_count(T x, T z) {
  if constexpr (PRED == TW_PRED_HALF)
    return (unsigned)__builtin_popcountll(__ballot(x > z)) +
           (unsigned)__builtin_popcountll(__ballot(x >= z));
  else
    return (unsigned)__builtin_popcountll(__ballot(pair_pred<T, PRED>(x, z)));
}

// One wave item: its 64*R x-values (from x0, valid below xe) against z[z0, z1).  Returns the
// wave's count (wave-uniform).
template <typename T, int R, int NS, int PRED>
__device__ __forceinline__ unsigned long long count_item(const T* __restrict__ x, int64_t x0,
                                                         int64_t xe, const T* __restrict__ z,
                                                         int64_t z0, int64_t z1, int lane) {
  static_assert(NS == 0 || std::is_floating_point<T>::value,
                "scalar-unit counting needs NaN padding");
  T xv[R];
  unsigned acc[R];
  bool valid[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = x0 + r * kWave + lane;
    valid[r] = i < xe;
    if constexpr (NS > 0)
      xv[r] = valid[r] ? x[i] : (T)__builtin_nan("");
    else
      xv[r] = valid[r] ? x[i] : (T)0;
    acc[r] = 0;
  }

  const T* __restrict__ zp = z + z0;
  const int nz = (int)(z1 - z0);
  // wave-uniform scalar-unit counts, one per scalar-counted x-value: independent s_add chains
  // let the scheduler spread the SALU work between the compares (one shared accumulator made
  // a 16-long dependent chain at the loop end and cost ~10%)
#ifndef TW_NS_EXTRA
#define TW_NS_EXTRA 0
#endif
  // NSE: x-values counted on the scalar unit for odd z of a group (NS for even z), so the
  // scalar share can sit between NS/R and (NS+1)/R
  constexpr int NSE = (NS > 0 && NS + TW_NS_EXTRA <= R) ? NS + TW_NS_EXTRA : NS;
  unsigned sacc[NSE > 0 ? NSE : 1];
#pragma unroll
  for (int r = 0; r < (NSE > 0 ? NSE : 1); ++r) sacc[r] = 0;
  if constexpr (NS == 0) {
#pragma unroll 8
    for (int j = 0; j < nz; ++j) {
      const T zv = zp[j];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] += pair_pred<T, PRED>(xv[r], zv);
    }
  } else {
    // one z against the R x-values of every lane, NSZ of them counted on the scalar unit
    auto one_z = [&](const T zu, auto nsz) {
      constexpr int NSZ = decltype(nsz)::value;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < NSZ) {
          sacc[r] += scalar_count<T, PRED>(xv[r], zu);
        } else {
          acc[r] += pair_pred<T, PRED>(xv[r], zu);
        }
      }
#ifndef TW_COUNT_NO_SCHED
        // interleave per z: groups of (VALU, SALU) so each wave's instruction stream alternates
        // compare and scalar-count work instead of clustering the SALU at the loop end
        // (+9%, profiles/r01_count_variants.log "nosched"; carrying the masks one z forward or
        // putting the SALU group first measured within noise, 5 of 8 x-values on the scalar
        // unit likewise).  TW_SCHED_G / TW_NS8 / TW_NS4 are build-time tuning hooks
        // (tools/build_count_variants.sh).
#ifndef TW_SCHED_G
#define TW_SCHED_G NS
#endif
        constexpr int kG = TW_SCHED_G;  // groups per z
        constexpr int kM = PRED == TW_PRED_HALF ? 2 : 1;  // compares per pair
        constexpr int kV = (kM * (2 * R - NSZ) + kG - 1) / kG, kS = (2 * kM * NSZ + kG - 1) / kG;
#pragma unroll
        for (int k = 0; k < kG; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x002, kV, 0);
          __builtin_amdgcn_sched_group_barrier(0x004, kS, 0);
        }
#endif
    };
    // 8 z (one s_load_dwordx16)
    auto group8 = [&](const T (&zv)[8]) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        one_z(zv[u], std::integral_constant<int, NS>{});
        one_z(zv[u + 1], std::integral_constant<int, NSE>{});
      }
    };
    int j = 0;
#ifndef TW_COUNT_NO_ZPIPE
    // z loads one group ahead, two register buffers (no per-group copies on the SALU): the
    // scalar loads of group g+1 are in flight while group g is compared.  Loads past the
    // chunk are clamped to its last full group (in bounds, unused).
    if (nz >= 16) {
      T za[8], zb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) za[u] = zp[u];
      const int last = nz - 8;
      for (; j + 16 <= nz; j += 16) {
        const T* qb = zp + j + 8;
#pragma unroll
        for (int u = 0; u < 8; ++u) zb[u] = qb[u];
        group8(za);
        const T* qa = zp + (j + 16 <= last ? j + 16 : last);
#pragma unroll
        for (int u = 0; u < 8; ++u) za[u] = qa[u];
        group8(zb);
      }
    }
#endif
    for (; j + 8 <= nz; j += 8) {
      T zv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) zv[u] = zp[j + u];
      group8(zv);
    }
    for (; j < nz; ++j) {
      const T zv = zp[j];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r < NS)
          sacc[r] += scalar_count<T, PRED>(xv[r], zv);
        else
          acc[r] += pair_pred<T, PRED>(xv[r], zv);
      }
    }
  }

  unsigned long long tot = 0;
#pragma unroll
  for (int r = NS; r < R; ++r) tot += valid[r] ? (unsigned long long)acc[r] : 0ull;
  tot = wave_sum_u64(tot);
  unsigned long long stot = 0;
#pragma unroll
  for (int r = 0; r < NSE; ++r) stot += sacc[r];
  return tot + stot;
}

// Mixed VALU/SALU accumulation (double, strict predicate).  Per pair the compare is one
// v_cmp_*_f64; accumulating its 64 result bits costs one more VALU op (carry-add into a per-lane
// counter) — the VALU issue ceiling of §4.1 — or, if the compare writes an SGPR pair, two
// SCALAR ops (s_bcnt1_i32_b64 + s_add) on the scalar unit, which issues beside the VALU.
// Counting NS of the R x-values per lane on the scalar unit moves that share of the work off
// the VALU (tools/mb_mix.hip, profiles/r01_microbench_salu_mix.log: R=4 with NS=2 reaches
// 0.63 of the lane-op peak against 0.49 for VALU-only accumulation).  Padded lanes hold NaN,
// for which every predicate is false, so the scalar counts need no lane mask.
template <typename T, int R, int NS, int PRED>
__global__ __launch_bounds__(kBlock) void k_count_complete(
    const T* __restrict__ x, const int64_t* __restrict__ x_off, const T* __restrict__ z,
    const int64_t* __restrict__ z_off, int n_shards, int tiles_x, int zchunks, int64_t z_chunk,
    unsigned long long* __restrict__ out, NextStep nxt) {
  // Spare blocks (block-uniform branch), in groups of kXcds so count blocks keep their XCD:
  // group g occupies blocks [g*every, g*every + kXcds) — every == kXcds: the leading blocks,
  // every > kXcds: spread through the grid — or, with tail != 0, the last nxt.blocks blocks.
  int cb = blockIdx.x;  // index among the count blocks
  if (nxt.blocks) {
    const int b = blockIdx.x, ng = nxt.blocks / kXcds;
    if (nxt.tail) {
      if (b >= (int)gridDim.x - nxt.blocks) {
        next_step_part<kBlock>(nxt, b - ((int)gridDim.x - nxt.blocks));
        return;
      }
    } else {
      const int g = b / nxt.every, r = b - g * nxt.every;
      if (r < kXcds && g < ng) {
        next_step_part<kBlock>(nxt, g * kXcds + r);
        return;
      }
      cb = b - kXcds * ((g < ng ? g : ng) + ((r >= kXcds && g < ng) ? 1 : 0));
    }
  }
  // Work items are per WAVE: (shard, x wave-tile of 64*R values, z chunk), x tile fastest, so
  // a shard pads its x-values to a multiple of 64*R (not 256*R) and a block's 4 waves share
  // one z chunk (scalar-cache hits) on consecutive x tiles.
  const int per_shard = tiles_x * zchunks;
  const int lb = xcd_block(cb, gridDim.x - nxt.blocks);  // whole shards per XCD
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int item = lb * (kBlock / kWave) + wid;
  const int s = item / per_shard;
  bool active = s < n_shards;  // wave-uniform (no early return: the block reduces below)
  int64_t x0 = 0, xe = 0, z0 = 0, z1 = 0;
  if (active) {
    const int rem = item - s * per_shard;
    const int cz = rem / tiles_x;
    const int tx = rem - cz * tiles_x;
    const int64_t xb = x_off[s], zb = z_off[s], ze = z_off[s + 1];
    xe = x_off[s + 1];
    x0 = xb + (int64_t)tx * (kWave * R);
    z0 = zb + (int64_t)cz * z_chunk;
    z1 = (z0 + z_chunk < ze) ? z0 + z_chunk : ze;
    active = x0 < xe && z0 < ze;  // ragged shard smaller than the grid
  }

  unsigned long long tot = 0;
  if (active) tot = count_item<T, R, NS, PRED>(x, x0, xe, z, z0, z1, lane);
  // Block reduction: the 4 waves of a block normally count the same shard, and one atomic per
  // block and shard keeps same-address atomics rare (a single-shard launch with one atomic
  // per wave serialised on them: tools/tune_c2.py).
  __shared__ unsigned long long part[kBlock / kWave];
  __shared__ int part_s[kBlock / kWave];
  if (lane == 0) {
    part[wid] = tot;
    part_s[wid] = active ? s : -1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int cur = part_s[0];
    unsigned long long sum = part[0];
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) {
      if (part_s[w] != cur) {
        if (cur >= 0 && sum) atomicAdd(out + cur, sum);
        cur = part_s[w];
        sum = 0;
      }
      sum += part[w];
    }
    if (cur >= 0 && sum) atomicAdd(out + cur, sum);
  }
}

// Incomplete count on explicit index pairs (replay of NumPy's randint draws).
// I: int64_t (NumPy's randint dtype) or int32_t (narrowed by the host after its bound check).
template <typename T, int PRED, int PPT, typename I>
__global__ __launch_bounds__(kBlock) void k_count_idx(const T* __restrict__ x,
                                                      const T* __restrict__ z,
                                                      const I* __restrict__ ix,
                                                      const I* __restrict__ iz,
                                                      const int64_t* __restrict__ pair_off,
                                                      int blocks_per_shard,
                                                      unsigned long long* __restrict__ out) {
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // whole shards per XCD
  const int s = lb / blocks_per_shard;
  const int bi = lb - s * blocks_per_shard;
  const int64_t pb = pair_off[s], pe = pair_off[s + 1];
  const int64_t p0 = pb + (int64_t)bi * (kBlock * PPT);
  if (p0 >= pe) return;
  unsigned acc = 0;
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int64_t p = p0 + k * kBlock + threadIdx.x;
    if (p < pe) acc += pair_pred<T, PRED>(x[ix[p]], z[iz[p]]);
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = part[0] + part[1] + part[2] + part[3];
    if (b) atomicAdd(out + s, b);
  }
}

// Incomplete count with pairs drawn on the device (with replacement, like UB's randint).
// One Philox4x32-10 block (counter (q lo, q hi, shard, 0)) gives the 4 words of TWO pairs,
// 2q (words a, b) and 2q+1 (words c, d): word -> index by Lemire's multiply-shift with
// rejection, exactly uniform on [0, n).  A rejected word (probability < n / 2^32) is replaced by
// the same word of the block at counter word 3 = 1, 2, ...  The Philox multiplies
// (v_mad_u64_u32) dominate the kernel, so two pairs per block halves its cost.  Shards of 2^32
// or more values use the 64-bit multiply-high of two words instead (one pair per block).
template <typename T, int PRED, int PPT>
__global__ __launch_bounds__(kBlock) void k_count_rng(const T* __restrict__ x,
                                                      const int64_t* __restrict__ x_off,
                                                      const T* __restrict__ z,
                                                      const int64_t* __restrict__ z_off,
                                                      int64_t B, int blocks_per_shard,
                                                      uint32_t k0, uint32_t k1, uint32_t sid,
                                                      unsigned long long* __restrict__ out) {
  const int lb = xcd_block(blockIdx.x, gridDim.x);  // whole shards per XCD
  const int s = lb / blocks_per_shard;
  const int bi = lb - s * blocks_per_shard;
  const int64_t xb = x_off[s], nx = x_off[s + 1] - xb;
  const int64_t zb = z_off[s], nz = z_off[s + 1] - zb;
  const uint32_t ss = (uint32_t)s + sid;
  unsigned acc = 0;
  if (nx > 0 && nz > 0) {
    if (((nx | nz) >> 32) == 0) {
      const int64_t nq = (B + 1) / 2;  // Philox blocks of this shard
      const int64_t q0 = (int64_t)bi * (kBlock * (PPT / 2));
      if (q0 < nq) {
#pragma unroll
        for (int k = 0; k < PPT / 2; ++k) {
          const int64_t q = q0 + k * kBlock + threadIdx.x;
          if (q < nq) {
            const u32x4 r = philox4x32_10(u32x4{(uint32_t)q, (uint32_t)(q >> 32), ss, 0u}, k0, k1);
            const uint32_t i0 = lemire_index(r.a, (uint32_t)nx, q, ss, 0, k0, k1);
            const uint32_t j0 = lemire_index(r.b, (uint32_t)nz, q, ss, 1, k0, k1);
            acc += pair_pred<T, PRED>(x[xb + i0], z[zb + j0]);
            if (2 * q + 1 < B) {
              const uint32_t i1 = lemire_index(r.c, (uint32_t)nx, q, ss, 2, k0, k1);
              const uint32_t j1 = lemire_index(r.d, (uint32_t)nz, q, ss, 3, k0, k1);
              acc += pair_pred<T, PRED>(x[xb + i1], z[zb + j1]);
            }
          }
        }
      }
    } else {  // huge shards: one pair per block, 64-bit multiply-high
      for (int64_t p = (int64_t)bi * (kBlock * PPT) + threadIdx.x,
                   pe = std::min<int64_t>(B, (int64_t)(bi + 1) * (kBlock * PPT));
           p < pe; p += kBlock) {
        const u32x4 r = philox4x32_10(u32x4{(uint32_t)p, (uint32_t)(p >> 32), ss, 0u}, k0, k1);
        const uint64_t i = mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)nx);
        const uint64_t j = mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)nz);
        acc += pair_pred<T, PRED>(x[xb + i], z[zb + j]);
      }
    }
  }
  unsigned long long tot = wave_sum_u64((unsigned long long)acc);
  __shared__ unsigned long long part[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) part[wid] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = part[0] + part[1] + part[2] + part[3];
    if (b) atomicAdd(out + s, b);
  }
}

// ---------------------------------------------------------------- launch plans
struct CompletePlan {
  int R, tiles_x, zchunks;
  int64_t z_chunk;
  int64_t blocks;
};

// R in {1,2,4,8}: least padded x-slots per shard, larger R on ties (fewer z loads per
// compare); then split z into chunks until the grid has >= 16 blocks per CU.
static int g_force_R = 0;            // tuning hook (tw_count_set_plan); 0 = automatic
static int64_t g_force_zchunk = 0;

static int g_scalar_mix = 1;  // tw_count_set_scalar_mix: 0 = VALU-only accumulation

// Measured pair rates (fraction of the lane-op peak on the bench shape: tools/tune_count.py,
// profiles/r01s41_tune_zpipe.log;
// tools/count_variants.py; profiles/r01_count_mix_sweep.log, r01_count_variants.log) used to
// pick R: VALU-only accumulation is flat in R; the mixed VALU/SALU one is best at R = 8.
inline double pair_rate(int R, bool mix) {
  if (!mix) return 0.465;
  switch (R) {
    case 8: return 0.605;
    case 4: return 0.582;
    case 2: return 0.504;
    default: return 0.465;
  }
}

inline CompletePlan plan_complete(int64_t max_nx, int64_t max_nz, int32_t n_shards,
                                  bool mix = false) {
  CompletePlan p{8, 1, 1, max_nz, 0};
  double best = -1.0;
  for (int R : {8, 4, 2, 1}) {  // least modelled time per shard (padded slots / rate)
    if (g_force_R && R != g_force_R) continue;
    const int64_t slots = ceil_div(max_nx, (int64_t)kWave * R) * kWave * R;
    const double cost = (double)slots / pair_rate(R, mix);
    if (best < 0 || cost < best * (1.0 - 1e-9)) {
      best = cost;
      p.R = R;
    }
  }
  p.tiles_x = (int)ceil_div(max_nx, (int64_t)kWave * p.R);  // wave tiles
  // Many short z-chunks balance the tail across 256 CUs (measured: 1024-long chunks beat
  // 5k-15k chunks by 10-30% on 64 shards of 15625); below ~512 the per-block x loads and
  // epilogue start to show.
  const int64_t target = 256 * 128 * (kBlock / kWave);  // wave items
  const int64_t base = (int64_t)p.tiles_x * n_shards;
  int64_t zc = base >= target ? 1 : ceil_div(target, base);
  const int64_t min_chunk = 512;
  zc = std::min<int64_t>(zc, std::max<int64_t>(1, max_nz / min_chunk));
  zc = std::max<int64_t>(zc, ceil_div(max_nz, (int64_t)1 << 24));  // u32 counters never wrap
  p.z_chunk = ceil_div(max_nz, zc);
  p.z_chunk = ceil_div(p.z_chunk, 8) * 8;
  if (g_force_zchunk > 0) p.z_chunk = g_force_zchunk;
  p.zchunks = (int)ceil_div(max_nz, p.z_chunk);
  p.blocks = ceil_div((int64_t)p.tiles_x * p.zchunks * n_shards, kBlock / kWave);
  return p;
}

template <typename T, int PRED>
int launch_complete(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                    int32_t n_shards, int64_t max_nx, int64_t max_nz, uint64_t* out,
                    const NextStep& nxt, hipStream_t st) {
  // scalar-unit counting for the one-bit predicate on doubles (NaN padding)
  constexpr bool kMixable = std::is_floating_point<T>::value;
  const bool mix = kMixable && g_scalar_mix;
  const CompletePlan p = plan_complete(max_nx, max_nz, n_shards, mix);
  TW_ARG_CHECK((p.blocks + nxt.blocks) * (kBlock / kWave) < (1ll << 31),
               "tw_count_pairs: grid too large (%lld blocks)",
               (long long)p.blocks);
  TW_ARG_CHECK(p.z_chunk < (1ll << 30), "tw_count_pairs: z chunk too large");
  const T* xs = (const T*)x;
  const T* zs = (const T*)z;
  auto* o = (unsigned long long*)out;
  dim3 g((unsigned)(p.blocks + nxt.blocks)), b(kBlock);
#define TW_CC(R_, NS_) hipLaunchKernelGGL((k_count_complete<T, R_, NS_, PRED>), g, b, 0, st, xs, x_off, zs, z_off, n_shards, p.tiles_x, p.zchunks, p.z_chunk, o, nxt)
  if constexpr (kMixable) {
    if (mix) {
      switch (p.R) {
#ifndef TW_NS8
#define TW_NS8 4
#endif
#ifndef TW_NS4
#define TW_NS4 2
#endif
        case 8: TW_CC(8, TW_NS8); break;
        case 4: TW_CC(4, TW_NS4); break;
        case 2: TW_CC(2, 1); break;
        default: TW_CC(1, 0); break;
      }
      TW_LAUNCH_CHECK();
      return TW_OK;
    }
  }
  switch (p.R) {
    case 8: TW_CC(8, 0); break;
    case 4: TW_CC(4, 0); break;
    case 2: TW_CC(2, 0); break;
    default: TW_CC(1, 0); break;
  }
#undef TW_CC
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T>
int dispatch_complete(int32_t pred, const void* x, const int64_t* x_off, const void* z,
                      const int64_t* z_off, int32_t n_shards, int64_t max_nx, int64_t max_nz,
                      uint64_t* out, const NextStep& nxt, hipStream_t st) {
  switch (pred) {
    case TW_PRED_GT: return launch_complete<T, TW_PRED_GT>(x, x_off, z, z_off, n_shards, max_nx, max_nz, out, nxt, st);
    case TW_PRED_HALF: return launch_complete<T, TW_PRED_HALF>(x, x_off, z, z_off, n_shards, max_nx, max_nz, out, nxt, st);
    case TW_PRED_SUBGT: return launch_complete<T, TW_PRED_SUBGT>(x, x_off, z, z_off, n_shards, max_nx, max_nz, out, nxt, st);
  }
  set_error("tw_count_pairs: unknown predicate %d", pred);
  return TW_ERR_ARG;
}

constexpr int kPPT = 8;  // pairs per thread in the incomplete kernels

template <typename T, int PRED, typename I>
int launch_idx(const void* x, const void* z, const I* ix, const I* iz,
               const int64_t* pair_off, int32_t n_shards, int64_t max_pairs, uint64_t* out,
               hipStream_t st) {
  const int64_t bps = std::max<int64_t>(1, ceil_div(max_pairs, (int64_t)kBlock * kPPT));
  TW_ARG_CHECK(bps * n_shards < (1ll << 31), "tw_count_pairs_idx: grid too large");
  hipLaunchKernelGGL((k_count_idx<T, PRED, kPPT, I>), dim3((unsigned)(bps * n_shards)), dim3(kBlock), 0, st,
                     (const T*)x, (const T*)z, ix, iz, pair_off, (int)bps, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

template <typename T, int PRED>
int launch_rng(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
               int32_t n_shards, int64_t B, uint64_t seed, uint64_t sid, uint64_t* out,
               hipStream_t st) {
  const int64_t bps = std::max<int64_t>(1, ceil_div(B, (int64_t)kBlock * kPPT));
  TW_ARG_CHECK(bps * n_shards < (1ll << 31), "tw_count_pairs_rng: grid too large");
  hipLaunchKernelGGL((k_count_rng<T, PRED, kPPT>), dim3((unsigned)(bps * n_shards)), dim3(kBlock), 0, st,
                     (const T*)x, x_off, (const T*)z, z_off, B, (int)bps, (uint32_t)seed,
                     (uint32_t)(seed >> 32), (uint32_t)sid, (unsigned long long*)out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

}  // namespace tw

using namespace tw;

extern "C" int tw_count_set_scalar_mix(int32_t on) {
  TW_ARG_CHECK(on == 0 || on == 1, "tw_count_set_scalar_mix: 0 or 1");
  g_scalar_mix = on;
  return TW_OK;
}

extern "C" int tw_count_set_plan(int32_t R, int64_t z_chunk) {
  TW_ARG_CHECK(R == 0 || R == 1 || R == 2 || R == 4 || R == 8, "tw_count_set_plan: R in {0,1,2,4,8}");
  TW_ARG_CHECK(z_chunk >= 0 && z_chunk < (1ll << 30), "tw_count_set_plan: bad z_chunk");
  g_force_R = R;
  g_force_zchunk = z_chunk;
  return TW_OK;
}

extern "C" int tw_count_pairs(const void* d_x, const int64_t* d_x_off, const void* d_z,
                              const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                              int64_t max_nz, int32_t dtype, int32_t pred, uint64_t* d_out,
                              void* stream) {
  TW_ARG_CHECK(n_shards >= 0, "tw_count_pairs: n_shards < 0");
  TW_ARG_CHECK(max_nx >= 0 && max_nz >= 0, "tw_count_pairs: negative shard size");
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (max_nx == 0 || max_nz == 0) return TW_OK;
  const NextStep none{};
  if (dtype == TW_F64) return dispatch_complete<double>(pred, d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_out, none, st);
  if (dtype == TW_I64) return dispatch_complete<long long>(pred, d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_out, none, st);
  set_error("tw_count_pairs: unknown dtype %d", dtype);
  return TW_ERR_ARG;
}

// Spare blocks given to the next repartition: enough threads for ~8 gathers each, at most
// 2 per CU, a multiple of the XCD count.  Tuning hook tw_count_step_set_plan overrides the
// number and placement.
// Measured (tools/tune_step.py, bench workload): the last 512-768 blocks cost ~8 us over the
// bare count (they fill the count's tail); leading / spread placements cost 18-23 us.
static int g_step_blocks = 0, g_step_every = 0, g_step_tail = 1;
static int next_step_blocks(int64_t elems) {
  int64_t b = ceil_div(elems, (int64_t)kBlock * 8);
  b = std::min<int64_t>(std::max<int64_t>(b, 8), 512);
  if (g_step_blocks > 0) b = g_step_blocks;
  return (int)(ceil_div(b, kXcds) * kXcds);
}

extern "C" int tw_count_step_set_plan(int32_t blocks, int32_t every, int32_t tail) {
  TW_ARG_CHECK(blocks >= 0 && every >= 0 && every % kXcds == 0 && (tail == 0 || tail == 1),
               "tw_count_step_set_plan: blocks >= 0, every a multiple of 8, tail 0/1");
  g_step_blocks = blocks;
  g_step_every = every;
  g_step_tail = tail;
  return TW_OK;
}

extern "C" int tw_count_pairs_step(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                   const int64_t* d_z_off, int32_t n_shards, int64_t max_nx,
                                   int64_t max_nz, int32_t dtype, int32_t pred, uint64_t* d_out,
                                   int64_t n_x, void* d_x_next, uint64_t key_x, int64_t n_z,
                                   void* d_z_next, uint64_t key_z, uint64_t* d_out_next,
                                   int32_t n_next_shards, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && n_x >= 0 && n_z >= 0 &&
                   n_x < (1ll << 60) && n_z < (1ll << 60) && n_next_shards >= 0,
               "tw_count_pairs_step: bad sizes");
  TW_ARG_CHECK(dtype == TW_F64 || dtype == TW_I64, "tw_count_pairs_step: unknown dtype %d", dtype);
  TW_ARG_CHECK(pred == TW_PRED_GT || pred == TW_PRED_HALF || pred == TW_PRED_SUBGT,
               "tw_count_pairs_step: unknown predicate %d", pred);
  TW_ARG_CHECK(d_x_next == nullptr || ((n_x == 0 || d_x_next != d_x) &&
                                       (n_z == 0 || (d_z_next != nullptr && d_z_next != d_z))),
               "tw_count_pairs_step: next arrays must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  NextStep nxt{};
  if (d_x_next != nullptr) {
    nxt = NextStep{(const uint64_t*)d_x, (uint64_t*)d_x_next, n_x, (const uint64_t*)d_z,
                   (uint64_t*)d_z_next, n_z, (unsigned long long*)d_out_next,
                   d_out_next ? (int64_t)n_next_shards : 0,
                   make_feistel(std::max<int64_t>(n_x, 1), key_x),
                   make_feistel(std::max<int64_t>(n_z, 1), key_z),
                   next_step_blocks(n_x + n_z), 0, g_step_tail};
    // spread over the grid by default: one group of 8 every `every` blocks
    const CompletePlan p = plan_complete(std::max<int64_t>(max_nx, 1),
                                         std::max<int64_t>(max_nz, 1), std::max(n_shards, 1),
                                         dtype == TW_F64 &&
                                             g_scalar_mix);
    const int ng = nxt.blocks / kXcds;
    nxt.every = g_step_every ? g_step_every
                             : (int)std::max<int64_t>(kXcds, (p.blocks / ng) / kXcds * kXcds);
    if (n_shards == 0 || max_nx == 0 || max_nz == 0 ||
        (int64_t)(ng - 1) * nxt.every + kXcds > p.blocks + nxt.blocks)
      nxt.every = kXcds;  // leading blocks
  } else if (d_out_next != nullptr && n_next_shards > 0) {
    TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
  }
  if (n_shards == 0 || max_nx == 0 || max_nz == 0) {  // nothing to count: only the next step
    if (nxt.blocks == 0) return TW_OK;
    hipLaunchKernelGGL((k_count_complete<double, 1, 0, TW_PRED_GT>), dim3(nxt.blocks), dim3(kBlock),
                       0, st, nullptr, nullptr, nullptr, nullptr, 0, 1, 1, 1, nullptr, nxt);
    TW_LAUNCH_CHECK();
    return TW_OK;
  }
  if (dtype == TW_F64) return dispatch_complete<double>(pred, d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_out, nxt, st);
  return dispatch_complete<long long>(pred, d_x, d_x_off, d_z, d_z_off, n_shards, max_nx, max_nz, d_out, nxt, st);
}

namespace tw {
template <typename I>
int count_idx(const void* d_x, const void* d_z, const I* d_ix, const I* d_iz,
              const int64_t* d_pair_off, int32_t n_shards, int64_t max_pairs, int32_t dtype,
              int32_t pred, uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_pairs >= 0, "tw_count_pairs_idx: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (max_pairs == 0) return TW_OK;
#define TW_IDX(T, P) return launch_idx<T, P, I>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, d_out, st)
  if (dtype == TW_F64) {
    if (pred == TW_PRED_GT || pred == TW_PRED_SUBGT) TW_IDX(double, TW_PRED_GT);
    if (pred == TW_PRED_HALF) TW_IDX(double, TW_PRED_HALF);
  } else if (dtype == TW_I64) {
    if (pred == TW_PRED_GT) TW_IDX(long long, TW_PRED_GT);
    if (pred == TW_PRED_HALF) TW_IDX(long long, TW_PRED_HALF);
    if (pred == TW_PRED_SUBGT) TW_IDX(long long, TW_PRED_SUBGT);
  }
#undef TW_IDX
  set_error("tw_count_pairs_idx: unknown dtype %d / predicate %d", dtype, pred);
  return TW_ERR_ARG;
}
}  // namespace tw

extern "C" int tw_count_pairs_idx(const void* d_x, const void* d_z, const int64_t* d_ix,
                                  const int64_t* d_iz, const int64_t* d_pair_off,
                                  int32_t n_shards, int64_t max_pairs, int32_t dtype,
                                  int32_t pred, uint64_t* d_out, void* stream) {
  return count_idx<int64_t>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, dtype, pred,
                            d_out, stream);
}

extern "C" int tw_count_pairs_idx32(const void* d_x, const void* d_z, const int32_t* d_ix,
                                    const int32_t* d_iz, const int64_t* d_pair_off,
                                    int32_t n_shards, int64_t max_pairs, int32_t dtype,
                                    int32_t pred, uint64_t* d_out, void* stream) {
  return count_idx<int32_t>(d_x, d_z, d_ix, d_iz, d_pair_off, n_shards, max_pairs, dtype, pred,
                            d_out, stream);
}

extern "C" int tw_count_pairs_rng(const void* d_x, const int64_t* d_x_off, const void* d_z,
                                  const int64_t* d_z_off, int32_t n_shards, int64_t B,
                                  uint64_t seed, uint64_t stream_id, int32_t dtype, int32_t pred,
                                  uint64_t* d_out, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && B >= 0, "tw_count_pairs_rng: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (n_shards == 0) return TW_OK;
  TW_HIP_CHECK(tw_zero_async(d_out, 0, sizeof(uint64_t) * n_shards, st));
  if (B == 0) return TW_OK;
#define TW_RNG(T, P) return launch_rng<T, P>(d_x, d_x_off, d_z, d_z_off, n_shards, B, seed, stream_id, d_out, st)
  if (dtype == TW_F64) {
    if (pred == TW_PRED_GT || pred == TW_PRED_SUBGT) TW_RNG(double, TW_PRED_GT);
    if (pred == TW_PRED_HALF) TW_RNG(double, TW_PRED_HALF);
  } else if (dtype == TW_I64) {
    if (pred == TW_PRED_GT) TW_RNG(long long, TW_PRED_GT);
    if (pred == TW_PRED_HALF) TW_RNG(long long, TW_PRED_HALF);
    if (pred == TW_PRED_SUBGT) TW_RNG(long long, TW_PRED_SUBGT);
  }
#undef TW_RNG
  set_error("tw_count_pairs_rng: unknown dtype %d / predicate %d", dtype, pred);
  return TW_ERR_ARG;
}
