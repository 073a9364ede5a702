// sgdseg.hip — a whole segment of SGD steps in ONE persistent launch (SURVEY.md §8 rows L1/L2,
// wide rows 32 < d <= 512: the C5 shape d = 512, N = 256).
//
//   for it in segment:                                    learning-experiment/make_exps.py:126-141
//       grads = [grad_inc_block(w, B, margin) per shard]  compute_stats.py:146-162
//       g = mean(grads, axis=0) + reg*w; dw = momentum*dw + lr*g (SGD: lr*g); w -= dw
//
// Launch-per-step (k_hinge_grad_stream + k_sgd_update) pays, every step, two kernel
// boundaries, the update kernel's own latency chain and the gradient's ramp (the first rows of
// every shard are requested only after the draws and the row tables resolve).  Here the grid is
// one block per CU (LDS 159 KiB => 1 block/CU, grid <= resident capacity, blocks loop over
// shards when N exceeds it) and every step is:
//   1. wait for barrier 2k (w of step k published), read w;
//   2. the block's shards, exactly as k_hinge_grad_stream: same chunking, same lane partials +
//      butterfly per pair, column sums in pair order from +0.0 — identical bits;
//   3. publish the shard gradients, arrive at barrier 2k+1;
//   4. PREFETCH: draws, row tables and the first two chunks' rows of step k+1's first shard are
//      issued now — they are independent of w, so they stream while the other blocks arrive;
//      the two chunks land as diff rows in LDS (the dot products wait for w);
//   5. wait for barrier 2k+1, update this block's columns [b*d/G, (b+1)*d/G) — shard-order sum
//      from +0.0, /N, + reg*w, momentum: k_sgd_update's arithmetic — publish w, dw, arrive at
//      barrier 2k+2.
//
// Inter-block hand-offs (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup
// visibility", table row 1): every handed-off word (grads, w, dw) is stored and loaded with
// agent-scope relaxed atomics (global_store/load sc1: write-through, L1-bypassing, coherent
// across the XCDs' L2s); each storing wave waits vmcnt(0), the block barriers, then ONE lane
// adds to the monotonic arrival counter; one lane polls it with s_sleep, then a block barrier.
// This is the guide's sc1-hand-off form (MI355X_MICROARCH.md "Valid forms", table row 1: every
// handed-off byte stored AND loaded sc1, each storing wave's vmcnt(0) before the workgroup
// barrier that precedes the one-lane agent-scope add, an sc1 poll, one workgroup per CU), so no
// release fence on the add and no acquire on the poll: on gfx950 those lower to buffer_wbl2 sc1
// / buffer_inv sc1 at ~1.7 us each (the guide's fence table), two hand-offs per step against a
// C4 step of ~8 us.  Any new handed-off word must keep to ld_agent / st_agent below.
// Residency: a plain launch of <= occupancy x CUs blocks is co-resident on an otherwise idle GPU
// (the learning loop runs on one stream); every spin is still bounded (2 s of the 100 MHz wall
// clock): a block that times out raises the abort word, every other waiter sees it and exits,
// and the caller finds ctl[1] != 0 afterwards (the segment's results are then invalid).
#include "sgd_common.h"
#include <algorithm>

// Per-step timestamps for kernel studies (tools/phase_segment.py builds a separate library with
// -DTW_SEG_TIMING; the product build compiles them out): thread 0 of block b stamps the 100 MHz
// wall clock at point p of step k < 32 — 0 w read, 1 gradients stored, 4 their stores landed
// (block barrier), 2 barrier 2k+1 passed, 5 the update's gradient loads landed, 3 update
// stored, 6 its stores landed (counter add), 7 step start (before waiting for barrier 2k).
#ifdef TW_SEG_TIMING
__device__ unsigned long long g_seg_t[1 << 16];
#define SEG_STAMP(k, p)                                                                     \
  do {                                                                                      \
    if (threadIdx.x == 0 && (k) < 32)                                                       \
      g_seg_t[(((size_t)blockIdx.x * 32 + (k)) * 8 + (p)) & 0xFFFF] = wall_clock64();       \
  } while (0)
extern "C" int tw_debug_seg_times(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_seg_t), sizeof(unsigned long long) * n) ==
                 hipSuccess ? 0 : 2;
}
#else
#define SEG_STAMP(k, p) \
  do {                  \
  } while (0)
#endif

namespace tw {

constexpr uint64_t kSegSpinTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
constexpr int kSegStage = 1408;                   // 11 KiB: LDS total 159.3 KiB

__device__ __forceinline__ double ld_agent(const double* p) {
  const uint64_t v = __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store((uint64_t*)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// ctl[0]: arrivals (monotonic within a launch, zeroed before it); ctl[1]: abort word, sticky
// (zeroed once by the caller: a later launch that finds it set exits at its first wait).
// Memory-model contract of the grid barrier: every published word is an agent-scope atomic
// store (st_agent); each storing wave waits for its own stores (s_waitcnt vmcnt(0) — the
// block barrier's workgroup-scope release does not wait for another wave's vector stores to
// reach the agent-coherent level), the block barrier orders them before thread 0's arrival,
// and the arrival is an agent-scope RELEASE add (gfx950: buffer_wbl2 sc1 before the atomic).
// The poller spins on RELAXED loads of the counter and, once it has seen the target, issues
// ONE agent-scope ACQUIRE fence (buffer_inv sc1) — acquire loads in the spin itself would
// invalidate the L2 on every iteration; the fence after the last relaxed load that read the
// release's value gives the same synchronisation (fence-atomic rule), and s_waitcnt vmcnt(0)
// holds the block barrier after the poll until the invalidate has completed, so every wave's
// loads of the published words (ld_agent) come after it.
// TW_SEG_BARRIER (A/B builds, tools/ab_barrier.py): 0 = relaxed arrival and spin, no fence
// (round 3); 1 = acquire loads in the spin; 2 (default) = as above.
#ifndef TW_SEG_BARRIER
#define TW_SEG_BARRIER 2
#endif
// arriver: the thread that adds the arrival — the release's L2 write-back (~0.6 us on gfx950)
// stalls only its wave, so the narrow kernel hands it to the last wave, which has no pairs in
// the next step's chain when B <= 192 (C4: B = 100): the stall hides behind the other waves'
// draws -> rows -> diff rows (tools/ab_barrier.py)
__device__ __forceinline__ void seg_arrive(uint32_t* ctl, int arriver = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's published stores landed
  __syncthreads();
  if ((int)threadIdx.x == arriver)
    __hip_atomic_fetch_add(ctl, 1u, TW_SEG_BARRIER ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// one lane: spin until the counter reaches target (false: aborted or timed out -> abort word)
__device__ __forceinline__ bool seg_poll(uint32_t* ctl, uint32_t target) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(ctl, TW_SEG_BARRIER == 1 ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
        wall_clock64() - t0 > kSegSpinTicks) {
      __hip_atomic_store(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (TW_SEG_BARRIER == 2) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // the invalidate completes before the block barrier lets any wave load (the consumer
    // recipe of MI355X_MICROARCH.md: relaxed poll -> acquire -> vmcnt(0) -> barrier -> loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  return true;
}

// the whole block waits (thread 0 polls)
__device__ __forceinline__ bool seg_wait(uint32_t* ctl, uint32_t target, int* s_ok) {
  if (threadIdx.x == 0) *s_ok = seg_poll(ctl, target) ? 1 : 0;
  __syncthreads();
  return *s_ok != 0;
}

// FULL: d == 512 (every lane column valid: no per-column masks, fewer live SGPR masks)
template <int LOSS, bool FULL>
__global__ __launch_bounds__(kWideBlock) void k_sgd_segment_wide(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz,
    int64_t draw_stride, int n_shards, int64_t B, double margin, uint64_t seed,
    uint64_t* d_step, uint32_t shard_base, int nsteps, double* w, double* dw, double* grads,
    double reg, double lr, double momentum, uint32_t* ctl, int prefetch_rows) {
  __shared__ double diff[2][kStreamCH * kWideMaxD];  // 128 KiB
  __shared__ int64_t prx[kIdxPhase], prz[kIdxPhase];  // 16 KiB
  __shared__ double flag[2][kStreamCH];
  __shared__ double stage[kSegStage];                 // the update's shard-gradient staging
  __shared__ double wsh[kWideMaxD];                   // w of the current step
  __shared__ int s_ok;
  const int G = gridDim.x, blk = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wid = tid / kWave;
  const int dd = FULL ? kWideMaxD : (int)d;
  const uint64_t step0 = d_step ? *d_step : 0;
  const int cA = (int)((int64_t)blk * dd / G), cB = (int)((int64_t)(blk + 1) * dd / G);
  double zv[2][kWideCols], xv[2][kWideCols];
  double acc = 0.0;  // thread j < d: column j of the current shard

  // pair rows of phase [P0, P0 + np) of shard s at step k -> prx/prz (as k_hinge_grad_stream)
  // absolute X / Z rows of pair b of shard s at step k (draw, then the SWR row tables)
  auto pair_rows = [&](int s, int k, int64_t b, int64_t& rx, int64_t& rz) {
    int64_t ax, az;
    if (ix) {
      ax = ix[(int64_t)k * draw_stride + (int64_t)s * B + b];
      az = iz[(int64_t)k * draw_stride + (int64_t)s * B + b];
    } else {
      const u32x4 r = sgd_draw(seed, step0 + (uint64_t)k, (uint32_t)b, shard_base + (uint32_t)s,
                               kTagPairs);
      ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
      az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
    }
    rx = rows_x ? rows_x[(int64_t)s * kx + ax] : ax;
    rz = rows_z ? rows_z[(int64_t)s * kz + az] : az;
  };
  // rows of phase [P0, P0 + np) of shard s at step k -> prx/prz, threads t0, t0 + ts, ...
  auto setup = [&](int s, int k, int64_t P0, int np, int t0, int ts) {
    for (int t = t0; t < np; t += ts) pair_rows(s, k, P0 + t, prx[t], prz[t]);
  };
  auto load = [&](int st, int c0, int np) {  // this wave's pair of the chunk at c0 -> stage st
    const int t = c0 + wid;
    if (t < np) {
      const double* zr = Z + prz[t] * d;
      const double* xr = X + prx[t] * d;
#pragma unroll
      for (int c = 0; c < kWideCols; ++c) {
        const int j = lane + c * kWave;
        zv[st][c] = (FULL || j < dd) ? zr[j] : 0.0;
        xv[st][c] = (FULL || j < dd) ? xr[j] : 0.0;
      }
    }
  };
  // from_lds: the chunk's diff rows were written by the prefetch (same v, same order: bits)
  auto chunk = [&](int st, int c0, int np, bool from_lds) {
    const int nb = std::min(kStreamCH, np - c0);
    if (wid < nb) {
      double part = 0.0;
      if (from_lds) {
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          if (FULL || j < dd) part += diff[st][wid * dd + j] * wsh[j];
        }
      } else {
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          if (FULL || j < dd) {
            const double v = zv[st][c] - xv[st][c];
            diff[st][wid * dd + j] = v;
            part += v * wsh[j];
          }
        }
      }
      part = wave_sum_dpp_f64(part);
      if (lane == 0) flag[st][wid] = pair_weight<LOSS>(part + margin);
    }
    if (c0 + 2 * kStreamCH < np) load(st, c0 + 2 * kStreamCH, np);  // refill: chunk k+2
    __syncthreads();
    if (tid < dd) {
      double a = acc;
      int u0 = 0;
      for (; u0 + 8 <= nb; u0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[st][u0 + u], diff[st][(u0 + u) * dd + tid]);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
      }
      for (; u0 < nb; ++u0) a += weighted<LOSS>(flag[st][u0], diff[st][u0 * dd + tid]);
      acc = a;
    }
  };

  bool pre = false;       // step k's first shard: phase 0's row indices already in prx/prz
  bool pre_rows = false;  // ... and chunks 0/1 already as diff rows in LDS
  for (int k = 0; k < nsteps; ++k) {
    SEG_STAMP(k, 7);
    if (k > 0 && !seg_wait(ctl, (uint32_t)(2 * k) * (uint32_t)G, &s_ok)) return;
    if (tid < dd) wsh[tid] = ld_agent(w + tid);
    __syncthreads();
    SEG_STAMP(k, 0);
    for (int s = blk; s < n_shards; s += G) {
      acc = 0.0;
      for (int64_t P0 = 0; P0 < B; P0 += kIdxPhase) {
        const int np = (int)std::min<int64_t>(kIdxPhase, B - P0);
        const bool lds0 = pre_rows && P0 == 0;
        if (!(pre && P0 == 0)) {
          __syncthreads();  // the previous phase's readers of prx/prz and diff/flag are done
          setup(s, k, P0, np, tid, kWideBlock);
          __syncthreads();
        }
        if (!lds0) {
          load(0, 0, np);
          if (kStreamCH < np) load(1, kStreamCH, np);
        }
        int c0 = 0;
        for (; c0 + kStreamCH < np; c0 += 2 * kStreamCH) {
          chunk(0, c0, np, lds0 && c0 == 0);
          chunk(1, c0 + kStreamCH, np, lds0 && c0 == 0);
        }
        if (c0 < np) chunk(0, c0, np, lds0 && c0 == 0);
        pre = pre_rows = false;
      }
      if (tid < dd) st_agent(grads + (int64_t)s * d + tid, acc / (double)B);
    }
    SEG_STAMP(k, 1);
    seg_arrive(ctl);  // barrier 2k+1: every shard gradient of step k published
    SEG_STAMP(k, 4);
    const bool more = k + 1 < nsteps;
    if (wid == 0) {
      // control wave: waits for barrier 2k+1, updates columns [cA, cB), arrives at 2k+2.  It
      // has no loads in flight, so nothing queues in front of its polls and loads.
      int ok = 1;
      if (lane == 0) ok = seg_poll(ctl, (uint32_t)(2 * k + 1) * (uint32_t)G) ? 1 : 0;
      ok = __shfl(ok, 0, kWave);
      SEG_STAMP(k, 2);
      for (int g0 = cA; ok && g0 < cB; g0 += kWave) {  // column groups of <= 64 lanes
        const int nc = std::min(kWave, cB - g0);
        double wj = 0.0, dwj = 0.0;
        if (lane < nc) {
          wj = ld_agent(w + g0 + lane);
          if (momentum >= 0.0) dwj = ld_agent(dw + g0 + lane);
        }
        const int SS = kSegStage / nc;  // shards staged per pass
        double sum = 0.0;               // lane c < nc: column g0 + c, shard order from +0.0
        for (int s0 = 0; s0 < n_shards; s0 += SS) {
          const int ns = std::min(SS, n_shards - s0), tot = ns * nc;
          for (int e0 = 0; e0 < tot; e0 += 8 * kWave) {  // 8 loads in flight per lane
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int e = e0 + u * kWave + lane, r = e / nc;
              v[u] = e < tot ? ld_agent(grads + (int64_t)(s0 + r) * d + g0 + (e - r * nc)) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int e = e0 + u * kWave + lane;
              if (e < tot) stage[e] = v[u];
            }
          }
          __builtin_amdgcn_wave_barrier();
          SEG_STAMP(k, 5);
          if (lane < nc) {
            int r = 0;
            for (; r + 8 <= ns; r += 8) {
              double v[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) v[u] = stage[(r + u) * nc + lane];
#pragma unroll
              for (int u = 0; u < 8; ++u) sum += v[u];
            }
            for (; r < ns; ++r) sum += stage[r * nc + lane];
          }
          __builtin_amdgcn_wave_barrier();
        }
        if (lane < nc) {
          const double g = sum / (double)n_shards + reg * wj;
          const double stp = momentum >= 0.0 ? momentum * dwj + lr * g : lr * g;
          st_agent(dw + g0 + lane, stp);
          st_agent(w + g0 + lane, wj - stp);
        }
      }
      SEG_STAMP(k, 3);
      if (ok) {  // barrier 2k+2: this wave's w and dw stores landed (the only stores it signals)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        SEG_STAMP(k, 6);
        if (lane == 0)
          __hip_atomic_fetch_add(ctl, 1u, TW_SEG_BARRIER ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        if (!more && blk == 0 && lane == 0 && d_step) *d_step = step0 + (uint64_t)nsteps;
      }
    } else if (more && prefetch_rows) {
      // waves 1..15 prefetch step k+1's first shard: the 32 pairs of chunks 0 and 1 as diff
      // rows in LDS (wave w: pairs w-1, w+14, w+29), then phase 0's row indices (prx/prz free:
      // seg_arrive's barrier follows their last reads)
      const int np = (int)std::min<int64_t>(kIdxPhase, B);
      const int npre = std::min(np, 2 * kStreamCH);
      for (int t1 = wid - 1; t1 < npre; t1 += 2 * (kStreamCH - 1)) {
        const int t2 = t1 + (kStreamCH - 1);
        int64_t rx1, rz1, rx2 = 0, rz2 = 0;
        pair_rows(blk, k + 1, t1, rx1, rz1);
        if (t2 < npre) pair_rows(blk, k + 1, t2, rx2, rz2);
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          const bool in = FULL || j < dd;
          zv[0][c] = in ? Z[rz1 * d + j] : 0.0;
          xv[0][c] = in ? X[rx1 * d + j] : 0.0;
          zv[1][c] = (in && t2 < npre) ? Z[rz2 * d + j] : 0.0;
          xv[1][c] = (in && t2 < npre) ? X[rx2 * d + j] : 0.0;
        }
#pragma unroll
        for (int c = 0; c < kWideCols; ++c) {
          const int j = lane + c * kWave;
          if (FULL || j < dd) {
            diff[t1 / kStreamCH][(t1 % kStreamCH) * dd + j] = zv[0][c] - xv[0][c];
            if (t2 < npre) diff[t2 / kStreamCH][(t2 % kStreamCH) * dd + j] = zv[1][c] - xv[1][c];
          }
        }
      }
      setup(blk, k + 1, 0, np, tid - kWave, kWideBlock - kWave);
    } else if (more) {  // indices only: the rows stream once w is known
      setup(blk, k + 1, 0, (int)std::min<int64_t>(kIdxPhase, B), tid - kWave,
            kWideBlock - kWave);
    }
    pre = more;
    pre_rows = more && prefetch_rows;
  }
}

// ---- narrow rows (d <= 32, C4): a segment of k_sgd_step_narrow steps in ONE launch --------
// One block per shard (all co-resident), ONE grid barrier per step: the update is recomputed
// redundantly by every block from the published shard gradients (k_sgd_step_narrow's
// prologue), so no second barrier publishes w.  Per step:
//   1. the pair chain of step k (draws -> row tables -> rows -> diff rows in LDS) — independent
//      of w, so it runs BEFORE the barrier and overlaps the wait for the slowest block;
//   2. k > 0: wait until every block has published step k-1 (arrivals >= k*G), load the N x d
//      shard gradients of slot (k-1)&1 (agent scope), update w, dw in shard order exactly as
//      k_sgd_update / k_sgd_step_narrow;
//   3. S = diff . w + margin (sequential j), weights, column sums in row order from +0.0 ->
//      grads slot k&1 (agent-scope stores), arrive.
// Two gradient slots suffice: a block writes slot k&1 at step k only after barrier k, which
// needs every block to have finished step k-1 — and with it its reads of slot (k-2)&1.
// The state after the segment's last update goes to w_out / dw_out (block 0); the last step's
// gradients (slot (nsteps-1)&1) are applied by the caller's tw_sgd_update_to, as in the
// one-launch-per-step path.  Same arithmetic and order: same bits.
constexpr int kNarrowMaxD = 32, kNarrowMaxGrads = 4096;

// Replay segments through reshuffles (tw_sgd_segment_narrow_tables): the row tables are stacks
// of tables x / z words apart, and step k of the segment reads table (phase + k) / mod — the
// segment's first step is step `phase` of a reshuffle period.  mod = 0: one table.
struct TabSteps {
  int64_t x, z;
  uint64_t phase, mod;
};

template <int LOSS>
__global__ __launch_bounds__(kBlock) void k_sgd_segment_narrow(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz,
    int64_t draw_stride, int64_t B, double margin, uint64_t seed,
    const uint64_t* __restrict__ d_step, uint32_t shard_base, int n_shards, int nsteps,
    const double* __restrict__ w_in, const double* __restrict__ dw_in, double reg, double lr,
    double momentum, double* grads0, double* grads1, double* __restrict__ w_out,
    double* __restrict__ dw_out, uint32_t* ctl, int64_t n_X, int64_t n_Z, uint64_t swr_mod,
    uint64_t swr_base, TabSteps tab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* diff = (double*)smem;         // B * d
  double* flag = diff + B * d;          // B pair weights
  double* wsh = flag + B;               // kNarrowMaxD: this step's w
  double* gt = wsh + kNarrowMaxD;       // n_shards * d: the previous step's shard gradients
  __shared__ int s_ok;
  const int s = blockIdx.x, tid = threadIdx.x, dd = (int)d, G = gridDim.x;
  const int ng = n_shards * dd;
  const uint64_t step0 = d_step ? *d_step : 0;
  double wj = 0.0, dwj = 0.0;  // thread tid < d: column tid of w and dw
  if (tid < dd) {
    wj = w_in[tid];
    dwj = dw_in[tid];
    wsh[tid] = wj;
  }
  for (int k = 0; k < nsteps; ++k) {
    // replay through reshuffles: the row tables of this step's last reshuffle, table
    // (phase + k) / mod of the stacks (table 0: the tables in force when the segment starts)
    const int64_t tk = tab.mod ? (int64_t)((tab.phase + (uint64_t)k) / tab.mod) : 0;
    const int64_t* __restrict__ rtx = rows_x ? rows_x + tk * tab.x : nullptr;
    const int64_t* __restrict__ rtz = rows_z ? rows_z + tk * tab.z : nullptr;
    // 1. this step's pairs -> diff rows (independent of w)
    for (int t = tid; t < B; t += kBlock) {
      int64_t ax, az;
      if (ix) {
        ax = ix[(int64_t)k * draw_stride + (int64_t)s * B + t];
        az = iz[(int64_t)k * draw_stride + (int64_t)s * B + t];
      } else {
        const u32x4 r = sgd_draw(seed, step0 + (uint64_t)k, (uint32_t)t,
                                 shard_base + (uint32_t)s, kTagPairs);
        ax = (int64_t)mulhi_u64(((uint64_t)r.b << 32) | r.a, (uint64_t)kx);
        az = (int64_t)mulhi_u64(((uint64_t)r.d << 32) | r.c, (uint64_t)kz);
      }
      int64_t rxt, rzt;
      if (swr_mod) {
        // the SWR row tables in the kernel (device RNG): the rows k_swr_rows drew at this
        // step's last reshuffle, counter c - (c - base) % mod — one Philox per side, so a
        // segment runs through its reshuffles without a table-drawing launch
        const uint64_t c = step0 + (uint64_t)k, rc = c - (c - swr_base) % swr_mod;
        const u32x4 qx = sgd_draw(seed, rc, (uint32_t)ax, shard_base + (uint32_t)s, kTagRowsX);
        const u32x4 qz = sgd_draw(seed, rc, (uint32_t)az, shard_base + (uint32_t)s, kTagRowsZ);
        rxt = (int64_t)mulhi_u64(((uint64_t)qx.b << 32) | qx.a, (uint64_t)n_X);
        rzt = (int64_t)mulhi_u64(((uint64_t)qz.b << 32) | qz.a, (uint64_t)n_Z);
      } else {
        rxt = rtx ? rtx[(int64_t)s * kx + ax] : ax;
        rzt = rtz ? rtz[(int64_t)s * kz + az] : az;
      }
      const double* zr = Z + rzt * d;
      const double* xr = X + rxt * d;
      double* dr = diff + (int64_t)t * d;
#pragma unroll 4
      for (int j = 0; j < dd; ++j) dr[j] = zr[j] - xr[j];
    }
    // 2. the previous step's update, once every block has published its gradients
    if (k > 0) {
      if (!seg_wait(ctl, (uint32_t)k * (uint32_t)G, &s_ok)) return;
      const double* gin = ((k - 1) & 1) ? grads1 : grads0;
      for (int e = tid; e < ng; e += kBlock) gt[e] = ld_agent(gin + e);
      __syncthreads();
      if (tid < dd) {
        double sum = 0.0;  // shard order, as np.mean(axis=0) / k_sgd_update
        int r = 0;
        for (; r + 8 <= n_shards; r += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gt[(r + u) * dd + tid];
#pragma unroll
          for (int u = 0; u < 8; ++u) sum += v[u];
        }
        for (; r < n_shards; ++r) sum += gt[r * dd + tid];
        const double g = sum / (double)n_shards + reg * wj;
        const double st = momentum >= 0.0 ? momentum * dwj + lr * g : lr * g;
        wj = wj - st;
        dwj = st;
        wsh[tid] = wj;
      }
    }
    __syncthreads();
    // 3. S = diff . w + margin, weights, column sums in row order
    for (int t = tid; t < B; t += kBlock) {
      const double* dr = diff + (int64_t)t * d;
      double part = 0.0;
      for (int j = 0; j < dd; ++j) part += dr[j] * wsh[j];
      flag[t] = pair_weight<LOSS>(part + margin);
    }
    __syncthreads();
    if (tid < dd) {
      double a = 0.0;
      int t = 0;
      for (; t + 8 <= B; t += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = weighted<LOSS>(flag[t + u], diff[(t + u) * dd + tid]);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
      }
      for (; t < B; ++t) a += weighted<LOSS>(flag[t], diff[t * dd + tid]);
      st_agent(((k & 1) ? grads1 : grads0) + (int64_t)s * d + tid, a / (double)B);
    }
    seg_arrive(ctl, B <= kBlock - kWave ? kBlock - kWave : 0);  // also: every thread is done
                                                                // with diff / flag / gt
  }
  if (s == 0) {
    if (tid < dd) {
      w_out[tid] = wj;
      dw_out[tid] = dwj;
    }
    // leave the arrival counter at zero for the next launch (no memset node): block 0 waits
    // for the last arrivals of this launch, after which no block touches the counter
    if (nsteps > 0 && seg_wait(ctl, (uint32_t)nsteps * (uint32_t)G, &s_ok) && tid == 0)
      __hip_atomic_store(ctl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static int g_seg_grid = 0;      // tw_sgd_segment_set_grid: 0 = resident capacity
static int g_seg_prefetch = 1;  // tw_sgd_segment_set_prefetch: 1 = rows, 0 = indices only

static int seg_capacity() {
  static int cap[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cap[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, k_sgd_segment_wide<TW_LOSS_HINGE, false>, kWideBlock, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    // 145 KiB of LDS per block: one per CU (never trust more than that here)
    cap[dev] = std::min(per_cu, 1) * cus;
  }
  return cap[dev];
}

}  // namespace tw

using namespace tw;

static size_t narrow_lds(int64_t d, int32_t n_shards, int64_t B) {
  return sizeof(double) * ((size_t)B * d + B + kNarrowMaxD + (size_t)n_shards * d);
}

// every block resident at once (the kernel's grid barriers), within 64 KiB of LDS per block
extern "C" int tw_sgd_segment_narrow_ok(int64_t d, int32_t n_shards, int64_t B) {
  if (d < 1 || d > kNarrowMaxD || n_shards < 1 || (int64_t)n_shards * d > kNarrowMaxGrads ||
      B < 1 || narrow_lds(d, n_shards, B) > 64 * 1024)
    return 0;
  int dev = 0, per_cu = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sgd_segment_narrow<TW_LOSS_HINGE>,
                                                   kBlock, narrow_lds(d, n_shards, B)) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (int64_t)std::min(per_cu, 1) * cus >= n_shards;  // one block per CU at most
}

static int segment_narrow(const double* d_X, const double* d_Z, int64_t d,
                          const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                          int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                          int64_t draw_stride, int32_t n_shards, int64_t B, double margin,
                          int32_t loss, uint64_t seed, const uint64_t* d_step,
                          int32_t shard_base, int32_t nsteps, const double* d_w_in,
                          const double* d_dw_in, double reg, double lr, double momentum,
                          double* d_grads0, double* d_grads1, double* d_w_out, double* d_dw_out,
                          uint32_t* d_ctl, int64_t n_X, int64_t n_Z, uint64_t swr_mod,
                          uint64_t swr_base, void* stream, TabSteps tab = TabSteps{0, 0, 0, 0}) {
  // shape limits only: the residency query (tw_sgd_segment_narrow_ok) is a HIP API call the
  // caller makes once, before any stream capture — this entry runs inside captured graphs
  TW_ARG_CHECK(d >= 1 && d <= kNarrowMaxD && n_shards >= 1 &&
                   (int64_t)n_shards * d <= kNarrowMaxGrads && B >= 1 &&
                   narrow_lds(d, n_shards, B) <= 64 * 1024,
               "tw_sgd_segment_narrow: d=%lld, n_shards=%d, B=%lld unsupported", (long long)d,
               n_shards, (long long)B);
  TW_ARG_CHECK(kx >= 1 && kz >= 1 && shard_base >= 0 && nsteps >= 0 && nsteps <= (1 << 20) &&
                   draw_stride >= 0,
               "tw_sgd_segment_narrow: bad kx/kz/shard_base/nsteps/draw_stride");
  TW_ARG_CHECK((d_ix == nullptr) == (d_iz == nullptr), "tw_sgd_segment_narrow: ix and iz go together");
  TW_ARG_CHECK(d_ix != nullptr || d_step != nullptr, "tw_sgd_segment_narrow: device draws need d_step");
  TW_ARG_CHECK(d_w_in && d_dw_in && d_grads0 && d_grads1 && d_w_out && d_dw_out && d_ctl,
               "tw_sgd_segment_narrow: w, dw, both gradient slots, outputs and ctl required");
  TW_ARG_CHECK(loss == TW_LOSS_HINGE || loss == TW_LOSS_LOGISTIC, "unknown loss %d", loss);
  if (nsteps == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = narrow_lds(d, n_shards, B);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(n_shards), dim3(kBlock), lds, st, d_X, d_Z, d, d_rows_x, kx,
                       d_rows_z, kz, d_ix, d_iz, draw_stride, B, margin, seed, d_step,
                       (uint32_t)shard_base, (int)n_shards, (int)nsteps, d_w_in, d_dw_in, reg,
                       lr, momentum, d_grads0, d_grads1, d_w_out, d_dw_out, d_ctl, n_X, n_Z,
                       swr_mod, swr_base, tab);
  };
  if (loss == TW_LOSS_LOGISTIC)
    go(k_sgd_segment_narrow<TW_LOSS_LOGISTIC>);
  else
    go(k_sgd_segment_narrow<TW_LOSS_HINGE>);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_sgd_segment_narrow(const double* d_X, const double* d_Z, int64_t d,
                                     const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                                     int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                                     int64_t draw_stride, int32_t n_shards, int64_t B,
                                     double margin, int32_t loss, uint64_t seed,
                                     const uint64_t* d_step, int32_t shard_base, int32_t nsteps,
                                     const double* d_w_in, const double* d_dw_in, double reg,
                                     double lr, double momentum, double* d_grads0,
                                     double* d_grads1, double* d_w_out, double* d_dw_out,
                                     uint32_t* d_ctl, void* stream) {
  return segment_narrow(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, draw_stride,
                        n_shards, B, margin, loss, seed, d_step, shard_base, nsteps, d_w_in,
                        d_dw_in, reg, lr, momentum, d_grads0, d_grads1, d_w_out, d_dw_out, d_ctl,
                        1, 1, 0, 0, stream);
}

extern "C" int tw_sgd_segment_narrow_tables(
    const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x, int64_t kx,
    const int64_t* d_rows_z, int64_t kz, int64_t tab_x, int64_t tab_z, int64_t tab_phase,
    int64_t tab_mod, const int64_t* d_ix, const int64_t* d_iz, int64_t draw_stride,
    int32_t n_shards, int64_t B, double margin, int32_t loss, uint64_t seed,
    const uint64_t* d_step, int32_t shard_base, int32_t nsteps, const double* d_w_in,
    const double* d_dw_in, double reg, double lr, double momentum, double* d_grads0,
    double* d_grads1, double* d_w_out, double* d_dw_out, uint32_t* d_ctl, void* stream) {
  TW_ARG_CHECK(tab_mod >= 1 && tab_phase >= 0 && tab_phase < tab_mod &&
                   tab_x >= (int64_t)n_shards * kx && tab_z >= (int64_t)n_shards * kz &&
                   d_rows_x != nullptr && d_rows_z != nullptr,
               "tw_sgd_segment_narrow_tables: bad table stacks (stride, phase, mod)");
  return segment_narrow(d_X, d_Z, d, d_rows_x, kx, d_rows_z, kz, d_ix, d_iz, draw_stride,
                        n_shards, B, margin, loss, seed, d_step, shard_base, nsteps, d_w_in,
                        d_dw_in, reg, lr, momentum, d_grads0, d_grads1, d_w_out, d_dw_out, d_ctl,
                        1, 1, 0, 0, stream,
                        TabSteps{tab_x, tab_z, (uint64_t)tab_phase, (uint64_t)tab_mod});
}

extern "C" int tw_sgd_segment_narrow_swr(const double* d_X, const double* d_Z, int64_t d,
                                         int64_t n_X, int64_t n_Z, int64_t kx, int64_t kz,
                                         int32_t n_shards, int64_t B, double margin,
                                         int32_t loss, uint64_t seed, const uint64_t* d_step,
                                         int32_t shard_base, int32_t nsteps, int64_t swr_mod,
                                         uint64_t swr_base, const double* d_w_in,
                                         const double* d_dw_in, double reg, double lr,
                                         double momentum, double* d_grads0, double* d_grads1,
                                         double* d_w_out, double* d_dw_out, uint32_t* d_ctl,
                                         void* stream) {
  TW_ARG_CHECK(swr_mod >= 1 && n_X >= 1 && n_Z >= 1 && d_step != nullptr,
               "tw_sgd_segment_narrow_swr: swr_mod, n_X, n_Z >= 1 and d_step required");
  return segment_narrow(d_X, d_Z, d, nullptr, kx, nullptr, kz, nullptr, nullptr, 0, n_shards,
                        B, margin, loss, seed, d_step, shard_base, nsteps, d_w_in, d_dw_in, reg,
                        lr, momentum, d_grads0, d_grads1, d_w_out, d_dw_out, d_ctl, n_X, n_Z,
                        (uint64_t)swr_mod, swr_base, stream);
}

extern "C" int tw_sgd_segment_ok(int64_t d, int32_t n_shards) {
  return d > 32 && d <= kWideMaxD && n_shards >= 1;
}

extern "C" int tw_sgd_segment_set_grid(int32_t max_blocks) {
  TW_ARG_CHECK(max_blocks >= 0, "tw_sgd_segment_set_grid: max_blocks < 0");
  g_seg_grid = max_blocks;
  return TW_OK;
}

extern "C" int tw_sgd_segment_set_prefetch(int32_t rows) {
  TW_ARG_CHECK(rows == 0 || rows == 1, "tw_sgd_segment_set_prefetch: 0 or 1");
  g_seg_prefetch = rows;
  return TW_OK;
}

extern "C" int tw_sgd_segment(const double* d_X, const double* d_Z, int64_t d,
                              const int64_t* d_rows_x, int64_t kx, const int64_t* d_rows_z,
                              int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
                              int64_t draw_stride, int32_t n_shards, int64_t B, double margin,
                              int32_t loss, uint64_t seed, uint64_t* d_step, int32_t shard_base,
                              int32_t nsteps, double* d_w, double* d_dw, double* d_grads,
                              double reg, double lr, double momentum, uint32_t* d_ctl,
                              void* stream) {
  TW_ARG_CHECK(tw_sgd_segment_ok(d, n_shards), "tw_sgd_segment: d=%lld, n_shards=%d unsupported",
               (long long)d, n_shards);
  TW_ARG_CHECK(B >= 1 && B < (1ll << 32) && kx >= 1 && kz >= 1 && shard_base >= 0 &&
                   nsteps >= 0 && nsteps <= (1 << 20) && draw_stride >= 0,
               "tw_sgd_segment: bad B/kx/kz/shard_base/nsteps/draw_stride");
  TW_ARG_CHECK((d_ix == nullptr) == (d_iz == nullptr), "tw_sgd_segment: ix and iz go together");
  TW_ARG_CHECK(d_ix != nullptr || d_step != nullptr, "tw_sgd_segment: device draws need d_step");
  TW_ARG_CHECK(d_w && d_dw && d_grads && d_ctl, "tw_sgd_segment: w, dw, grads, ctl required");
  TW_ARG_CHECK(loss == TW_LOSS_HINGE || loss == TW_LOSS_LOGISTIC, "unknown loss %d", loss);
  if (nsteps == 0) return TW_OK;
  const int cap = seg_capacity();
  TW_ARG_CHECK(cap >= 1, "tw_sgd_segment: no resident capacity for the segment kernel");
  int grid = std::min(n_shards, cap);
  if (g_seg_grid > 0) grid = std::min(grid, g_seg_grid);
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_ctl, 0, sizeof(uint32_t), st));  // the arrival counter only
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWideBlock), 0, st, d_X, d_Z, d, d_rows_x, kx,
                       d_rows_z, kz, d_ix, d_iz, draw_stride, (int)n_shards, B, margin, seed,
                       d_step, (uint32_t)shard_base, (int)nsteps, d_w, d_dw, d_grads, reg, lr,
                       momentum, d_ctl, g_seg_prefetch);
  };
  const bool full = d == kWideMaxD;
  if (loss == TW_LOSS_LOGISTIC)
    full ? go(k_sgd_segment_wide<TW_LOSS_LOGISTIC, true>)
         : go(k_sgd_segment_wide<TW_LOSS_LOGISTIC, false>);
  else
    full ? go(k_sgd_segment_wide<TW_LOSS_HINGE, true>) : go(k_sgd_segment_wide<TW_LOSS_HINGE, false>);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
