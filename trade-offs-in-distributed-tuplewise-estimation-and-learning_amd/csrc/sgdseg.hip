// sgdseg.hip — a whole segment of SGD steps in ONE persistent launch (SURVEY.md §8 rows L1/L2;
// narrow rows d <= 32: the C4 shuttle shape d = 10, N = 100).
//
//   for it in segment:                                    learning-experiment/make_exps.py:126-141
//       grads = [grad_inc_block(w, B, margin) per shard]  compute_stats.py:146-162
//       g = mean(grads, axis=0) + reg*w; dw = momentum*dw + lr*g (SGD: lr*g); w -= dw
//
// Launch-per-step (the gradient + update launches, or tw_sgd_step) pays a kernel boundary per
// step against a C4 step of ~8 us.  Here one block per shard (all co-resident) runs the whole
// segment with ONE grid barrier per step (k_sgd_segment_narrow below), and over ranks the same
// kernel exchanges the shard gradients with the other ranks' kernels through IPC-mapped peer
// buffers instead of a host collective (PEER, csrc/peer.h).  Wide rows (d > 32, C5) run per-step
// launches: a wide persistent segment (grid barriers between gradient and update) measured
// slower than the launches at C5 and was removed in round 5.
//
// Inter-block hand-offs (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup
// visibility"): every handed-off word is stored and loaded with agent-scope relaxed atomics
// (global_store/load sc1), each storing wave waits vmcnt(0), the block barriers, then ONE lane
// adds to the monotonic arrival counter (release), and the poller's one acquire fence follows
// its relaxed poll (the contract is spelled out at seg_arrive / seg_poll below).  Any new
// handed-off word must keep to ld_agent / st_agent.
// Residency: a plain launch of <= occupancy x CUs blocks is co-resident on an otherwise idle GPU
// (the learning loop runs on one stream); every spin is still bounded (2 s of the 100 MHz wall
// clock): a block that times out raises the abort word, every other waiter sees it and exits,
// and the caller finds ctl[1] != 0 afterwards (the segment's results are then invalid).
#include "peer.h"
#include "sgd_common.h"
#include <algorithm>

namespace tw {

constexpr uint64_t kSegSpinTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

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
// TW_SEG_BARRIER (A/B builds, tools/ab_barrier.py): 0 (default since round 5) = relaxed
// arrival and spin, no fence; 1 = acquire loads in the spin; 2 = the release/acquire form
// above (round 4).  Form 0 is the fence-free hand-off of MI355X_MICROARCH.md §Workgroup
// dispatch, "Valid forms": EVERY handed-off word goes out as an sc1 store (st_agent) and comes
// back as an sc1 load (ld_agent), each storing wave drains them (s_waitcnt vmcnt(0)) before the
// workgroup barrier and ONE lane's agent-scope atomic add, and the consumer polls with sc1
// loads and joins a workgroup barrier before loading — no L2 write-back per arrival and no
// invalidate per poll (the peer segment has used the same form at system scope all round).
// C4: 124-125k steps/s with form 2 against 132k with form 0 (profiles/
// r04s8_ab_barrier_fence_wait.log).
#ifndef TW_SEG_BARRIER
#define TW_SEG_BARRIER 0
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

// ---- peers: the narrow segment over ranks (round 5) ----------------------------------------
// With several ranks (one process per GPU) the shard gradients of a step are exchanged IN the
// persistent launch instead of by a host-enqueued RCCL all-gather between two launches: every
// rank owns one peer buffer (csrc/peer.hip: device memory allocated uncached, mapped into every
// other rank through an IPC handle), and each block pushes its shard's d gradient words into
// EVERY rank's slot for the step (global shard order), then adds one arrival to every rank's
// counter.  A rank's blocks wait until its own counter shows all n_total shards of the step
// (the ranks' blocks together), read the n_total x d slot from their own memory and apply the
// same shard-ordered update as the one-process kernel: the trajectory is the one-GPU one, bit
// for bit.  Memory model across devices: every handed-off word (gradient words, counters) is
// stored and loaded with SYSTEM-scope relaxed atomics on uncached memory (sc0 sc1: no cache of
// any device keeps a line), each storing wave waits vmcnt(0) before the workgroup barrier that
// precedes its block's counter adds, and the consumer loads only after its poll has matched
// (the system-scope analogue of the guide's sc1 hand-off form, table row 1).
// Slots: step e (global, counted from the rank's epoch) writes slot e & 1; a block writes it
// on rank p only after its own counter showed every block's arrival for step e - 1, i.e. after
// every block of every rank finished reading slot (e - 2) & 1 — two slots suffice, also across
// launches (the epoch word continues the parity).  Counters are monotonic (64-bit): the wait
// of step e is arrivals >= (e + 1) * n_total.

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

template <int LOSS, bool PEER>
__global__ __launch_bounds__(kBlock) void k_sgd_segment_narrow(
    const double* __restrict__ X, const double* __restrict__ Z, int64_t d,
    const int64_t* __restrict__ rows_x, int64_t kx, const int64_t* __restrict__ rows_z,
    int64_t kz, const int64_t* __restrict__ ix, const int64_t* __restrict__ iz,
    int64_t draw_stride, int64_t B, double margin, uint64_t seed,
    const uint64_t* __restrict__ d_step, uint32_t shard_base, int n_shards, int nsteps,
    const double* __restrict__ w_in, const double* __restrict__ dw_in, double reg, double lr,
    double momentum, double* grads0, double* grads1, double* __restrict__ w_out,
    double* __restrict__ dw_out, uint32_t* ctl, int64_t n_X, int64_t n_Z, uint64_t swr_mod,
    uint64_t swr_base, TabSteps tab, PeerSeg ps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* diff = (double*)smem;         // B * d
  double* flag = diff + B * d;          // B pair weights
  double* wsh = flag + B;               // kNarrowMaxD: this step's w
  double* gt = wsh + kNarrowMaxD;       // n_shards * d (peers: n_total * d): the previous
                                        // step's shard gradients
  __shared__ int s_ok;
  const int s = blockIdx.x, tid = threadIdx.x, dd = (int)d, G = gridDim.x;
  // the shards of the update: this launch's blocks, or every rank's (peers)
  const int n_upd = PEER ? ps.n_total : n_shards;
  const int ng = n_upd * dd;
  const uint64_t step0 = d_step ? *d_step : 0;
  // peers: the global step count before this launch (steps done by earlier peer launches)
  const uint64_t ep = PEER ? __hip_atomic_load(ps.epoch, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) : 0;
  const size_t slot_words = (size_t)ps.n_total * dd;
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
      if constexpr (PEER) {
        // every rank's blocks have pushed step ep + k - 1 into this rank's slot
        if (!peer_wait(ps.my_ctr, (ep + (uint64_t)k) * (uint64_t)ps.n_total, ctl + 1, &s_ok))
          return;
        const double* gin = ps.my_slot + ((ep + (uint64_t)k - 1) & 1) * slot_words;
        for (int e = tid; e < ng; e += kBlock) gt[e] = ld_sys(gin + e);
      } else {
        if (!seg_wait(ctl, (uint32_t)k * (uint32_t)G, &s_ok)) return;
        const double* gin = ((k - 1) & 1) ? grads1 : grads0;
        for (int e = tid; e < ng; e += kBlock) gt[e] = ld_agent(gin + e);
      }
      __syncthreads();
      if (tid < dd) {
        double sum = 0.0;  // shard order, as np.mean(axis=0) / k_sgd_update
        int r = 0;
        for (; r + 8 <= n_upd; r += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gt[(r + u) * dd + tid];
#pragma unroll
          for (int u = 0; u < 8; ++u) sum += v[u];
        }
        for (; r < n_upd; ++r) sum += gt[r * dd + tid];
        const double g = sum / (double)n_upd + reg * wj;
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
      if constexpr (PEER) {
        // this shard's row of step ep + k into every rank's slot (global shard order)
        const size_t o = ((ep + (uint64_t)k) & 1) * slot_words +
                         (size_t)(shard_base + (uint32_t)s) * dd + tid;
        for (int p = 0; p < ps.G; ++p) st_sys(ps.slot[p] + o, a / (double)B);
      } else {
        st_agent(((k & 1) ? grads1 : grads0) + (int64_t)s * d + tid, a / (double)B);
      }
    }
    if constexpr (PEER) {
      // every storing wave's stores performed, then one lane per rank adds this block's
      // arrival (the barrier also ends every thread's use of diff / flag / gt)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid < ps.G)
        __hip_atomic_fetch_add(ps.ctr[tid], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      seg_arrive(ctl, B <= kBlock - kWave ? kBlock - kWave : 0);  // also: every thread is done
                                                                  // with diff / flag / gt
    }
  }
  if constexpr (PEER) {
    // the last step's update in the launch (block 0): w_out / dw_out, the epoch, the step
    // counter — every block of this launch has read epoch and step counter long before
    if (s == 0 && nsteps > 0) {
      const uint64_t e = ep + (uint64_t)nsteps;
      if (!peer_wait(ps.my_ctr, e * (uint64_t)ps.n_total, ctl + 1, &s_ok)) return;
      const double* gin = ps.my_slot + ((e - 1) & 1) * slot_words;
      for (int i = tid; i < ng; i += kBlock) gt[i] = ld_sys(gin + i);
      __syncthreads();
      if (tid < dd) {
        double sum = 0.0;
        int r = 0;
        for (; r + 8 <= n_upd; r += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gt[(r + u) * dd + tid];
#pragma unroll
          for (int u = 0; u < 8; ++u) sum += v[u];
        }
        for (; r < n_upd; ++r) sum += gt[r * dd + tid];
        const double g = sum / (double)n_upd + reg * wj;
        const double st = momentum >= 0.0 ? momentum * dwj + lr * g : lr * g;
        w_out[tid] = wj - st;
        dw_out[tid] = st;
      }
      if (tid == 0) {
        __hip_atomic_store(ps.epoch, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d_step) *(uint64_t*)d_step = step0 + (uint64_t)nsteps;
      }
    }
    return;
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
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu,
                                                   k_sgd_segment_narrow<TW_LOSS_HINGE, false>,
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
                          uint64_t swr_base, void* stream, TabSteps tab = TabSteps{0, 0, 0, 0},
                          const PeerSeg* peer = nullptr) {
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
  if (peer)
    TW_ARG_CHECK(peer->n_total >= n_shards && (int64_t)peer->n_total * d <= kNarrowMaxGrads &&
                     narrow_lds(d, peer->n_total, B) <= 64 * 1024,
                 "tw_sgd_segment_narrow_peer: %d shards in all unsupported", peer->n_total);
  if (nsteps == 0) return TW_OK;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = narrow_lds(d, peer ? peer->n_total : n_shards, B);
  const PeerSeg ps = peer ? *peer : PeerSeg{};
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(n_shards), dim3(kBlock), lds, st, d_X, d_Z, d, d_rows_x, kx,
                       d_rows_z, kz, d_ix, d_iz, draw_stride, B, margin, seed, d_step,
                       (uint32_t)shard_base, (int)n_shards, (int)nsteps, d_w_in, d_dw_in, reg,
                       lr, momentum, d_grads0, d_grads1, d_w_out, d_dw_out, d_ctl, n_X, n_Z,
                       swr_mod, swr_base, tab, ps);
  };
  if (peer) {
    if (loss == TW_LOSS_LOGISTIC)
      go(k_sgd_segment_narrow<TW_LOSS_LOGISTIC, true>);
    else
      go(k_sgd_segment_narrow<TW_LOSS_HINGE, true>);
  } else if (loss == TW_LOSS_LOGISTIC) {
    go(k_sgd_segment_narrow<TW_LOSS_LOGISTIC, false>);
  } else {
    go(k_sgd_segment_narrow<TW_LOSS_HINGE, false>);
  }
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

// The narrow persistent segment over ranks (round 5; csrc/peer.h): the local shards
// [shard_base, shard_base + n_shards) of n_total, their gradients pushed into every rank's
// peer buffer (d_peer_bases: G device addresses in rank order — this rank's own buffer and
// the IPC-mapped ones of the others), the update of every step from this rank's own slot, the
// last one in the launch (w / dw in place; d_step advanced by nsteps when given).
static int peer_seg_of(void* const* d_peer_bases, int32_t G, int32_t rank, int32_t n_total,
                       int64_t d, PeerSeg& ps) {
  TW_ARG_CHECK(d_peer_bases != nullptr && G >= 1 && G <= kPeerMax && rank >= 0 && rank < G &&
                   n_total >= 1,
               "peer segment: bad ranks (G=%d, rank=%d, at most %d ranks)", G, rank, kPeerMax);
  ps = PeerSeg{};
  for (int p = 0; p < G; ++p) {
    char* b = (char*)d_peer_bases[p];
    TW_ARG_CHECK(b != nullptr, "peer segment: rank %d's buffer missing", p);
    ps.slot[p] = (double*)(b + kPeerHdr);
    ps.ctr[p] = (unsigned long long*)(b + kPeerSegCtr);
  }
  char* mine = (char*)d_peer_bases[rank];
  ps.my_ctr = (unsigned long long*)(mine + kPeerSegCtr);
  ps.epoch = (unsigned long long*)(mine + kPeerEpoch);
  ps.my_slot = (const double*)(mine + kPeerHdr);
  ps.G = G;
  ps.n_total = n_total;
  return TW_OK;
}

extern "C" int tw_sgd_segment_narrow_peer(
    const double* d_X, const double* d_Z, int64_t d, const int64_t* d_rows_x, int64_t kx,
    const int64_t* d_rows_z, int64_t kz, const int64_t* d_ix, const int64_t* d_iz,
    int64_t draw_stride, int32_t n_shards, int64_t B, double margin, int32_t loss,
    uint64_t seed, uint64_t* d_step, int32_t shard_base, int32_t nsteps, int64_t n_X,
    int64_t n_Z, int64_t swr_mod, double* d_w, double* d_dw, double reg, double lr,
    double momentum, uint32_t* d_ctl, void* const* d_peer_bases, int32_t G, int32_t rank,
    int32_t n_total, void* stream) {
  PeerSeg ps;
  if (const int rc = peer_seg_of(d_peer_bases, G, rank, n_total, d, ps)) return rc;
  TW_ARG_CHECK(shard_base + n_shards <= n_total, "tw_sgd_segment_narrow_peer: shards past n_total");
  TW_ARG_CHECK(swr_mod >= 0 && (swr_mod == 0 || (d_step != nullptr && n_X >= 1 && n_Z >= 1)),
               "tw_sgd_segment_narrow_peer: swr_mod needs d_step, n_X, n_Z");
  TW_ARG_CHECK(swr_mod > 0 || (d_rows_x != nullptr && d_rows_z != nullptr),
               "tw_sgd_segment_narrow_peer: row tables or swr_mod");
  // the gradient slots of the one-process kernel are not used: the peer slots replace them
  return segment_narrow(d_X, d_Z, d, swr_mod ? nullptr : d_rows_x, kx,
                        swr_mod ? nullptr : d_rows_z, kz, d_ix, d_iz, draw_stride, n_shards, B,
                        margin, loss, seed, d_step, shard_base, nsteps, d_w, d_dw, reg, lr,
                        momentum, d_w, d_w, d_w, d_dw, d_ctl, swr_mod ? n_X : 1,
                        swr_mod ? n_Z : 1, (uint64_t)swr_mod, 0, stream, TabSteps{0, 0, 0, 0},
                        &ps);
}
