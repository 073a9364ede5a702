// devshuffle.hip — the swaps of NumPy's RandomState.shuffle (legacy _shuffle_raw: for
// i = n-1 down to 1, swap a[i] and a[j_i], j_i <= i) applied on the device to 8-byte items,
// from the index draws the host made in NumPy's order (numpy_rng.cpp tw_np_shuffle_draws32).
// The drop-in's UN shuffles the caller's X and Z in place before cutting blocks
// (compute_stats.py:66-67, estimation-experiment/main.py:46-47); at C3 size the host's
// sequential swaps (one cache miss per swap) were half of est.UnNT's host time.
//
// Parallel rounds with deterministic reservations: iteration i touches positions i and j_i; it
// may run once no EARLIER iteration (larger i) that touches either position is still pending.
// Each round every pending iteration writes its priority into both positions (atomicMax); an
// iteration that finds its own priority in both runs its swap, the others stay pending.  Two
// iterations that run in one round touch disjoint positions, and every iteration runs after all
// earlier iterations sharing a position with it, so the result is the sequential loop's
// permutation, bit for bit.  The Knuth shuffle's iteration dependence depth is O(log n) w.h.p.
// (Shun, Gu, Blelloch, Fineman, Gibbons, SODA 2015): ~3.5 ln n rounds measured.
//
// Reservations carry the round: key = (round << 32) | g, so stale keys of earlier rounds lose
// every atomicMax and the two reservation arrays (round parity) never need clearing.  A round
// reads the reservations of ITS parity and writes the next round's into the other array, so
// the checks of one launch never see the writes of the same launch.  Positions and priorities
// of X and Z share one global numbering (Z's shifted by nx): both arrays run in the same
// launches, never interacting.
#include "tw_common.h"
#include <algorithm>
#include <cmath>

namespace tw {

constexpr int kShThreads = 256;

struct ShItem {
  uint64_t* a;     // the array the iteration swaps in
  int64_t i, j;    // local positions
  int64_t gi, gj;  // global positions (reservation slots)
};

__device__ __forceinline__ ShItem sh_item(int64_t g, uint64_t* x, uint64_t* z,
                                          const uint32_t* jx, const uint32_t* jz, int64_t nx) {
  ShItem it;
  if (g < nx) {
    it.a = x;
    it.i = g;
    it.j = jx[g];
    it.gj = it.j;
  } else {
    it.a = z;
    it.i = g - nx;
    it.j = jz[it.i];
    it.gj = nx + it.j;
  }
  it.gi = g;
  return it;
}

__device__ __forceinline__ unsigned long long sh_key(int round, int64_t g) {
  return ((unsigned long long)(unsigned)round << 32) | (unsigned long long)g;
}

// Iterations enter in kShWindows chunks of decreasing i (priority order): round r checks the
// iterations still pending from round r-1 plus chunk r, which reserved in round r-1's launch
// (chunk 0 in k_sh_reserve0); only iterations of the entered chunks reserve, and no later
// chunk can block them (lower priority).  Fewer failed attempts than letting all n iterations
// compete from round 0: ~1.5 n attempts instead of ~3.5 n at 16 chunks, for a few more rounds
// (~58 vs ~55 at n = 1e6).
constexpr int kShWindows = 16;

struct ShChunks {  // chunk c of an array of n items: local i in [hi(c) - size(c), hi(c)), i >= 1
  int64_t nx, nz, px, pz;
  __device__ __forceinline__ int64_t lo_x(int c) const {
    return std::max<int64_t>(1, nx - (int64_t)(c + 1) * px);
  }
  __device__ __forceinline__ int64_t hi_x(int c) const {
    return std::max<int64_t>(1, nx - (int64_t)c * px);
  }
  __device__ __forceinline__ int64_t lo_z(int c) const {
    return std::max<int64_t>(1, nz - (int64_t)(c + 1) * pz);
  }
  __device__ __forceinline__ int64_t hi_z(int c) const {
    return std::max<int64_t>(1, nz - (int64_t)c * pz);
  }
  __device__ __forceinline__ int64_t count(int c) const {
    return c < kShWindows ? (hi_x(c) - lo_x(c)) + (hi_z(c) - lo_z(c)) : 0;
  }
  // t-th iteration of chunk c as a global index
  __device__ __forceinline__ int64_t item(int c, int64_t t) const {
    const int64_t cx = hi_x(c) - lo_x(c);
    return t < cx ? lo_x(c) + t : nx + lo_z(c) + (t - cx);
  }
};

__device__ __forceinline__ void sh_reserve(unsigned long long* R, int64_t g, int64_t gj,
                                           unsigned long long k) {
  atomicMax(R + g, k);
  if (gj != g) atomicMax(R + gj, k);
}

// chunk 0's reservations for round 0
__global__ __launch_bounds__(kShThreads) void k_sh_reserve0(const uint32_t* __restrict__ jx,
                                                           const uint32_t* __restrict__ jz,
                                                           ShChunks ch,
                                                           unsigned long long* __restrict__ R0) {
  const int64_t total = ch.count(0);
  for (int64_t t = (int64_t)blockIdx.x * kShThreads + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kShThreads) {
    const int64_t g = ch.item(0, t);
    const int64_t gj = g < ch.nx ? (int64_t)jx[g] : ch.nx + (int64_t)jz[g - ch.nx];
    sh_reserve(R0, g, gj, sh_key(0, g));
  }
}

// round r over [pending list of round r-1 | chunk r | chunk r+1 (reserve only)]: an iteration
// holding both of its reservations runs its swap, the others reserve for round r+1 and go to
// list_out; chunk r+1 only reserves (its iterations are pending in round r+1 by range)
__global__ __launch_bounds__(kShThreads) void k_sh_round(
    int round, uint64_t* __restrict__ x, uint64_t* __restrict__ z, const uint32_t* __restrict__ jx,
    const uint32_t* __restrict__ jz, ShChunks ch, const uint32_t* __restrict__ list_in,
    const unsigned* __restrict__ cnt_in, uint32_t* __restrict__ list_out,
    unsigned* __restrict__ cnt_out, const unsigned long long* __restrict__ Rcur,
    unsigned long long* __restrict__ Rnext) {
  const int64_t n_list = *cnt_in;
  const int64_t n_cur = n_list + ch.count(round);
  const int64_t total = n_cur + ch.count(round + 1);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t stride = (int64_t)gridDim.x * kShThreads;
  const int64_t nx = ch.nx;
  // the loop bound is wave-uniform, so the ballot below sees every lane of the wave
  for (int64_t base = (int64_t)blockIdx.x * kShThreads + (threadIdx.x - lane); base < total;
       base += stride) {
    const int64_t t = base + lane;
    bool pending = false;
    int64_t g = 0;
    if (t < total) {
      g = t < n_list ? (int64_t)list_in[t]
                     : (t < n_cur ? ch.item(round, t - n_list) : ch.item(round + 1, t - n_cur));
      const ShItem it = sh_item(g, x, z, jx, jz, nx);
      if (t >= n_cur) {
        sh_reserve(Rnext, it.gi, it.gj, sh_key(round + 1, g));
      } else {
        const unsigned long long k = sh_key(round, g);
        if (Rcur[it.gi] == k && Rcur[it.gj] == k) {
          const uint64_t vi = it.a[it.i], vj = it.a[it.j];
          it.a[it.j] = vi;
          it.a[it.i] = vj;
        } else {
          sh_reserve(Rnext, it.gi, it.gj, sh_key(round + 1, g));
          pending = true;
        }
      }
    }
    const unsigned long long m = __ballot(pending);
    if (m) {
      unsigned at = 0;
      if (lane == 0) at = atomicAdd(cnt_out, (unsigned)__popcll(m));
      at = __shfl(at, 0, kWave);
      if (pending) list_out[at + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)g;
    }
  }
}

// The tail of a batch in ONE workgroup: once every chunk has entered, only the pending list is
// left and it shrinks geometrically (x0.8 per round), so the last ~40 rounds of a 1e6-item
// shuffle are a few thousand iterations each — a launch apiece cost more than the work.  Rounds
// [r0, r1) run here back to back with workgroup barriers between them: the same per-iteration
// step as k_sh_round (same reservations, same lists and counters), one CU, so plain loads and
// stores of the arrays and lists stay coherent through its L1; the reservations, written by
// L2 atomics, are read with agent-scope loads (not L1).  Stops early once a round leaves no
// pending iteration (cnt_final = 0); otherwise cnt_final = the count after round r1 - 1, as
// after a batch of launches.
constexpr int kShFinThreads = 1024;
__global__ __launch_bounds__(kShFinThreads) void k_sh_finish(
    int r0, int r1, uint64_t* __restrict__ x, uint64_t* __restrict__ z,
    const uint32_t* __restrict__ jx, const uint32_t* __restrict__ jz, int64_t nx,
    uint32_t* __restrict__ L0, uint32_t* __restrict__ L1, unsigned* __restrict__ cnt,
    unsigned long long* __restrict__ R0, unsigned long long* __restrict__ R1,
    unsigned* __restrict__ cnt_final) {
  __shared__ unsigned s_n;
  const int lane = threadIdx.x & (kWave - 1);
  for (int r = r0; r < r1; ++r) {
    // round r reads the list of round r-1 and counter cnt[r - r0], writes the other list and
    // cnt[r - r0 + 1] (the caller's cnt points at the counter of round r0's input)
    if (threadIdx.x == 0)
      s_n = __hip_atomic_load(cnt + (r - r0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int64_t n_list = s_n;
    if (n_list == 0) {
      if (threadIdx.x == 0) *cnt_final = 0u;
      return;
    }
    const uint32_t* list_in = (r & 1) ? L0 : L1;  // L[(r + 1) & 1]
    uint32_t* list_out = (r & 1) ? L1 : L0;       // L[r & 1]
    const unsigned long long* Rcur = (r & 1) ? R1 : R0;
    unsigned long long* Rnext = (r & 1) ? R0 : R1;
    unsigned* cnt_out = cnt + (r - r0) + 1;
    for (int64_t base = threadIdx.x - lane; base < n_list; base += kShFinThreads) {
      const int64_t t = base + lane;
      bool pending = false;
      int64_t g = 0;
      if (t < n_list) {
        g = (int64_t)list_in[t];
        const ShItem it = sh_item(g, x, z, jx, jz, nx);
        const unsigned long long k = sh_key(r, g);
        const unsigned long long a = __hip_atomic_load(Rcur + it.gi, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_load(Rcur + it.gj, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        if (a == k && b == k) {
          const uint64_t vi = it.a[it.i], vj = it.a[it.j];
          it.a[it.j] = vi;
          it.a[it.i] = vj;
        } else {
          sh_reserve(Rnext, it.gi, it.gj, sh_key(r + 1, g));
          pending = true;
        }
      }
      const unsigned long long m = __ballot(pending);
      if (m) {
        unsigned at = 0;
        if (lane == 0) at = atomicAdd(cnt_out, (unsigned)__popcll(m));
        at = __shfl(at, 0, kWave);
        if (pending) list_out[at + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)g;
      }
    }
    __syncthreads();  // this round's swaps, reservations and list entries before the next
  }
  if (threadIdx.x == 0)
    *cnt_final = __hip_atomic_load(cnt + (r1 - r0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct ShPlan {
  int rounds;                       // rounds per batch
  int64_t R, list, cnt, bytes;      // workspace offsets
};

static int g_sh_rounds = 0;  // tw_shuffle_swaps_set_rounds (tests: force resumed batches)
static int g_sh_tail = 1;    // tw_shuffle_swaps_set_tail: the one-workgroup tail (k_sh_finish)

inline ShPlan plan_sh(int64_t nx, int64_t nz) {
  ShPlan p{};
  const int64_t n = std::max<int64_t>(2, std::max(nx, nz));
  // every chunk enters within the first batch (so the pending list is all that is left)
  p.rounds = g_sh_rounds > 0 ? std::max(g_sh_rounds, kShWindows + 1)
                             : (int)std::ceil(4.5 * std::log((double)n)) + 8 + kShWindows;
  auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  const int64_t total = nx + nz;
  p.R = 0;
  p.list = al(2 * total * 8);
  p.cnt = p.list + al(2 * total * 4);
  p.bytes = p.cnt + al((int64_t)(p.rounds + 1) * 4);
  return p;
}

}  // namespace tw

using namespace tw;

extern "C" int64_t tw_shuffle_swaps_work_bytes(int64_t nx, int64_t nz) {
  if (nx < 0 || nz < 0) return 0;
  return plan_sh(nx, nz).bytes;
}

// rounds per batch (0: the default 4.5 ln n + 8 + kShWindows; at least kShWindows + 1); a test
// hook for the resumed-batch path
extern "C" int tw_shuffle_swaps_set_rounds(int32_t rounds) {
  TW_ARG_CHECK(rounds >= 0 && rounds < (1 << 20), "tw_shuffle_swaps_set_rounds: bad count");
  g_sh_rounds = rounds;
  return TW_OK;
}

// 1: the tail rounds of a batch in one workgroup (default); 0: one launch per round (A/B, tests)
extern "C" int tw_shuffle_swaps_set_tail(int32_t on) {
  TW_ARG_CHECK(on == 0 || on == 1, "tw_shuffle_swaps_set_tail: 0 or 1");
  g_sh_tail = on;
  return TW_OK;
}

extern "C" int32_t tw_shuffle_swaps_rounds(int64_t nx, int64_t nz) {
  return plan_sh(std::max<int64_t>(nx, 0), std::max<int64_t>(nz, 0)).rounds;
}

namespace tw {
// rounds [k_begin, k_end) of one batch (k counts from round0); k_begin = 0 also sets the batch
// up (first: clear the workspace, reserve round 0; else continue from the previous batch's
// list); last: the batch's remaining rounds (k_end ignored), its tail and *d_pending
static int swaps_batch(uint64_t* d_x, int64_t nx, uint64_t* d_z, int64_t nz,
                       const uint32_t* d_jx, const uint32_t* d_jz, int first, int round0,
                       int k_begin, int k_end, int last, void* d_work, uint32_t* d_pending,
                       hipStream_t st) {
  const int64_t total = nx + nz;
  if (nx <= 1 && nz <= 1) {  // no iteration at all
    if (last) TW_HIP_CHECK(tw_zero_async(d_pending, 0, 4, st));
    return TW_OK;
  }
  const ShPlan p = plan_sh(nx, nz);
  char* w = (char*)d_work;
  unsigned long long* R[2] = {(unsigned long long*)(w + p.R),
                              (unsigned long long*)(w + p.R) + total};
  uint32_t* L[2] = {(uint32_t*)(w + p.list), (uint32_t*)(w + p.list) + total};
  unsigned* cnt = (unsigned*)(w + p.cnt);
  auto grid_for = [&](double est) {
    return (unsigned)std::max<double>(
        1.0, std::min<double>(2048.0, std::ceil(est / (kShThreads * 4.0))));
  };
  ShChunks ch;
  ch.nx = nx;
  ch.nz = nz;
  ch.px = nx > 1 ? ceil_div(nx - 1, kShWindows) : 0;
  ch.pz = nz > 1 ? ceil_div(nz - 1, kShWindows) : 0;
  const double per = (double)total / kShWindows;
  if (k_begin == 0) {
    if (first) {
      TW_HIP_CHECK(tw_zero_async(w, 0, (size_t)p.bytes, st));
      hipLaunchKernelGGL(k_sh_reserve0, dim3(grid_for(per)), dim3(kShThreads), 0, st, d_jx,
                         d_jz, ch, R[0]);
    } else {
      // continue: the previous batch's last list (parity of its last round) is round0's
      // input; its count moves to slot 0
      TW_HIP_CHECK(hipMemcpyAsync(cnt, cnt + p.rounds, 4, hipMemcpyDeviceToDevice, st));
      TW_HIP_CHECK(tw_zero_async(cnt + 1, 0, (size_t)p.rounds * 4, st));
    }
  }
  // rounds of the whole grid while chunks enter and the list is long, then the tail in one
  // workgroup (k_sh_finish) once the expected list is under ~kShFinThreads * 8 iterations
  const double tail_items = (double)kShFinThreads * 8;
  int k_fin = p.rounds;
  for (int k = k_begin; k < p.rounds; ++k) {
    const int r = round0 + k;
    const double est =
        r < kShWindows ? 2.0 * per : 2.0 * per * std::pow(0.8, (double)(r - kShWindows + 1));
    if (g_sh_tail && r > kShWindows && est < tail_items) {
      k_fin = k;
      break;
    }
    if (!last && k >= k_end) return TW_OK;  // a part: the next one continues at k_end
    // round r reads the list of round r-1 (L[(r+1)&1]) and writes L[r&1]
    hipLaunchKernelGGL(k_sh_round, dim3(grid_for(est)), dim3(kShThreads), 0, st, r, d_x, d_z,
                       d_jx, d_jz, ch, L[(r + 1) & 1], cnt + k, L[r & 1], cnt + k + 1, R[r & 1],
                       R[(r + 1) & 1]);
  }
  TW_LAUNCH_CHECK();
  if (!last) return TW_OK;
  if (k_fin < p.rounds) {
    hipLaunchKernelGGL(k_sh_finish, dim3(1), dim3(kShFinThreads), 0, st, round0 + k_fin,
                       round0 + p.rounds, d_x, d_z, d_jx, d_jz, (int64_t)nx, L[0], L[1],
                       cnt + k_fin, R[0], R[1], d_pending);
    TW_LAUNCH_CHECK();
    // the next batch (if any) starts from cnt[p.rounds]
    TW_HIP_CHECK(hipMemcpyAsync(cnt + p.rounds, d_pending, 4, hipMemcpyDeviceToDevice, st));
    return TW_OK;
  }
  TW_HIP_CHECK(hipMemcpyAsync(d_pending, cnt + p.rounds, 4, hipMemcpyDeviceToDevice, st));
  return TW_OK;
}
}  // namespace tw

// Enqueue one batch of tw_shuffle_swaps_rounds rounds.  first != 0: the first batch (clears
// the workspace, reserves round 0, round 0 runs over every iteration); round0 = 0.  Later
// batches (first == 0, round0 = the previous round0 + rounds) continue from the previous
// batch's pending list.  *d_pending (device) receives the number of iterations still pending
// after the batch: the caller reads it and enqueues another batch while it is not 0 — with
// ~3.5 ln n rounds needed and 4.5 ln n + 8 per batch, one batch finishes w.h.p.
extern "C" int tw_shuffle_swaps(uint64_t* d_x, int64_t nx, uint64_t* d_z, int64_t nz,
                                const uint32_t* d_jx, const uint32_t* d_jz, int32_t first,
                                int32_t round0, void* d_work, uint32_t* d_pending,
                                void* stream) {
  TW_ARG_CHECK(nx >= 0 && nz >= 0 && d_work != nullptr && d_pending != nullptr && round0 >= 0,
               "tw_shuffle_swaps: bad arguments");
  TW_ARG_CHECK(nx + nz < (1ll << 31), "tw_shuffle_swaps: more than 2^31 items");
  TW_ARG_CHECK((nx <= 1 || (d_x && d_jx)) && (nz <= 1 || (d_z && d_jz)),
               "tw_shuffle_swaps: null array");
  return swaps_batch(d_x, nx, d_z, nz, d_jx, d_jz, first, round0, 0, 0, 1, d_work, d_pending,
                     (hipStream_t)stream);
}

// The draw windows of the swap rounds: iterations enter in kShWindows chunks of
// p = ceil((n - 1) / kShWindows) draws each, window c holding i in [max(1, n - (c + 1) p),
// n - c p) — the order the host draws them in.
extern "C" int32_t tw_shuffle_swaps_windows() { return kShWindows; }

// The FIRST batch of tw_shuffle_swaps in parts, enqueued as the draws arrive (the streamed
// last shuffle of the drop-in, _engine.DeviceShuffles): rounds [r_begin, r_end) — round r
// reads the draws of windows 0 .. r + 1, so once windows [0, c) are on the device rounds up to
// c - 2 may run (r_end = c - 1).  r_begin = 0 also clears the workspace and reserves round 0
// (window 0 needed); last != 0 enqueues every remaining round, the tail and *d_pending
// (r_end ignored).  The parts in sequence (r_begin = the previous r_end) are exactly
// tw_shuffle_swaps(first = 1, round0 = 0).
extern "C" int tw_shuffle_swaps_part(uint64_t* d_x, int64_t nx, uint64_t* d_z, int64_t nz,
                                     const uint32_t* d_jx, const uint32_t* d_jz,
                                     int32_t r_begin, int32_t r_end, int32_t last,
                                     void* d_work, uint32_t* d_pending, void* stream) {
  TW_ARG_CHECK(nx >= 0 && nz >= 0 && d_work != nullptr && d_pending != nullptr &&
                   r_begin >= 0 && (last || (r_end >= r_begin && r_end < kShWindows)),
               "tw_shuffle_swaps_part: bad arguments (a part ends before round %d)",
               kShWindows);
  TW_ARG_CHECK(nx + nz < (1ll << 31), "tw_shuffle_swaps_part: more than 2^31 items");
  TW_ARG_CHECK((nx <= 1 || (d_x && d_jx)) && (nz <= 1 || (d_z && d_jz)),
               "tw_shuffle_swaps_part: null array");
  return swaps_batch(d_x, nx, d_z, nz, d_jx, d_jz, 1, 0, r_begin, r_end, last, d_work,
                     d_pending, (hipStream_t)stream);
}
