// peer.hip — device-resident gradient exchange between ranks (round 5; SURVEY.md §8(e)
// "Learning").  Reference: the per-step shard mean of learning-experiment/make_exps.py:126-141
// (grads = UN_split(X_s, Z_s, grad_inc_block(w, B, margin)), compute_stats.py:44-46), which a
// multi-GPU run splits over ranks: every rank computes its shards' partial gradients and every
// rank needs all of them, in shard order, before the update.
//
// Over RCCL that is a host-enqueued all-gather between the gradient and the update launches:
// three host launches and a collective's latency per step, against an 8-us step on one GPU
// (C4).  Here the GPUs exchange the partials themselves, through one peer buffer per rank
// (layout: csrc/peer.h) allocated UNCACHED and mapped into every other rank with an IPC handle
// (xGMI peer access; HSA_ENABLE_IPC_MODE_LEGACY=0: dmabuf handles).  Two forms:
//  * the persistent narrow segment (csrc/sgdseg.hip, tw_sgd_segment_narrow_peer): C4's
//    segments, the exchange inside the launch;
//  * per step (any d, any gradient kernel; C5): the gradient launch writes the rank's
//    (N/G, d) partials as usual, then ONE tw_peer_step launch pushes them into every rank's
//    per-step slot of the step's parity, adds its arrivals to every rank's parity counter,
//    waits for all ranks' arrivals on its own counter and applies k_sgd_update's arithmetic
//    to the slot (same bits as the one-GPU update).  No host collective per step.
// Counter reuse of the per-step form: step(t) waits for counter[t & 1] >= P * G (P blocks per
// rank, a function of d); step(t + 1) zeroes this rank's counter[t & 1] (step(t) is done:
// stream order) in its block 0, whose arrivals on the peers come after that store (vmcnt(0)),
// and a peer can add to counter[t & 1] again only in step(t + 2), after its step(t + 1) saw
// all of this rank's arrivals of step t + 1 — block 0's included.  Slots likewise: slot t & 1
// of a rank is rewritten by step(t + 2), after every rank's step(t) has read it.
#include "peer.h"
#include <algorithm>
#include <cstring>

namespace tw {

// One launch per step after the gradient launch: its blocks push this rank's partials, then
// wait for every rank's arrivals and update.  The grid is capped (kStepBlocks, blocks looping
// over column groups) so that every rank's blocks are resident together: a waiting block holds
// its CU, and a rank whose blocks could not start would never arrive (ranks co-resident on one
// GPU in rehearsals included: 128 blocks of 32 KB LDS per rank, at least 10 ranks' grids fit).
constexpr int kStepBlocks = 128, kPUpdCols = 8, kPUpdRows = 512;

static int step_blocks(int64_t d) {
  return (int)std::min<int64_t>(kStepBlocks, ceil_div(d, (int64_t)kPUpdCols));
}

// (1) this rank's (rows, d) partials -> rows [row0, row0 + rows) of every rank's slot `par`,
//     then one arrival per block on every rank's counter of parity `par`;
// (2) wait for P * G arrivals on this rank's counter, then k_sgd_update (csrc/hinge.hip) on the
//     slot: the same shard-order sum from +0.0, /N, + reg * w, momentum — the same bits
__global__ __launch_bounds__(kBlock) void k_peer_step(const double* __restrict__ src,
                                                      int64_t words, int64_t off, PeerSeg ps,
                                                      int par, unsigned long long* reset,
                                                      uint64_t target, int n_shards, int64_t d,
                                                      double* w, double* dw, double reg,
                                                      double lr, double momentum,
                                                      uint64_t* __restrict__ d_step,
                                                      uint32_t* abort_word) {
  __shared__ double tile[kPUpdRows * kPUpdCols];
  __shared__ int s_ok;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(reset, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const size_t base = (size_t)par * ps.n_total + off;  // in words: ps.n_total holds N * d here
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < words;
       i += (int64_t)gridDim.x * kBlock) {
    const double v = src[i];
    for (int p = 0; p < ps.G; ++p)  // the peers' slots; this rank reads its own rows from src
      if (ps.slot[p] != ps.my_slot) st_sys(ps.slot[p] + base + i, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores (and the reset) done
  __syncthreads();
  if ((int)threadIdx.x < ps.G)
    __hip_atomic_fetch_add(ps.ctr[threadIdx.x], 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);

  if (!peer_wait(ps.my_ctr, target, abort_word, &s_ok)) return;
  if (d_step && blockIdx.x == 0 && threadIdx.x == 0) *d_step += 1;
  const double* slot = ps.my_slot + (size_t)par * ps.n_total;
  for (int64_t j0 = (int64_t)blockIdx.x * kPUpdCols; j0 < d;
       j0 += (int64_t)gridDim.x * kPUpdCols) {
    const int nc = (int)std::min<int64_t>(kPUpdCols, d - j0);
    double sum = 0.0;
    for (int s0 = 0; s0 < n_shards; s0 += kPUpdRows) {
      const int ns = std::min(kPUpdRows, n_shards - s0);
      __syncthreads();
      for (int e = threadIdx.x; e < ns * kPUpdCols; e += kBlock) {
        const int r = e / kPUpdCols, c = e - r * kPUpdCols;
        const int64_t at = (int64_t)(s0 + r) * d + j0 + c;  // word of the global slot
        tile[e] = c >= nc ? 0.0 : (at >= off && at < off + words) ? src[at - off]
                                                                   : ld_sys(slot + at);
      }
      __syncthreads();
      if ((int)threadIdx.x < nc) {
        int r = 0;
        for (; r + 8 <= ns; r += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = tile[(r + u) * kPUpdCols + threadIdx.x];
#pragma unroll
          for (int u = 0; u < 8; ++u) sum += v[u];
        }
        for (; r < ns; ++r) sum += tile[r * kPUpdCols + threadIdx.x];
      }
    }
    if ((int)threadIdx.x < nc) {
      const int64_t j = j0 + threadIdx.x;
      const double wj = w[j];
      const double g = sum / (double)n_shards + reg * wj;
      const double step = momentum >= 0.0 ? momentum * dw[j] + lr * g : lr * g;
      dw[j] = step;
      w[j] = wj - step;
    }
  }
}

// Column-owned form (round 6): rank p OWNS columns [cb(p), cb(p+1)) of w,
// cb(p) = p d / G.  One launch per step after the gradient launch:
//  (A) this rank's (rows, d) partials, each column only to its owner's slot of parity `par`
//      (1/G of the bytes of k_peer_step's push), then one arrival per block on every rank's
//      gradient counter of that parity;
//  (B) once P * G arrivals are in, the owner sums ITS columns over all n_shards rows in shard
//      order from +0.0 (own rows from `src`, the others from its slot) and applies
//      k_sgd_update's arithmetic to them (the same bits as the one-GPU update), publishes the
//      updated w and dw columns into every rank's publication slot of parity `par`, then one
//      arrival per block on every rank's publication counter;
//  (C) once P * G publication arrivals are in, the other owners' columns of w and dw are read
//      from this rank's publication slot.
// Per step a rank pushes rows_loc d (G-1)/G + 2 d (G-1)/G words instead of rows_loc d (G-1),
// and its update reads n_shards d / G slot words instead of n_shards d.  Counter and slot
// reuse: as k_peer_step's, for each of the two counter pairs (block 0 zeroes both of this
// rank's counters of the other parity; every arrival of step t+2 on them is ordered after this
// rank's step t+1, which waited for step t+1's publication of every rank).
struct PubSeg {
  unsigned long long* ctr[kPeerMax];  // rank p's publication counter of this parity
  double* slot[kPeerMax];             // rank p's publication slots [2][2][d]
  unsigned long long* my_ctr;
  const double* my_slot;
};

__device__ __forceinline__ int64_t col_begin(int p, int G, int64_t d) {
  return (int64_t)p * d / G;
}

__global__ __launch_bounds__(kBlock) void k_peer_step_cols(
    const double* __restrict__ src, int64_t rows, int64_t row0, PeerSeg ps, PubSeg pb, int rank,
    int par, unsigned long long* reset_g, unsigned long long* reset_p, uint64_t target,
    int n_shards, int64_t d, double* w, double* dw, double reg, double lr, double momentum,
    uint64_t* __restrict__ d_step, uint32_t* abort_word) {
  __shared__ double tile[kPUpdRows * kPUpdCols];
  __shared__ int s_ok;
  const int G = ps.G;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    __hip_atomic_store(reset_g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(reset_p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const size_t base = (size_t)par * ps.n_total + (size_t)row0 * d;
  // (A) per column owner: its columns of this rank's rows, into the owner's slot
  for (int p = 0; p < G; ++p) {
    if (p == rank) continue;
    const int64_t c0 = col_begin(p, G, d), nc = col_begin(p + 1, G, d) - c0;
    const int64_t words = rows * nc;
    double* dst = ps.slot[p] + base;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < words;
         i += (int64_t)gridDim.x * kBlock) {
      const int64_t r = i / nc, c = c0 + (i - r * nc);
      st_sys(dst + r * d + c, src[r * d + c]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if ((int)threadIdx.x < G)
    __hip_atomic_fetch_add(ps.ctr[threadIdx.x], 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  if (!peer_wait(ps.my_ctr, target, abort_word, &s_ok)) return;
  if (d_step && blockIdx.x == 0 && threadIdx.x == 0) *d_step += 1;
  // (B) this rank's columns: the shard-order sum, the update, the publication
  const int64_t m0 = col_begin(rank, G, d), m1 = col_begin(rank + 1, G, d);
  const double* slot = ps.my_slot + (size_t)par * ps.n_total;
  const int64_t lo = row0 * d, hi = (row0 + rows) * d;
  for (int64_t j0 = m0 + (int64_t)blockIdx.x * kPUpdCols; j0 < m1;
       j0 += (int64_t)gridDim.x * kPUpdCols) {
    const int nc = (int)std::min<int64_t>(kPUpdCols, m1 - j0);
    double sum = 0.0;
    for (int s0 = 0; s0 < n_shards; s0 += kPUpdRows) {
      const int ns = std::min(kPUpdRows, n_shards - s0);
      __syncthreads();
      for (int e = threadIdx.x; e < ns * kPUpdCols; e += kBlock) {
        const int r = e / kPUpdCols, c = e - r * kPUpdCols;
        const int64_t at = (int64_t)(s0 + r) * d + j0 + c;
        tile[e] = c >= nc ? 0.0 : (at >= lo && at < hi) ? src[at - lo] : ld_sys(slot + at);
      }
      __syncthreads();
      if ((int)threadIdx.x < nc) {
        int r = 0;
        for (; r + 8 <= ns; r += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = tile[(r + u) * kPUpdCols + threadIdx.x];
#pragma unroll
          for (int u = 0; u < 8; ++u) sum += v[u];
        }
        for (; r < ns; ++r) sum += tile[r * kPUpdCols + threadIdx.x];
      }
    }
    if ((int)threadIdx.x < nc) {
      const int64_t j = j0 + threadIdx.x;
      const double wj = w[j];
      const double g = sum / (double)n_shards + reg * wj;
      const double step = momentum >= 0.0 ? momentum * dw[j] + lr * g : lr * g;
      dw[j] = step;
      w[j] = wj - step;
      for (int p = 0; p < G; ++p) {
        if (p == rank) continue;
        double* pub = pb.slot[p] + (size_t)par * 2 * d;
        st_sys(pub + j, wj - step);
        st_sys(pub + d + j, step);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if ((int)threadIdx.x < G)
    __hip_atomic_fetch_add(pb.ctr[threadIdx.x], 1ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  // (C) the other owners' columns
  if (!peer_wait(pb.my_ctr, target, abort_word, &s_ok)) return;
  const double* pub = pb.my_slot + (size_t)par * 2 * d;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < d;
       j += (int64_t)gridDim.x * kBlock) {
    if (j >= m0 && j < m1) continue;
    w[j] = ld_sys(pub + j);
    dw[j] = ld_sys(pub + d + j);
  }
}

// setup handshake: lane p swaps this rank's token into rank p's hello word for this rank —
// a system-scope read-modify-write through the mapping, the kind of operation every step's
// arrivals are (a peer whose remote atomics do not land fails the check, and the ranks fall
// back to the all-gather)
__global__ void k_peer_hello(PeerSeg ps, int rank, unsigned long long token) {
  const int p = (int)threadIdx.x;
  if (p < ps.G) {
    auto* w = (unsigned long long*)((char*)ps.ctr[p] + kPeerHello) + rank;
    (void)__hip_atomic_exchange(w, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace tw

using namespace tw;

// Setup handshake of the peer mapping: every rank writes `token` into its slot of every rank's
// hello words (tw_peer_hello, then a host barrier over the ranks); tw_peer_check then reads its
// own buffer's G hello words and sets *ok = 1 when each holds `token` — the IPC mappings
// work and GPU stores through them land, before any step relies on them.
extern "C" int tw_peer_hello(void* const* d_peer_bases, int32_t G, int32_t rank, uint64_t token,
                             void* stream) {
  TW_ARG_CHECK(d_peer_bases != nullptr && G >= 1 && G <= kPeerMax && rank >= 0 && rank < G,
               "tw_peer_hello: bad ranks");
  PeerSeg ps{};
  for (int p = 0; p < G; ++p) {
    TW_ARG_CHECK(d_peer_bases[p] != nullptr, "tw_peer_hello: rank %d's buffer missing", p);
    ps.ctr[p] = (unsigned long long*)d_peer_bases[p];
  }
  ps.G = G;
  hipLaunchKernelGGL(k_peer_hello, dim3(1), dim3(64), 0, (hipStream_t)stream, ps, (int)rank,
                     (unsigned long long)token);
  TW_LAUNCH_CHECK();
  TW_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return TW_OK;
}

extern "C" int tw_peer_check(void* d_my_base, int32_t G, uint64_t token, int32_t* out_ok) {
  TW_ARG_CHECK(d_my_base != nullptr && G >= 1 && G <= kPeerMax && out_ok != nullptr,
               "tw_peer_check: bad arguments");
  uint64_t h[kPeerMax] = {0};
  TW_HIP_CHECK(hipMemcpy(h, (char*)d_my_base + kPeerHello, sizeof(uint64_t) * G,
                         hipMemcpyDeviceToHost));
  int ok = 1;
  for (int p = 0; p < G; ++p) ok &= h[p] == token ? 1 : 0;
  *out_ok = ok;
  return TW_OK;
}

// Column-owned per-step form (k_peer_step_cols): tw_peer_step's arguments and results (the
// same w / dw bits on every rank), with rank p updating only columns [p d / G, (p+1) d / G).
extern "C" int tw_peer_step_cols(const double* d_grads_loc, int64_t words, int64_t offset_words,
                                 void* const* d_peer_bases, int32_t G, int32_t rank,
                                 int32_t n_total, int64_t d, int32_t par, double* d_w,
                                 double* d_dw, double reg, double lr, double momentum,
                                 uint64_t* d_step, uint32_t* d_abort, void* stream) {
  TW_ARG_CHECK(d_peer_bases != nullptr && G >= 1 && G <= kPeerMax && rank >= 0 && rank < G &&
                   n_total >= 1 && d >= 1 && words >= 0 && offset_words >= 0 &&
                   offset_words + words <= (int64_t)n_total * d && (par == 0 || par == 1) &&
                   words % d == 0 && offset_words % d == 0,
               "tw_peer_step_cols: bad sizes");
  TW_ARG_CHECK(d_w && d_dw && d_abort, "tw_peer_step_cols: w, dw and the abort word required");
  PeerSeg ps{};
  PubSeg pb{};
  const size_t step_slots = kPeerHdr + sizeof(double) * peer_slots_words(n_total, d);
  const size_t pub_slots = step_slots + sizeof(double) * peer_slots_words(n_total, d);
  for (int p = 0; p < G; ++p) {
    char* b = (char*)d_peer_bases[p];
    TW_ARG_CHECK(b != nullptr, "tw_peer_step_cols: rank %d's buffer missing", p);
    ps.slot[p] = (double*)(b + step_slots);
    ps.ctr[p] = (unsigned long long*)(b + kPeerStepCtr + 64 * par);
    pb.ctr[p] = (unsigned long long*)(b + kPeerPubCtr + 64 * par);
    pb.slot[p] = (double*)(b + pub_slots);
  }
  char* mine = (char*)d_peer_bases[rank];
  ps.G = G;
  ps.n_total = (int)((int64_t)n_total * d);
  ps.my_ctr = (unsigned long long*)(mine + kPeerStepCtr + 64 * par);
  ps.my_slot = (const double*)(mine + step_slots);
  pb.my_ctr = (unsigned long long*)(mine + kPeerPubCtr + 64 * par);
  pb.my_slot = (const double*)(mine + pub_slots);
  auto* reset_g = (unsigned long long*)(mine + kPeerStepCtr + 64 * (1 - par));
  auto* reset_p = (unsigned long long*)(mine + kPeerPubCtr + 64 * (1 - par));
  const int P = step_blocks(d);  // the same on every rank: d is
  hipLaunchKernelGGL(k_peer_step_cols, dim3(P), dim3(kBlock), 0, (hipStream_t)stream,
                     d_grads_loc, words / d, offset_words / d, ps, pb, (int)rank, (int)par,
                     reset_g, reset_p, (uint64_t)P * (uint64_t)G, (int)n_total, d, d_w, d_dw,
                     reg, lr, momentum, d_step, d_abort);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int64_t tw_peer_buffer_bytes(int32_t n_total, int64_t d) {
  if (n_total < 1 || d < 1) return -1;
  return (int64_t)peer_buffer_bytes(n_total, d);
}

extern "C" int tw_peer_alloc(int64_t bytes, void** d_out, int32_t* out_uncached) {
  TW_ARG_CHECK(bytes > 0 && d_out != nullptr, "tw_peer_alloc: bytes > 0 and an output");
  void* p = nullptr;
  // Uncached or nothing: the hand-off relies on no device cache holding a slot or counter
  // line (peer.h), and a cached fallback would let an owner read stale gradient rows that the
  // hello handshake (one remote atomic) cannot detect.  Failing here makes every rank take
  // the RCCL all-gather together (learning.py _PeerBuffers.create).
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    set_error("tw_peer_alloc: uncached device memory is unavailable; the peer exchange needs it");
    return TW_ERR_HIP;
  }
  const int unc = 1;
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    set_error("tw_peer_alloc: zeroing the buffer failed");
    return TW_ERR_HIP;
  }
  *d_out = p;
  if (out_uncached) *out_uncached = unc;
  return TW_OK;
}

extern "C" int tw_peer_free(void* d_ptr) {
  if (d_ptr) TW_HIP_CHECK(hipFree(d_ptr));
  return TW_OK;
}

extern "C" int tw_peer_handle(void* d_ptr, uint8_t* out_handle) {
  TW_ARG_CHECK(d_ptr != nullptr && out_handle != nullptr, "tw_peer_handle: pointer and output");
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 bytes");
  hipIpcMemHandle_t h;
  TW_HIP_CHECK(hipIpcGetMemHandle(&h, d_ptr));
  std::memset(out_handle, 0, 64);
  std::memcpy(out_handle, &h, sizeof(h));
  return TW_OK;
}

extern "C" int tw_peer_open(const uint8_t* handle, void** d_out) {
  TW_ARG_CHECK(handle != nullptr && d_out != nullptr, "tw_peer_open: handle and output");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  TW_HIP_CHECK(hipIpcOpenMemHandle(d_out, h, hipIpcMemLazyEnablePeerAccess));
  return TW_OK;
}

extern "C" int tw_peer_close(void* d_ptr) {
  if (d_ptr) TW_HIP_CHECK(hipIpcCloseMemHandle(d_ptr));
  return TW_OK;
}

// per-step form, one launch after the gradient launch: this rank's `words` partial words
// (rows shard_base.. of the global order, d columns; offset_words = shard_base * d) into every
// rank's per-step slot of parity `par` with this launch's arrivals; then, once every rank's
// arrivals of that parity are in, k_sgd_update's arithmetic on this rank's slot
extern "C" int tw_peer_step(const double* d_grads_loc, int64_t words, int64_t offset_words,
                            void* const* d_peer_bases, int32_t G, int32_t rank, int32_t n_total,
                            int64_t d, int32_t par, double* d_w, double* d_dw, double reg,
                            double lr, double momentum, uint64_t* d_step, uint32_t* d_abort,
                            void* stream) {
  TW_ARG_CHECK(d_peer_bases != nullptr && G >= 1 && G <= kPeerMax && rank >= 0 && rank < G &&
                   n_total >= 1 && d >= 1 && words >= 0 && offset_words >= 0 &&
                   offset_words + words <= (int64_t)n_total * d && (par == 0 || par == 1),
               "tw_peer_step: bad sizes");
  TW_ARG_CHECK(d_w && d_dw && d_abort, "tw_peer_step: w, dw and the abort word required");
  PeerSeg ps{};
  const size_t step_slots = kPeerHdr + sizeof(double) * peer_slots_words(n_total, d);
  for (int p = 0; p < G; ++p) {
    char* b = (char*)d_peer_bases[p];
    TW_ARG_CHECK(b != nullptr, "tw_peer_step: rank %d's buffer missing", p);
    ps.slot[p] = (double*)(b + step_slots);
    ps.ctr[p] = (unsigned long long*)(b + kPeerStepCtr + 64 * par);
  }
  char* mine = (char*)d_peer_bases[rank];
  ps.G = G;
  ps.n_total = (int)((int64_t)n_total * d);  // one slot's words
  ps.my_ctr = (unsigned long long*)(mine + kPeerStepCtr + 64 * par);
  ps.my_slot = (const double*)(mine + step_slots);
  auto* reset = (unsigned long long*)(mine + kPeerStepCtr + 64 * (1 - par));
  const int P = step_blocks(d);  // the same on every rank: d is
  hipLaunchKernelGGL(k_peer_step, dim3(P), dim3(kBlock), 0, (hipStream_t)stream, d_grads_loc,
                     words, offset_words, ps, par, reset, (uint64_t)P * (uint64_t)G, n_total, d,
                     d_w, d_dw, reg, lr, momentum, d_step, d_abort);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
