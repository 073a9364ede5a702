// records.h — a sequence of est.UnNT repartitions kept as destination-bucketed records
// (tw_count_pairs_sorted_steps, csrc/rankcount.hip).
//
// A device repartition is a keyed bijection of positions (csrc/feistel.h).  Applied as a gather
// (nextstep.h, permute.hip) every element costs one random 8-B read: a whole 64-B line of HBM
// traffic, ~25 us for 2e6 scores whatever kernel carries it.  The sorted count does not need
// the scores in position order, only each shard's multiset — so across the T steps of one
// UnNT call the partition is kept as RECORDS {value, position} grouped by destination shard:
// the record slots of bucket s are exactly the position range [off[s], off[s+1]) of shard s
// (prop-SWOR shards have fixed sizes), so a count reads bucket s where it would have read
// shard s.  The next repartition is then a streaming pass over the records: each record's new
// position q = perm(p), its new bucket q / k, and a block-aggregated append into that bucket
// (one LDS histogram, one global cursor reservation per bucket and block, runs of ~100
// records per bucket and block).  Positions travel with the values; the arrays are written in
// position order once, after the last step.
#pragma once
#include "feistel.h"

namespace tw {

struct EmitStep {
  // current records (slot ranges = destination position ranges); pos == nullptr: implicit
  // (slot index = position, the arrays in position order)
  const uint64_t* xv;
  const uint32_t* xp;
  int64_t nx;
  const uint64_t* zv;
  const uint32_t* zp;
  int64_t nz;
  // next records and their bucket cursors (N + 1 each: the shards, then the tail that belongs
  // to no shard), zero on entry
  uint64_t* nxv;
  uint32_t* nxp;
  uint64_t* nzv;
  uint32_t* nzp;
  unsigned* cur_x;
  unsigned* cur_z;
  // cursors the NEXT launch appends with, zeroed here (may be null)
  unsigned* zero_x;
  unsigned* zero_z;
  Feistel fx, fz;
  FastDiv dx, dz;  // shard sizes kx, kz (divisor 1 when the size is 0)
  int64_t kx, kz;
  const int64_t* x_off;
  const int64_t* z_off;
  int n_shards;
  int active;
};

__device__ __forceinline__ int emit_bucket(uint64_t q, int64_t k, const FastDiv& d, int N) {
  if (k <= 0) return N;
  const uint64_t b = fast_div(q, d);
  return b < (uint64_t)N ? (int)b : N;
}

// Append the records of slots [a, b) of one sample to their next buckets.  Block-uniform
// bounds (the __syncthreads inside); hist / base: N + 1 LDS words each.
template <int BS, int EPR>
__device__ void emit_range(const uint64_t* __restrict__ v, const uint32_t* __restrict__ p,
                           int64_t a, int64_t b, int64_t n, const Feistel& F, int64_t k,
                           const FastDiv& dk, int N, const int64_t* __restrict__ off,
                           unsigned* __restrict__ cur, uint64_t* __restrict__ nv,
                           uint32_t* __restrict__ np, unsigned* hist, unsigned* base) {
  for (int64_t r0 = a; r0 < b; r0 += (int64_t)BS * EPR) {
    for (int i = threadIdx.x; i <= N; i += BS) hist[i] = 0;
    __syncthreads();
    uint64_t val[EPR];
    uint32_t q[EPR];
    int bk[EPR];
    unsigned slot[EPR];
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      const int64_t e = r0 + threadIdx.x + (int64_t)r * BS;
      bk[r] = -1;
      if (e < b) {
        val[r] = v[e];
        const uint64_t pos = p ? (uint64_t)p[e] : (uint64_t)e;
        q[r] = (uint32_t)feistel_perm(F, pos, (uint64_t)n);
        bk[r] = emit_bucket(q[r], k, dk, N);
      }
    }
#pragma unroll
    for (int r = 0; r < EPR; ++r)
      if (bk[r] >= 0) slot[r] = atomicAdd(&hist[bk[r]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i <= N; i += BS) base[i] = hist[i] ? atomicAdd(&cur[i], hist[i]) : 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < EPR; ++r) {
      if (bk[r] < 0) continue;
      const int64_t d = off[bk[r]] + (int64_t)base[bk[r]] + slot[r];
      nv[d] = val[r];
      np[d] = q[r];
    }
    __syncthreads();  // hist / base are reused by the next round
  }
}

// A block's stride of the tails [off[N], n) that belong to no shard (chunks of BS * 8 slots).
template <int BS>
__device__ void emit_tails(const EmitStep& em, int lb, int nblocks, unsigned* hist,
                           unsigned* base) {
  constexpr int EPR = 8;
  constexpr int64_t C = (int64_t)BS * EPR;
  const int N = em.n_shards;
  const int64_t tx = em.x_off[N], tz = em.z_off[N];
  for (int64_t c = tx + (int64_t)lb * C; c < em.nx; c += (int64_t)nblocks * C)
    emit_range<BS, EPR>(em.xv, em.xp, c, c + C < em.nx ? c + C : em.nx, em.nx, em.fx, em.kx,
                        em.dx, N, em.x_off, em.cur_x, em.nxv, em.nxp, hist, base);
  for (int64_t c = tz + (int64_t)lb * C; c < em.nz; c += (int64_t)nblocks * C)
    emit_range<BS, EPR>(em.zv, em.zp, c, c + C < em.nz ? c + C : em.nz, em.nz, em.fz, em.kz,
                        em.dz, N, em.z_off, em.cur_z, em.nzv, em.nzp, hist, base);
}

// Block-wide exclusive scan of n <= 2 * BS unsigned words in place (returns the total).
template <int BS>
__device__ unsigned block_scan_excl(unsigned* a, int n, unsigned* wave_tot) {
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const unsigned a0 = 2 * t < n ? a[2 * t] : 0u, a1 = 2 * t + 1 < n ? a[2 * t + 1] : 0u;
  unsigned v = a0 + a1, inc = v;
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wave_tot[w] = inc;
  __syncthreads();
  unsigned before = 0, total = 0;
  for (int i = 0; i < BS / kWave; ++i) {
    before += i < w ? wave_tot[i] : 0u;
    total += wave_tot[i];
  }
  const unsigned ex = before + inc - v;
  __syncthreads();  // every thread has read its inputs
  if (2 * t < n) a[2 * t] = ex;
  if (2 * t + 1 < n) a[2 * t + 1] = ex + a0;
  __syncthreads();
  return total;
}

// One block's share of the next repartition in ONE round, its stores coalesced: the X slots
// [xa, xb) and Z slots [za, zb) (together <= BS * 8) get their new positions and buckets (X
// buckets 0..N, Z buckets N+1..2N+1), an LDS histogram, one cursor reservation per bucket, and
// are staged in LDS ordered by bucket so that consecutive threads write consecutive slots of a
// bucket run.  LDS: hist/base/start 2N+2 words each, sv/sq/sb: BS * 8 staged records.
template <int BS>
__device__ void emit_block_staged(const EmitStep& em, int64_t xa, int64_t xb, int64_t za,
                                  int64_t zb, unsigned* hist, unsigned* base, unsigned* start,
                                  uint64_t* sv, uint32_t* sq, uint16_t* sb, unsigned* wave_tot) {
  constexpr int EPR = 8;
  const int N = em.n_shards, NB = 2 * N + 2;
  const int nxs = (int)(xb - xa), cnt = nxs + (int)(zb - za);
  for (int i = threadIdx.x; i < NB; i += BS) hist[i] = 0;
  __syncthreads();
  uint64_t val[EPR];
  uint32_t q[EPR];
  int bk[EPR];
  unsigned slot[EPR];
#pragma unroll
  for (int r = 0; r < EPR; ++r) {
    const int i = threadIdx.x + r * BS;
    bk[r] = -1;
    if (i < cnt) {
      const bool isx = i < nxs;
      const int64_t e = isx ? xa + i : za + (i - nxs);
      val[r] = isx ? em.xv[e] : em.zv[e];
      const uint32_t* pp = isx ? em.xp : em.zp;
      const uint64_t pos = pp ? (uint64_t)pp[e] : (uint64_t)e;
      q[r] = (uint32_t)(isx ? feistel_perm(em.fx, pos, (uint64_t)em.nx)
                            : feistel_perm(em.fz, pos, (uint64_t)em.nz));
      bk[r] = isx ? emit_bucket(q[r], em.kx, em.dx, N)
                  : N + 1 + emit_bucket(q[r], em.kz, em.dz, N);
    }
  }
#pragma unroll
  for (int r = 0; r < EPR; ++r)
    if (bk[r] >= 0) slot[r] = atomicAdd(&hist[bk[r]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < NB; i += BS) {
    const unsigned h = hist[i];
    unsigned* cur = i <= N ? em.cur_x + i : em.cur_z + (i - N - 1);
    base[i] = h ? atomicAdd(cur, h) : 0u;
    start[i] = h;
  }
  __syncthreads();
  block_scan_excl<BS>(start, NB, wave_tot);
#pragma unroll
  for (int r = 0; r < EPR; ++r) {
    if (bk[r] < 0) continue;
    const unsigned j = start[bk[r]] + slot[r];
    sv[j] = val[r];
    sq[j] = q[r];
    sb[j] = (uint16_t)bk[r];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < cnt; j += BS) {
    const int b = sb[j];
    const bool isx = b <= N;
    const int bb = isx ? b : b - N - 1;
    const int64_t d = (isx ? em.x_off[bb] : em.z_off[bb]) + (int64_t)base[b] + (j - start[b]);
    if (isx) {
      em.nxv[d] = sv[j];
      em.nxp[d] = sq[j];
    } else {
      em.nzv[d] = sv[j];
      em.nzp[d] = sq[j];
    }
  }
  __syncthreads();
}

}  // namespace tw
