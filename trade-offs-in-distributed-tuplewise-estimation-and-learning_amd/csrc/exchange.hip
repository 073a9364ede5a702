// exchange.hip — row exchange for the row-partitioned learning layout.
//
// The reference re-draws the learning shards with SWR_divide (compute_stats.py:48-54): N
// shards of int(n/N) rows drawn with replacement, returned as copies.  With X replicated on
// every GPU a reshuffle is only new index arrays.  With X row-partitioned (rank r keeps rows
// [lo_r, hi_r), 1/G of the memory) the drawn rows must travel: every rank knows all N shards'
// draws (the replay draw is global; device Philox draws are keyed by the global shard id), so
// each owner can work out, without any request round, which of its rows each requester needs.
//
//   tw_row_route_counts  per requester q: how many of q's positions this rank owns
//   tw_row_pack          records {row (d doubles), destination position (bit-cast)} grouped
//                        by requester, ready for one all_to_all
//   tw_row_unpack        scatter received records into the requester's shard-local matrix
//
// Positions are global over the shard-major draw array (p = s*k + j for shard s, draw j);
// requester q owns positions [q*M_q, (q+1)*M_q).  A block handles a contiguous chunk of
// positions, so it touches one or two requesters: LDS counters per requester, one global
// reservation per (block, requester), then lane groups copy the rows (coalesced along d).
// The order of records inside a requester's bucket depends on block scheduling, but every
// record carries its position, so the unpacked matrix is deterministic.
//
// Remote rows only (the default; tw_row_*_remote): a rank reads the rows it owns straight from
// its partition, so only rows owned elsewhere travel, and they stay where they land.  The
// rank's matrix is [partition | receive area]: bucket q of a send buffer holds c_q rows
// (d doubles each) followed by their c_q destination positions, padded to whole rows, so that
// after the all_to_all every received row starts on a row boundary of the matrix; the row
// tables then point at partition rows (owned) or receive-area rows (remote) — no unpack pass,
// and at G = 1 no exchange at all.
#include "tw_common.h"

namespace tw {

constexpr int kChunk = 1024;  // positions per block (4 per thread)
constexpr int kMaxRanks = 1024;

__global__ __launch_bounds__(kBlock) void k_route_counts(const int64_t* __restrict__ rows,
                                                         int64_t M, int64_t M_q, int64_t lo,
                                                         int64_t hi, int G,
                                                         unsigned long long* __restrict__ counts) {
  __shared__ int lcnt[kMaxRanks];
  for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += kBlock) {
    const int64_t p = c0 + i;
    if (p < M) {
      const int64_t row = rows[p];
      if (row >= lo && row < hi) atomicAdd(&lcnt[(int)(p / M_q)], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (lcnt[i]) atomicAdd(&counts[i], (unsigned long long)lcnt[i]);
}

__global__ __launch_bounds__(kBlock) void k_row_pack(
    const int64_t* __restrict__ rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi, int G,
    const double* __restrict__ part, int64_t d, const int64_t* __restrict__ start,
    unsigned long long* __restrict__ cursor, double* __restrict__ send, int lanes) {
  __shared__ int lcnt[kMaxRanks];
  __shared__ int64_t lbase[kMaxRanks];
  __shared__ int e_off[kChunk];   // chunk-local position
  __shared__ int e_rank[kChunk];  // rank of the entry inside its requester's block slice
  __shared__ int n_ent;
  for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
  if (threadIdx.x == 0) n_ent = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += kBlock) {
    const int64_t p = c0 + i;
    if (p < M) {
      const int64_t row = rows[p];
      if (row >= lo && row < hi) {
        const int k = atomicAdd(&n_ent, 1);
        e_off[k] = i;
        e_rank[k] = atomicAdd(&lcnt[(int)(p / M_q)], 1);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (lcnt[i]) lbase[i] = start[i] + (int64_t)atomicAdd(&cursor[i], (unsigned long long)lcnt[i]);
  __syncthreads();
  const int groups = kBlock / lanes;
  const int g = threadIdx.x / lanes, l = threadIdx.x % lanes;
  const int n = n_ent;
  for (int k = g; k < n; k += groups) {
    const int64_t p = c0 + e_off[k];
    const int q = (int)(p / M_q);
    const int64_t slot = lbase[q] + e_rank[k];
    const double* src = part + (rows[p] - lo) * d;
    double* dst = send + slot * (d + 1);
    for (int64_t c = l; c < d; c += lanes) dst[c] = src[c];
    if (l == 0) dst[d] = __longlong_as_double((long long)(p - (int64_t)q * M_q));
  }
}

__global__ __launch_bounds__(kBlock) void k_row_unpack(const double* __restrict__ rec, int64_t m,
                                                       int64_t d, double* __restrict__ out,
                                                       int lanes) {
  const int groups = kBlock / lanes;
  const int l = threadIdx.x % lanes;
  for (int64_t i = (int64_t)blockIdx.x * groups + threadIdx.x / lanes; i < m;
       i += (int64_t)gridDim.x * groups) {
    const double* r = rec + i * (d + 1);
    const int64_t pos = (int64_t)__double_as_longlong(r[d]);
    double* dst = out + pos * d;
    for (int64_t c = l; c < d; c += lanes) dst[c] = r[c];
  }
}


__global__ __launch_bounds__(kBlock) void k_row_pack_remote(
    const int64_t* __restrict__ rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi, int G,
    int me, const double* __restrict__ part, int64_t d, const int64_t* __restrict__ start,
    const int64_t* __restrict__ count, unsigned long long* __restrict__ cursor,
    double* __restrict__ send, int lanes) {
  __shared__ int lcnt[kMaxRanks];
  __shared__ int64_t lbase[kMaxRanks];
  __shared__ int e_off[kChunk];
  __shared__ int e_rank[kChunk];
  __shared__ int n_ent;
  for (int i = threadIdx.x; i < G; i += kBlock) lcnt[i] = 0;
  if (threadIdx.x == 0) n_ent = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += kBlock) {
    const int64_t p = c0 + i;
    if (p < M) {
      const int64_t row = rows[p];
      const int q = (int)(p / M_q);
      if (q != me && row >= lo && row < hi) {
        const int k = atomicAdd(&n_ent, 1);
        e_off[k] = i;
        e_rank[k] = atomicAdd(&lcnt[q], 1);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G; i += kBlock)
    if (lcnt[i]) lbase[i] = (int64_t)atomicAdd(&cursor[i], (unsigned long long)lcnt[i]);
  __syncthreads();
  const int groups = kBlock / lanes;
  const int g = threadIdx.x / lanes, l = threadIdx.x % lanes;
  const int n = n_ent;
  for (int k = g; k < n; k += groups) {
    const int64_t p = c0 + e_off[k];
    const int q = (int)(p / M_q);
    const int64_t slot = lbase[q] + e_rank[k];
    const double* src = part + (rows[p] - lo) * d;
    double* bucket = send + start[q];
    double* dst = bucket + slot * d;
    for (int64_t c = l; c < d; c += lanes) dst[c] = src[c];
    if (l == 0)
      bucket[count[q] * d + slot] = __longlong_as_double((long long)(p - (int64_t)q * M_q));
  }
}

// this rank's positions [me * M_q, (me + 1) * M_q): the partition row of an owned draw
__global__ __launch_bounds__(kBlock) void k_row_table_local(const int64_t* __restrict__ rows,
                                                            int64_t M_q, int64_t lo, int64_t hi,
                                                            int64_t* __restrict__ table) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < M_q;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t row = rows[i];
    table[i] = (row >= lo && row < hi) ? row - lo : -1;
  }
}

// received rows: record j of source g sits at row (base + rstart[g] / d + j) of the matrix;
// a position outside the table (a protocol error) is not written and raises *bad
__global__ __launch_bounds__(kBlock) void k_row_table_remote(
    const double* __restrict__ recv, int G, const int64_t* __restrict__ rstart,
    const int64_t* __restrict__ rcount, const int64_t* __restrict__ rprefix, int64_t total,
    int64_t d, int64_t base, int64_t* __restrict__ table, int64_t table_len, int64_t recv_len,
    int64_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    int a = 0, b = G;  // the last g with rprefix[g] <= i
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (rprefix[m] <= i) a = m; else b = m;
    }
    const int64_t j = i - rprefix[a];
    const int64_t at = rstart[a] + rcount[a] * d + j;
    if (at < 0 || at >= recv_len) {  // the split sizes disagree with the counts
      if (bad) atomicMax((unsigned long long*)bad, 1ull << 62);
      continue;
    }
    const int64_t pos = (int64_t)__double_as_longlong(recv[at]);
    if (pos < 0 || pos >= table_len) {
      if (bad) atomicMax((unsigned long long*)bad, (unsigned long long)(pos + 1 > 0 ? pos + 1 : 1));
      continue;
    }
    table[pos] = base + rstart[a] / d + j;
  }
}

static int lanes_for(int64_t d) {
  int l = 1;
  while (l < 64 && l < d) l <<= 1;
  return l;
}

}  // namespace tw

using namespace tw;

extern "C" int tw_row_route_counts(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo,
                                   int64_t hi, int32_t G, int64_t* d_counts, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxRanks, "tw_row_route_counts: G=%d outside [1, %d]", G,
               kMaxRanks);
  TW_ARG_CHECK(M >= 0 && M_q >= 1 && M <= M_q * (int64_t)G,
               "tw_row_route_counts: M=%lld positions do not fit G=%d requesters of %lld",
               (long long)M, G, (long long)M_q);
  TW_ARG_CHECK(lo >= 0 && hi >= lo, "tw_row_route_counts: bad owned range [%lld, %lld)",
               (long long)lo, (long long)hi);
  TW_ARG_CHECK(d_counts != nullptr && (M == 0 || d_rows != nullptr),
               "tw_row_route_counts: null pointer");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_counts, 0, sizeof(int64_t) * G, st));
  if (M == 0) return TW_OK;
  hipLaunchKernelGGL(k_route_counts, dim3((unsigned)ceil_div(M, kChunk)), dim3(kBlock), 0, st,
                     d_rows, M, M_q, lo, hi, (int)G, (unsigned long long*)d_counts);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_row_pack(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo, int64_t hi,
                           int32_t G, const double* d_part, int64_t d, const int64_t* d_start,
                           int64_t* d_cursor, double* d_send, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxRanks, "tw_row_pack: G=%d outside [1, %d]", G, kMaxRanks);
  TW_ARG_CHECK(M >= 0 && M_q >= 1 && M <= M_q * (int64_t)G && d >= 1,
               "tw_row_pack: bad sizes M=%lld M_q=%lld d=%lld", (long long)M, (long long)M_q,
               (long long)d);
  TW_ARG_CHECK(lo >= 0 && hi >= lo, "tw_row_pack: bad owned range");
  TW_ARG_CHECK(d_start != nullptr && d_cursor != nullptr, "tw_row_pack: null pointer");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_cursor, 0, sizeof(int64_t) * G, st));
  if (M == 0 || hi == lo) return TW_OK;
  TW_ARG_CHECK(d_rows && d_part && d_send, "tw_row_pack: null pointer");
  hipLaunchKernelGGL(k_row_pack, dim3((unsigned)ceil_div(M, kChunk)), dim3(kBlock), 0, st,
                     d_rows, M, M_q, lo, hi, (int)G, d_part, d, d_start,
                     (unsigned long long*)d_cursor, d_send, lanes_for(d));
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_row_unpack(const double* d_rec, int64_t m, int64_t d, double* d_out,
                             void* stream) {
  TW_ARG_CHECK(m >= 0 && d >= 1, "tw_row_unpack: bad sizes m=%lld d=%lld", (long long)m,
               (long long)d);
  if (m == 0) return TW_OK;
  TW_ARG_CHECK(d_rec && d_out, "tw_row_unpack: null pointer");
  const int lanes = lanes_for(d);
  const int64_t groups = kBlock / lanes;
  const int64_t blocks = std::min<int64_t>(ceil_div(m, groups), 256 * 64);
  hipLaunchKernelGGL(k_row_unpack, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)stream,
                     d_rec, m, d, d_out, lanes);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_row_route_remote_counts(const int64_t* d_rows, int64_t M, int64_t M_q,
                                          int64_t lo, int64_t hi, int32_t G, int32_t me,
                                          int64_t* d_counts, void* stream) {
  TW_ARG_CHECK(me >= 0 && me < G, "tw_row_route_remote_counts: rank %d outside [0, %d)", me, G);
  const int rc = tw_row_route_counts(d_rows, M, M_q, lo, hi, G, d_counts, stream);
  if (rc) return rc;
  TW_HIP_CHECK(tw_zero_async(d_counts + me, 0, sizeof(int64_t), (hipStream_t)stream));
  return TW_OK;
}

extern "C" int tw_row_pack_remote(const int64_t* d_rows, int64_t M, int64_t M_q, int64_t lo,
                                  int64_t hi, int32_t G, int32_t me, const double* d_part,
                                  int64_t d, const int64_t* d_start, const int64_t* d_count,
                                  int64_t* d_cursor, double* d_send, void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxRanks && me >= 0 && me < G,
               "tw_row_pack_remote: G=%d, rank %d", G, me);
  TW_ARG_CHECK(M >= 0 && M_q >= 1 && M <= M_q * (int64_t)G && d >= 1,
               "tw_row_pack_remote: bad sizes M=%lld M_q=%lld d=%lld", (long long)M,
               (long long)M_q, (long long)d);
  TW_ARG_CHECK(lo >= 0 && hi >= lo, "tw_row_pack_remote: bad owned range");
  TW_ARG_CHECK(d_start && d_count && d_cursor, "tw_row_pack_remote: null pointer");
  hipStream_t st = (hipStream_t)stream;
  TW_HIP_CHECK(tw_zero_async(d_cursor, 0, sizeof(int64_t) * G, st));
  if (M == 0 || hi == lo || G == 1) return TW_OK;
  TW_ARG_CHECK(d_rows && d_part && d_send, "tw_row_pack_remote: null pointer");
  hipLaunchKernelGGL(k_row_pack_remote, dim3((unsigned)ceil_div(M, kChunk)), dim3(kBlock), 0, st,
                     d_rows, M, M_q, lo, hi, (int)G, (int)me, d_part, d, d_start, d_count,
                     (unsigned long long*)d_cursor, d_send, lanes_for(d));
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_row_table_local(const int64_t* d_rows, int64_t M_q, int64_t lo, int64_t hi,
                                  int64_t* d_table, void* stream) {
  TW_ARG_CHECK(M_q >= 0 && lo >= 0 && hi >= lo, "tw_row_table_local: bad sizes");
  if (M_q == 0) return TW_OK;
  TW_ARG_CHECK(d_rows && d_table, "tw_row_table_local: null pointer");
  const int64_t blocks = std::min<int64_t>(ceil_div(M_q, kBlock), 4096);
  hipLaunchKernelGGL(k_row_table_local, dim3((unsigned)blocks), dim3(kBlock), 0,
                     (hipStream_t)stream, d_rows, M_q, lo, hi, d_table);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_row_table_remote(const double* d_recv, int32_t G, const int64_t* d_rstart,
                                   const int64_t* d_rcount, const int64_t* d_rprefix,
                                   int64_t total, int64_t d, int64_t base, int64_t* d_table,
                                   int64_t table_len, int64_t recv_len, int64_t* d_bad,
                                   void* stream) {
  TW_ARG_CHECK(G >= 1 && G <= kMaxRanks && total >= 0 && d >= 1 && base >= 0 &&
                   table_len >= 0,
               "tw_row_table_remote: bad sizes");
  if (total == 0) return TW_OK;
  TW_ARG_CHECK(d_recv && d_rstart && d_rcount && d_rprefix && d_table,
               "tw_row_table_remote: null pointer");
  const int64_t blocks = std::min<int64_t>(ceil_div(total, kBlock), 4096);
  hipLaunchKernelGGL(k_row_table_remote, dim3((unsigned)blocks), dim3(kBlock), 0,
                     (hipStream_t)stream, d_recv, (int)G, d_rstart, d_rcount, d_rprefix, total,
                     d, base, d_table, table_len, recv_len, d_bad);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
