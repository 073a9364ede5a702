// rankimage.hip — the all-pairs count of est.UnN on packed-f32 RANK IMAGES (SURVEY.md §8 rows
// A1/A6/A7; round 3).
//
// Reference: est.Un   estimation-experiment/main.py:29-31   mean(X[:,None] > Z[None,:])
//            est.UnN / UnNT   estimation-experiment/main.py:72-79 (the repartition loop)
//
// Why images.  csrc/count.hip compares the doubles themselves: one v_cmp_f64 per 64 pairs plus
// the count of its 64 result bits (a carry-add on the VALU or s_bcnt1 + s_add on the scalar
// unit) — an instruction mix whose issue ceiling is ~0.63 of the lane-op peak (DESIGN.md
// §4.1).  Packed f32 VALU ops (v_pk_*_f32, full rate on gfx950) process TWO lanes' worth per
// instruction, and with integer-valued operands a compare-and-count is two of them:
//     t   = clamp(gx + nz)           v_pk_add_f32 ... clamp   (nz = -gz from an SGPR)
//     acc = acc + t                  v_pk_add_f32
// where clamp(gx - gz) is exactly 1 when gx - gz >= 1 and 0 when gx - gz <= 0.  That is 1 VALU
// wave-instruction per 64 pairs and nothing on the scalar unit (tools/mb_pk.hip: 0.88 of the
// lane-op peak on the bench shape, profiles/r03_mb_pk.log).
//
// The images.  Over ONE call (est.UnNT's T repartitions) the multiset of scores does not change,
// only which shard holds which score.  So the images are computed once per call from the whole
// sample: sort X ∪ Z by the order key (NaN last, -0 == +0), stably, every x before every z (the
// input order), and give every element the number of z-elements sorted before it:
//     gx(x_i) = #{z : key(z) < key(x_i)}   (equal z come after x: never counted)
//     gz(z_j) = #{z before z_j in the sort} (equal z get distinct consecutive values)
// Then for any x, z:  x > z  <=>  gx > gz  <=>  gx - gz >= 1.  (key(x) > key(z): every z with
// key <= key(z) — z itself included — precedes x, so gx >= gz + 1.  key(x) <= key(z): the z
// counted in gx all precede z, so gx <= gz.)  NaN x get -2^25 (never greater); a NaN z sorts
// after every non-NaN x, so gz >= gx of every such x (never less).  Images are integers
// <= m < 2^24, so every f32 sum gx - gz is exact; sentinels are exact powers of two and keep
// their sign.  Per pair the count is the reference's integer, bit for bit.
//
// State between steps.  An element is an 8-B record: low word = its f32 image, high word = its
// index in the call's input array.  The repartition permutes records exactly as it permuted
// doubles (nextstep.h: the next step's gather rides on the tail blocks of the count launch, the
// same 8 B per element), and at the end of the call one gather writes the doubles in the final
// order (tw_gather_records).
//
// Sort and scan: rocPRIM's device radix sort (stable LSD, 64-bit keys) and lookback scan, once
// per call; the per-step kernel below is the hot path.
#include "nextstep.h"
#include "sortkeys.h"
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

namespace tw {

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr float kImgNever = -33554432.0f;  // -2^25: NaN x and padded lanes, never greater

// ----------------------------------------------------------------------------- images
template <typename T>
__global__ __launch_bounds__(kBlock) void k_rank_keys(const T* __restrict__ x, int64_t n,
                                                      const T* __restrict__ z, int64_t m,
                                                      uint64_t* __restrict__ keys,
                                                      uint32_t* __restrict__ ids) {
  const int64_t tot = n + m;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * kBlock) {
    keys[i] = order_key<T>(i < n ? x[i] : z[i - n]);
    ids[i] = (uint32_t)i;  // x first: the stable sort keeps every x before an equal z
  }
}

struct IsZ {
  uint32_t n;
  __host__ __device__ uint32_t operator()(uint32_t id) const { return id >= n ? 1u : 0u; }
};

// records: x_rec[i] = (image bits | i << 32), z_rec[j] = (-image bits | j << 32)
__global__ __launch_bounds__(kBlock) void k_rank_records(const uint64_t* __restrict__ keys_s,
                                                         const uint32_t* __restrict__ ids_s,
                                                         const uint32_t* __restrict__ cz,
                                                         int64_t n, int64_t tot, bool x_nan_key,
                                                         uint64_t* __restrict__ x_rec,
                                                         uint64_t* __restrict__ z_rec) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < tot;
       p += (int64_t)gridDim.x * kBlock) {
    const uint32_t id = ids_s[p];
    const float g = (float)cz[p];  // exact: cz <= m < 2^24
    if ((int64_t)id < n) {
      const float img = (x_nan_key && keys_s[p] == ~0ull) ? kImgNever : g;
      x_rec[id] = (uint64_t)__float_as_uint(img) | ((uint64_t)id << 32);
    } else {
      const uint32_t j = id - (uint32_t)n;
      z_rec[j] = (uint64_t)__float_as_uint(-g) | ((uint64_t)j << 32);
    }
  }
}

struct RankWork {
  uint64_t *keys_in, *keys_out;
  uint32_t *ids_in, *ids_out, *cz;
  void* temp;
  size_t temp_bytes;
  size_t total;
};

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

static int rank_work(int64_t n, int64_t m, char* base, RankWork* w) {
  const int64_t tot = n + m;
  size_t sort_b = 0, scan_b = 0;
  TW_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, sort_b, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)tot, 0,
                                         64));
  auto flags = rocprim::make_transform_iterator((const uint32_t*)nullptr, IsZ{(uint32_t)n});
  TW_HIP_CHECK(rocprim::exclusive_scan(nullptr, scan_b, flags, (uint32_t*)nullptr, 0u,
                                       (size_t)tot, rocprim::plus<uint32_t>()));
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align256(bytes);
    return base ? (void*)(base + o) : nullptr;
  };
  w->keys_in = (uint64_t*)take(8 * (size_t)tot);
  w->keys_out = (uint64_t*)take(8 * (size_t)tot);
  w->ids_in = (uint32_t*)take(4 * (size_t)tot);
  w->ids_out = (uint32_t*)take(4 * (size_t)tot);
  w->cz = (uint32_t*)take(4 * (size_t)tot);
  w->temp_bytes = std::max(sort_b, scan_b);
  w->temp = take(w->temp_bytes);
  w->total = off;
  return TW_OK;
}

static bool rank_sizes_ok(int64_t n, int64_t m) {
  // images are exact integers while m < 2^24; ids fit 32 bits
  return n >= 0 && m >= 0 && m < (1ll << 24) && n + m < (1ll << 31);
}

// ----------------------------------------------------------------------------- the count
// nz2: an SGPR pair holding one z record; both packed halves take its LOW word (the negated
// image): t = clamp(x_lo + nz, x_hi + nz).
__device__ __forceinline__ f2 gt_clamp(f2 x, uint64_t nz2) {
  f2 t;
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] clamp" : "=v"(t) : "v"(x), "s"(nz2));
  return t;
}
__device__ __forceinline__ void acc_add(f2& a, f2 t) {
  asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(t));
}

__device__ __forceinline__ float rec_image(uint64_t r) { return __uint_as_float((uint32_t)r); }

// One wave item: 64*R x-images (R per lane as R/2 packed pairs) against z records [z0, z1).
template <int R>
__device__ __forceinline__ unsigned long long count_rank_item(const uint64_t* __restrict__ xr,
                                                              int64_t x0, int64_t xe,
                                                              const uint64_t* __restrict__ zr,
                                                              int64_t z0, int64_t z1, int lane) {
  constexpr int P = R / 2;
  f2 xv[P], acc[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int64_t i0 = x0 + (2 * p) * kWave + lane, i1 = i0 + kWave;
    xv[p].x = i0 < xe ? rec_image(xr[i0]) : kImgNever;  // padded lanes: never greater
    xv[p].y = i1 < xe ? rec_image(xr[i1]) : kImgNever;
    acc[p] = f2{0.f, 0.f};
  }
  // all compares of one z first, then the accumulations: no adjacent dependent pair
  auto one_z = [&](uint64_t zu) {
    f2 t[P];
#pragma unroll
    for (int p = 0; p < P; ++p) t[p] = gt_clamp(xv[p], zu);
#pragma unroll
    for (int p = 0; p < P; ++p) acc_add(acc[p], t[p]);
  };
  const uint64_t* __restrict__ zp = zr + z0;
  const int nz = (int)(z1 - z0);
  int j = 0;
  // 8 records per s_load_dwordx16; the next group's loads are in flight while one is compared
  // (two register buffers, loads past the chunk clamped to its last full group)
  if (nz >= 16) {
    uint64_t za[8], zb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) za[u] = zp[u];
    const int last = nz - 8;
    for (; j + 16 <= nz; j += 16) {
      const uint64_t* qb = zp + j + 8;
#pragma unroll
      for (int u = 0; u < 8; ++u) zb[u] = qb[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) one_z(za[u]);
      const uint64_t* qa = zp + (j + 16 <= last ? j + 16 : last);
#pragma unroll
      for (int u = 0; u < 8; ++u) za[u] = qa[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) one_z(zb[u]);
    }
  }
  for (; j + 8 <= nz; j += 8) {
    uint64_t zv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) zv[u] = zp[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) one_z(zv[u]);
  }
  for (; j < nz; ++j) one_z(zp[j]);
  unsigned long long tot = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) tot += (unsigned)acc[p].x + (unsigned)acc[p].y;  // exact < 2^24
  return wave_sum_u64(tot);
}

// Same work decomposition and epilogue as k_count_complete (csrc/count.hip): per-wave items
// (shard, x tile, z chunk), XCD-aware block order, one u64 atomic per block and shard; the
// last nxt.blocks blocks carry the next repartition (nextstep.h) on the records.
template <int R>
__global__ __launch_bounds__(kBlock) void k_count_rank(
    const uint64_t* __restrict__ xr, const int64_t* __restrict__ x_off,
    const uint64_t* __restrict__ zr, const int64_t* __restrict__ z_off, int n_shards,
    int tiles_x, int zchunks, int64_t z_chunk, unsigned long long* __restrict__ out,
    NextStep nxt) {
  if (nxt.blocks && (int)blockIdx.x >= (int)gridDim.x - nxt.blocks) {
    next_step_part<kBlock>(nxt, (int)blockIdx.x - ((int)gridDim.x - nxt.blocks));
    return;
  }
  const int per_shard = tiles_x * zchunks;
  const int lb = xcd_block(blockIdx.x, gridDim.x - nxt.blocks);  // whole shards per XCD
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int item = lb * (kBlock / kWave) + wid;
  const int s = item / per_shard;
  bool active = s < n_shards;
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
    active = x0 < xe && z0 < ze;
  }
  unsigned long long tot = 0;
  if (active) tot = count_rank_item<R>(xr, x0, xe, zr, z0, z1, lane);
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

// Final order of the doubles: out[p] = in[rec[p] >> 32]
__global__ __launch_bounds__(kBlock) void k_gather_records(const uint64_t* __restrict__ in,
                                                           const uint64_t* __restrict__ rec,
                                                           int64_t n, uint64_t* __restrict__ out) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * kBlock)
    out[p] = in[rec[p] >> 32];
}

// ----------------------------------------------------------------------------- plan
struct RankPlan {
  int R, tiles_x, zchunks;
  int64_t z_chunk, blocks;
};
static int g_rank_R = 0;          // tuning hooks (tw_count_rank_set_plan); 0 = automatic
static int64_t g_rank_zchunk = 0;

// R in {16, 8}: least padded x-slots (ties to 16: half the z loads per compare); z chunks of
// ~1024 records (tools/mb_pk.hip: 528 is too short for R = 8, >= 2048 leaves the tail ragged).
static RankPlan plan_rank(int64_t max_nx, int64_t max_nz, int32_t n_shards) {
  RankPlan p{16, 1, 1, max_nz, 0};
  int64_t best = -1;
  for (int R : {16, 8}) {
    if (g_rank_R && R != g_rank_R) continue;
    const int64_t slots = ceil_div(max_nx, (int64_t)kWave * R) * kWave * R;
    if (best < 0 || slots < best) {
      best = slots;
      p.R = R;
    }
  }
  p.tiles_x = (int)ceil_div(max_nx, (int64_t)kWave * p.R);
  int64_t zc = g_rank_zchunk > 0 ? g_rank_zchunk : 1024;
  // enough work items to fill the chip when shards are few / short
  const int64_t target = 256 * 16 * (kBlock / kWave);
  const int64_t base = (int64_t)p.tiles_x * n_shards;
  if (g_rank_zchunk <= 0 && base * ceil_div(max_nz, zc) < target)
    zc = std::max<int64_t>(256, ceil_div(max_nz, std::max<int64_t>(1, target / base)));
  zc = std::min<int64_t>(zc, (int64_t)1 << 24);  // f32 lane counters stay exact
  p.z_chunk = ceil_div(std::min<int64_t>(zc, max_nz), 8) * 8;
  p.zchunks = (int)ceil_div(max_nz, p.z_chunk);
  p.blocks = ceil_div((int64_t)p.tiles_x * p.zchunks * n_shards, kBlock / kWave);
  return p;
}

static int next_rank_blocks(int64_t elems) {
  int64_t b = ceil_div(elems, (int64_t)kBlock * 8);
  b = std::min<int64_t>(std::max<int64_t>(b, 8), 512);
  return (int)(ceil_div(b, kXcds) * kXcds);
}

}  // namespace tw

using namespace tw;

extern "C" int64_t tw_rank_images_work_bytes(int64_t n_x, int64_t n_z) {
  if (!rank_sizes_ok(n_x, n_z)) return -1;
  RankWork w{};
  if (rank_work(n_x, n_z, nullptr, &w) != TW_OK) return -1;
  return (int64_t)w.total;
}

extern "C" int tw_rank_images(const void* d_x, int64_t n_x, const void* d_z, int64_t n_z,
                              int32_t dtype, void* d_work, int64_t work_bytes, uint64_t* d_x_rec,
                              uint64_t* d_z_rec, void* stream) {
  TW_ARG_CHECK(rank_sizes_ok(n_x, n_z),
               "tw_rank_images: needs n_z < 2^24 and n_x + n_z < 2^31 (got %lld, %lld)",
               (long long)n_x, (long long)n_z);
  TW_ARG_CHECK(dtype == TW_F64 || dtype == TW_I64, "tw_rank_images: unknown dtype %d", dtype);
  hipStream_t st = (hipStream_t)stream;
  const int64_t tot = n_x + n_z;
  if (tot == 0) return TW_OK;
  RankWork w{};
  if (rank_work(n_x, n_z, (char*)d_work, &w) != TW_OK) return TW_ERR_HIP;
  TW_ARG_CHECK(d_work != nullptr && work_bytes >= (int64_t)w.total,
               "tw_rank_images: work buffer of %lld bytes, %lld needed", (long long)work_bytes,
               (long long)w.total);
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(tot, kBlock));
  if (dtype == TW_F64)
    hipLaunchKernelGGL(k_rank_keys<double>, dim3(grid), dim3(kBlock), 0, st, (const double*)d_x,
                       n_x, (const double*)d_z, n_z, w.keys_in, w.ids_in);
  else
    hipLaunchKernelGGL(k_rank_keys<long long>, dim3(grid), dim3(kBlock), 0, st,
                       (const long long*)d_x, n_x, (const long long*)d_z, n_z, w.keys_in,
                       w.ids_in);
  TW_LAUNCH_CHECK();
  size_t tb = w.temp_bytes;
  TW_HIP_CHECK(rocprim::radix_sort_pairs(w.temp, tb, w.keys_in, w.keys_out, w.ids_in, w.ids_out,
                                         (size_t)tot, 0, 64, st));
  tb = w.temp_bytes;
  auto flags = rocprim::make_transform_iterator((const uint32_t*)w.ids_out,
                                                IsZ{(uint32_t)n_x});
  TW_HIP_CHECK(rocprim::exclusive_scan(w.temp, tb, flags, w.cz, 0u, (size_t)tot,
                                       rocprim::plus<uint32_t>(), st));
  hipLaunchKernelGGL(k_rank_records, dim3(grid), dim3(kBlock), 0, st, w.keys_out, w.ids_out,
                     w.cz, n_x, tot, dtype == TW_F64, d_x_rec, d_z_rec);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_count_rank_set_plan(int32_t R, int64_t z_chunk) {
  TW_ARG_CHECK(R == 0 || R == 8 || R == 16, "tw_count_rank_set_plan: R in {0, 8, 16}");
  TW_ARG_CHECK(z_chunk >= 0 && z_chunk <= (1ll << 24), "tw_count_rank_set_plan: bad z_chunk");
  g_rank_R = R;
  g_rank_zchunk = z_chunk;
  return TW_OK;
}

extern "C" int tw_count_pairs_rank_step(const uint64_t* d_x_rec, const int64_t* d_x_off,
                                        const uint64_t* d_z_rec, const int64_t* d_z_off,
                                        int32_t n_shards, int64_t max_nx, int64_t max_nz,
                                        uint64_t* d_out, int64_t n_x, uint64_t* d_x_next,
                                        uint64_t key_x, int64_t n_z, uint64_t* d_z_next,
                                        uint64_t key_z, uint64_t* d_out_next,
                                        int32_t n_next_shards, void* stream) {
  TW_ARG_CHECK(n_shards >= 0 && max_nx >= 0 && max_nz >= 0 && n_x >= 0 && n_z >= 0 &&
                   n_x < (1ll << 60) && n_z < (1ll << 60) && n_next_shards >= 0,
               "tw_count_pairs_rank_step: bad sizes");
  TW_ARG_CHECK(max_nz < (1ll << 24), "tw_count_pairs_rank_step: shards of < 2^24 z-values");
  TW_ARG_CHECK(d_x_next == nullptr || ((n_x == 0 || d_x_next != d_x_rec) &&
                                       (n_z == 0 || (d_z_next != nullptr && d_z_next != d_z_rec))),
               "tw_count_pairs_rank_step: next arrays must be distinct buffers");
  hipStream_t st = (hipStream_t)stream;
  NextStep nxt{};
  if (d_x_next != nullptr) {
    nxt = NextStep{d_x_rec, d_x_next, n_x, d_z_rec, d_z_next, n_z,
                   (unsigned long long*)d_out_next, d_out_next ? (int64_t)n_next_shards : 0,
                   make_feistel(std::max<int64_t>(n_x, 1), key_x),
                   make_feistel(std::max<int64_t>(n_z, 1), key_z), next_rank_blocks(n_x + n_z),
                   0, 1};
  } else if (d_out_next != nullptr && n_next_shards > 0) {
    TW_HIP_CHECK(tw_zero_async(d_out_next, 0, sizeof(uint64_t) * n_next_shards, st));
  }
  const bool counts = n_shards > 0 && max_nx > 0 && max_nz > 0;
  if (!counts) {
    if (nxt.blocks == 0) return TW_OK;
    hipLaunchKernelGGL((k_count_rank<16>), dim3(nxt.blocks), dim3(kBlock), 0, st, nullptr,
                       nullptr, nullptr, nullptr, 0, 1, 1, (int64_t)1, nullptr, nxt);
    TW_LAUNCH_CHECK();
    return TW_OK;
  }
  const RankPlan p = plan_rank(max_nx, max_nz, n_shards);
  TW_ARG_CHECK((p.blocks + nxt.blocks) * (kBlock / kWave) < (1ll << 31),
               "tw_count_pairs_rank_step: grid too large");
  dim3 g((unsigned)(p.blocks + nxt.blocks)), b(kBlock);
  auto* o = (unsigned long long*)d_out;
  if (p.R == 16)
    hipLaunchKernelGGL((k_count_rank<16>), g, b, 0, st, d_x_rec, d_x_off, d_z_rec, d_z_off,
                       n_shards, p.tiles_x, p.zchunks, p.z_chunk, o, nxt);
  else
    hipLaunchKernelGGL((k_count_rank<8>), g, b, 0, st, d_x_rec, d_x_off, d_z_rec, d_z_off,
                       n_shards, p.tiles_x, p.zchunks, p.z_chunk, o, nxt);
  TW_LAUNCH_CHECK();
  return TW_OK;
}

extern "C" int tw_gather_records(const void* d_in, const uint64_t* d_rec, int64_t n, void* d_out,
                                 void* stream) {
  TW_ARG_CHECK(n >= 0, "tw_gather_records: n < 0");
  TW_ARG_CHECK(n == 0 || d_in != d_out, "tw_gather_records: in and out must differ");
  if (n == 0) return TW_OK;
  const unsigned grid = (unsigned)std::min<int64_t>(4096, ceil_div(n, kBlock));
  hipLaunchKernelGGL(k_gather_records, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint64_t*)d_in, d_rec, n, (uint64_t*)d_out);
  TW_LAUNCH_CHECK();
  return TW_OK;
}
