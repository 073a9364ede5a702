// imagecount.h — incomplete counts on float32 score images in LDS (csrc/imagecount.hip),
// called by the tw_count_pairs_idx(32)_ws / tw_count_pairs_rng_ws entry points (rankcount.hip).
#pragma once
#include "tw_common.h"
#include "nextstep.h"

namespace tw {

inline int64_t al4h(int64_t n) { return (n + 3) & ~(int64_t)3; }

struct ImgPlan {
  bool ok;      // a shard pair's images fit in LDS and the predicate is GT / HALF
  int parts;    // 1024-thread blocks per shard
  size_t lds;   // bytes of images per block
};

// pairs: the largest number of pairs (or draws) of one shard
ImgPlan plan_images(int32_t n_shards, int64_t max_nx, int64_t max_nz, int32_t pred, int64_t pairs);

template <typename I>
int launch_idx_images(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, const I* ix, const I* iz, const int64_t* pair_off,
                      int32_t dtype, int32_t pred, const ImgPlan& p, uint64_t* out,
                      hipStream_t st);

// nxt: the next repartition carried by the count threads (nxt.blocks == 0: none)
int launch_rng_images(const void* x, const int64_t* x_off, const void* z, const int64_t* z_off,
                      int32_t n_shards, int64_t B, uint64_t seed, uint64_t sid, int32_t dtype,
                      int32_t pred, const ImgPlan& p, uint64_t* out, const NextStep& nxt,
                      hipStream_t st);

}  // namespace tw
