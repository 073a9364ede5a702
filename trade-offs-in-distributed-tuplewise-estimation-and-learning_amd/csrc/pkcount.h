// pkcount.h — the packed-f32 compare-and-count of rank images shared by csrc/rankimage.hip
// (records of one step) and csrc/chain.hip (per-step image bags of a whole call).
//
// With integer-valued images (x: g(x), z: -g(z); g(v) = #{z : z < v}) the pair predicate
// x > z is clamp(g(x) - g(z)) == 1, and a packed add with the clamp modifier evaluates it for
// two lanes' worth of pairs per instruction:
//     t   = clamp(gx + nz)      v_pk_add_f32 ... clamp      (nz from an SGPR pair)
//     acc = acc + t             v_pk_add_f32
#pragma once
#include "tw_common.h"

namespace tw {

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr float kImgNever = -33554432.0f;  // -2^25: NaN x and padded lanes, never greater

// nz2: an SGPR pair; both packed halves of x take its LOW word: t = clamp(x_lo + nz, x_hi + nz)
__device__ __forceinline__ f2 gt_clamp(f2 x, uint64_t nz2) {
  f2 t;
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] clamp" : "=v"(t) : "v"(x), "s"(nz2));
  return t;
}
// ... its HIGH word (op_sel picks the high half of src1 for both result halves)
__device__ __forceinline__ f2 gt_clamp_hi(f2 x, uint64_t nz2) {
  f2 t;
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1] clamp"
               : "=v"(t) : "v"(x), "s"(nz2));
  return t;
}
__device__ __forceinline__ void acc_add(f2& a, f2 t) {
  asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(t));
}

}  // namespace tw
