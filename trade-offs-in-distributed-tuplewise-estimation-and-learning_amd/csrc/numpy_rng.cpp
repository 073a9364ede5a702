// numpy_rng.cpp — bulk draws of NumPy's legacy global RNG, host code.
//
// The reference consumes np.random's legacy RandomState (MT19937) through many small calls:
// per learning step 2*N randint calls (grad_inc_block, compute_stats.py:155-156) and per
// reshuffle 2*N more (SWR_divide, compute_stats.py:52-53).  Bit-exact replay needs exactly
// those values; making them one Python call at a time costs ~3 us each.  These functions
// advance a copy of the RandomState key (np.random.get_state()) by the same algorithm NumPy
// uses and write all values of a batch of randint calls at once; the caller then puts the
// advanced state back (np.random.set_state), so the global RNG ends exactly where the
// reference's sequence of calls would leave it.
//
// Algorithms restated (NumPy 2.x legacy paths):
//   MT19937 genrand_int32 (Matsumoto & Nishimura 1998), 624-word state + position;
//   RandomState.randint(low, high, size) for int64 output: rng = high-1-low;
//     rng == 0          -> `low`, no draw;
//     rng <  2^32-1     -> masked rejection on 32-bit draws: v = next32 & mask until v <= rng;
//     rng == 2^32-1     -> low + next32;
//     rng >= 2^32       -> masked rejection on 64-bit draws (hi32 << 32 | lo32).
// Parity is pinned by tests/test_numpy_rng.py against np.random itself.
//
// Speed: the 624-word block is generated and tempered with vector loops, and the masked
// rejection is a left-pack of accepted draws (16 lanes with AVX-512 compress, 8 with an AVX2
// permutation LUT, chosen at run time by __builtin_cpu_supports; scalar branch-free compaction
// otherwise).
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <vector>

#define TW_INLINE inline __attribute__((always_inline))

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

struct MT {
  uint32_t* key;  // caller-owned 624 words (NumPy's untempered state)
  int pos;
  uint32_t tmp[kN];  // tempered outputs of the current state block
  int tempered_upto = 0;  // tmp[0, tempered_upto) valid for the current block

  TW_INLINE void generate() {
    int i = 0;
    uint32_t y;
    for (; i < kN - kM; ++i) {
      y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    y = (key[kN - 1] & kUpper) | (key[0] & kLower);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    pos = 0;
    tempered_upto = 0;
  }

  static inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // make tmp[pos, kN) valid (vectorisable loop over the rest of the block)
  TW_INLINE void temper_rest() {
    if (tempered_upto < kN) {
      const int from = pos > tempered_upto ? pos : tempered_upto;
      for (int i = from; i < kN; ++i) tmp[i] = temper(key[i]);
      tempered_upto = kN;
    }
  }

  uint32_t next32() {
    if (pos >= kN) generate();
    return temper(key[pos++]);
  }

  uint64_t next64() {
    const uint64_t hi = next32();
    return (hi << 32) | next32();
  }
};

// The 624-word twist with explicit vectors (the auto-vectorised loop above runs at ~1 ns per
// word, as much as all the rest of a draw): key[i] = key[i+397] ^ twist(key[i], key[i+1]) for
// i < 227 (reads only old words), then key[i] = key[i-227] ^ twist(...) for 227 <= i < 623
// (key[i-227] is new; 227 exceeds the vector width, so lanes never read a word this same
// vector writes), then the last word.  Same words as MT::generate.
template <int W>
struct TwistVec;
template <>
struct TwistVec<16> {
  __attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) static inline void step(uint32_t* key, int i,
                                                                            int off) {
    const __m512i up = _mm512_set1_epi32((int)kUpper), lo = _mm512_set1_epi32((int)kLower);
    const __m512i one = _mm512_set1_epi32(1), ma = _mm512_set1_epi32((int)kMatrixA);
    const __m512i a = _mm512_loadu_si512((const void*)(key + i));
    const __m512i b = _mm512_loadu_si512((const void*)(key + i + 1));
    const __m512i y = _mm512_or_si512(_mm512_and_si512(a, up), _mm512_and_si512(b, lo));
    const __m512i mag = _mm512_and_si512(_mm512_sub_epi32(_mm512_setzero_si512(),
                                                          _mm512_and_si512(y, one)), ma);
    const __m512i src = _mm512_loadu_si512((const void*)(key + i + off));
    _mm512_storeu_si512((void*)(key + i),
                        _mm512_xor_si512(_mm512_xor_si512(src, _mm512_srli_epi32(y, 1)), mag));
  }
};
template <>
struct TwistVec<8> {
  __attribute__((target("avx2"))) static inline void step(uint32_t* key, int i, int off) {
    const __m256i up = _mm256_set1_epi32((int)kUpper), lo = _mm256_set1_epi32((int)kLower);
    const __m256i one = _mm256_set1_epi32(1), ma = _mm256_set1_epi32((int)kMatrixA);
    const __m256i a = _mm256_loadu_si256((const __m256i*)(key + i));
    const __m256i b = _mm256_loadu_si256((const __m256i*)(key + i + 1));
    const __m256i y = _mm256_or_si256(_mm256_and_si256(a, up), _mm256_and_si256(b, lo));
    const __m256i mag = _mm256_and_si256(_mm256_sub_epi32(_mm256_setzero_si256(),
                                                          _mm256_and_si256(y, one)), ma);
    const __m256i src = _mm256_loadu_si256((const __m256i*)(key + i + off));
    _mm256_storeu_si256((__m256i*)(key + i),
                        _mm256_xor_si256(_mm256_xor_si256(src, _mm256_srli_epi32(y, 1)), mag));
  }
};

template <int W>
TW_INLINE void twist_vec(uint32_t* key) {
  int i = 0;
  for (; i + W <= kN - kM; i += W) TwistVec<W>::step(key, i, kM);  // 0 .. 227 (old words)
  for (; i < kN - kM; ++i) {
    const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
    key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
  }
  for (; i + W <= kN - 1; i += W) TwistVec<W>::step(key, i, kM - kN);  // 227 .. 623
  for (; i < kN - 1; ++i) {
    const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
    key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
  }
  const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
  key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
}

// The whole block's tempering with explicit vectors (MT::temper_rest's loop is vectorised for
// the baseline ISA only: 0.50 ns per word against 0.15 with 16 lanes, more than the twist's
// 0.23 — tools/mb_mt.cpp), straight after the twist.
__attribute__((target("avx2,avx512f,avx512vl"))) inline void temper_block16(const uint32_t* key,
                                                                           uint32_t* tmp) {
  const __m512i b = _mm512_set1_epi32((int)0x9d2c5680u), c = _mm512_set1_epi32((int)0xefc60000u);
  for (int i = 0; i < kN; i += 16) {  // kN = 39 * 16
    __m512i y = _mm512_loadu_si512((const void*)(key + i));
    y = _mm512_xor_si512(y, _mm512_srli_epi32(y, 11));
    y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 7), b));
    y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 15), c));
    y = _mm512_xor_si512(y, _mm512_srli_epi32(y, 18));
    _mm512_storeu_si512((void*)(tmp + i), y);
  }
}
__attribute__((target("avx2"))) inline void temper_block8(const uint32_t* key, uint32_t* tmp) {
  const __m256i b = _mm256_set1_epi32((int)0x9d2c5680u), c = _mm256_set1_epi32((int)0xefc60000u);
  for (int i = 0; i < kN; i += 8) {  // kN = 78 * 8
    __m256i y = _mm256_loadu_si256((const __m256i*)(key + i));
    y = _mm256_xor_si256(y, _mm256_srli_epi32(y, 11));
    y = _mm256_xor_si256(y, _mm256_and_si256(_mm256_slli_epi32(y, 7), b));
    y = _mm256_xor_si256(y, _mm256_and_si256(_mm256_slli_epi32(y, 15), c));
    y = _mm256_xor_si256(y, _mm256_srli_epi32(y, 18));
    _mm256_storeu_si256((__m256i*)(tmp + i), y);
  }
}

// the twist for SIMD level kIsa (2: 16 lanes, 1: 8 lanes, 0: MT::generate's loops); the vector
// levels temper the whole new block at once (tmp valid, temper_rest a no-op until the next)
template <int kIsa>
TW_INLINE void generate_isa(MT& mt) {
  static_assert(kN % 16 == 0, "the block tempering loops assume 16 | kN");
  if (kIsa == 2) {
    twist_vec<16>(mt.key);
    temper_block16(mt.key, mt.tmp);
  } else if (kIsa == 1) {
    twist_vec<8>(mt.key);
    temper_block8(mt.key, mt.tmp);
  } else {
    mt.generate();
    return;
  }
  mt.pos = 0;
  mt.tempered_upto = kN;
}

inline uint64_t gen_mask(uint64_t max) {
  uint64_t m = max;
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  m |= m >> 8;
  m |= m >> 16;
  m |= m >> 32;
  return m;
}

// lane indices of the accepted lanes of an 8-bit accept mask, packed to the front
struct PackLut {
  uint32_t idx[256][8];
  PackLut() {
    for (int m = 0; m < 256; ++m) {
      int k = 0;
      for (int l = 0; l < 8; ++l)
        if (m >> l & 1) idx[m][k++] = (uint32_t)l;
      for (; k < 8; ++k) idx[m][k] = 0;
    }
  }
};
const PackLut g_pack;

// 8 raw draws at a time: accept v = tmp & mask iff v <= r32, left-pack, widen, add low.
// Needs cnt - o >= 8 for the unconditional 8-wide store.  Returns the new p (o updated).
__attribute__((target("avx2,popcnt"))) inline int pack8_avx2(const uint32_t* tmp, int p,
                                                             uint32_t mask, uint32_t r32,
                                                             int64_t low, int64_t cnt,
                                                             int64_t* out, int64_t& o) {
  const __m256i vm = _mm256_set1_epi32((int)mask);
  const __m256i sign = _mm256_set1_epi32((int)0x80000000u);
  const __m256i vr = _mm256_set1_epi32((int)(r32 ^ 0x80000000u));
  const __m256i vlow = _mm256_set1_epi64x(low);
  while (p + 8 <= kN && cnt - o >= 8) {
    const __m256i v = _mm256_and_si256(_mm256_loadu_si256((const __m256i*)(tmp + p)), vm);
    const __m256i rej = _mm256_cmpgt_epi32(_mm256_xor_si256(v, sign), vr);  // unsigned v > r
    const int acc = ~_mm256_movemask_ps(_mm256_castsi256_ps(rej)) & 0xFF;
    const __m256i packed = _mm256_permutevar8x32_epi32(
        v, _mm256_loadu_si256((const __m256i*)g_pack.idx[acc]));
    const __m256i lo4 = _mm256_cvtepu32_epi64(_mm256_castsi256_si128(packed));
    const __m256i hi4 = _mm256_cvtepu32_epi64(_mm256_extracti128_si256(packed, 1));
    _mm256_storeu_si256((__m256i*)(out + o), _mm256_add_epi64(lo4, vlow));
    _mm256_storeu_si256((__m256i*)(out + o + 4), _mm256_add_epi64(hi4, vlow));
    o += __builtin_popcount((unsigned)acc);
    p += 8;
  }
  return p;
}

// the same with 16 lanes (AVX-512: compare to a mask register, compress the accepted lanes)
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) inline int pack16_avx512(
    const uint32_t* tmp, int p, uint32_t mask, uint32_t r32, int64_t low, int64_t cnt,
    int64_t* out, int64_t& o) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  const __m512i vlow = _mm512_set1_epi64(low);
  while (p + 16 <= kN && cnt - o >= 16) {
    const __m512i v = _mm512_and_si512(_mm512_loadu_si512((const void*)(tmp + p)), vm);
    const __mmask16 acc = _mm512_cmple_epu32_mask(v, vr);
    const __m512i packed = _mm512_maskz_compress_epi32(acc, v);
    const __m512i lo8 = _mm512_cvtepu32_epi64(_mm512_castsi512_si256(packed));
    const __m512i hi8 = _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(packed, 1));
    _mm512_storeu_si512((void*)(out + o), _mm512_add_epi64(lo8, vlow));
    _mm512_storeu_si512((void*)(out + o + 8), _mm512_add_epi64(hi8, vlow));
    o += __builtin_popcount((unsigned)acc);
    p += 16;
  }
  return p;
}

// A whole masked-rejection call with 16-lane AVX-512 batches and no scalar tail: a batch past
// the end of the 624-word block is a masked load, and the last batch of the call keeps only
// the lowest `cnt - o` accepted lanes (pdep) and consumes the words up to the last of them —
// NumPy stops drawing at the cnt-th accepted value.
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) inline void fill_masked16(
    MT& mt, uint32_t mask, uint32_t r32, int64_t low, int64_t cnt, int64_t* out) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  const __m512i vlow = _mm512_set1_epi64(low);
  int64_t o = 0;
  while (o < cnt) {
    if (mt.pos >= kN) generate_isa<2>(mt);
    mt.temper_rest();
    int p = mt.pos;
    while (p < kN && o < cnt) {
      const int avail = kN - p;
      const __mmask16 lm = avail >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << avail) - 1u);
      const __m512i v = _mm512_and_si512(_mm512_maskz_loadu_epi32(lm, mt.tmp + p), vm);
      uint32_t acc = (uint32_t)_mm512_mask_cmple_epu32_mask(lm, v, vr);
      const int64_t rem = cnt - o;
      int na = __builtin_popcount(acc);
      int used = avail >= 16 ? 16 : avail;
      if (na >= rem) {  // the call ends inside this batch: at its rem-th accepted word
        if (na > rem) acc = _pdep_u32((1u << rem) - 1u, acc);
        na = (int)rem;
        used = 32 - __builtin_clz(acc);
      }
      const __m512i packed = _mm512_maskz_compress_epi32((__mmask16)acc, v);
      const __m512i lo8 = _mm512_add_epi64(_mm512_cvtepu32_epi64(_mm512_castsi512_si256(packed)),
                                           vlow);
      const __m512i hi8 = _mm512_add_epi64(
          _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(packed, 1)), vlow);
      const uint32_t sm = (1u << na) - 1u;
      _mm512_mask_storeu_epi64((void*)(out + o), (__mmask8)(sm & 0xFF), lo8);
      _mm512_mask_storeu_epi64((void*)(out + o + 8), (__mmask8)(sm >> 8), hi8);
      o += na;
      p += used;
    }
    mt.pos = p;
  }
}

// kIsa: 0 portable, 1 AVX2, 2 AVX-512 (+ BMI2)
template <int kIsa>
TW_INLINE void randint_fill(MT& mt, int64_t low, int64_t high, int64_t cnt, int64_t* out) {
  const uint64_t rng = (uint64_t)(high - 1) - (uint64_t)low;
  if (rng == 0) {
    for (int64_t i = 0; i < cnt; ++i) out[i] = low;
    return;
  }
  if (rng <= 0xFFFFFFFFull) {
    if (rng == 0xFFFFFFFFull) {
      for (int64_t i = 0; i < cnt; ++i) out[i] = (int64_t)((uint64_t)low + mt.next32());
      return;
    }
    // masked rejection: every raw draw is written, the slot advances only when the draw is
    // accepted; raw draws come from a pre-tempered 624-word block
    const uint32_t mask = (uint32_t)gen_mask(rng);
    const uint32_t r32 = (uint32_t)rng;
    if (kIsa == 2) {
      fill_masked16(mt, mask, r32, low, cnt, out);
      return;
    }
    int64_t o = 0;
    while (o < cnt) {
      if (mt.pos >= kN) generate_isa<kIsa>(mt);
      mt.temper_rest();
      int p = mt.pos;
      if (kIsa >= 2) p = pack16_avx512(mt.tmp, p, mask, r32, low, cnt, out, o);
      if (kIsa >= 1) p = pack8_avx2(mt.tmp, p, mask, r32, low, cnt, out, o);
      while (p < kN && o < cnt) {
        const uint32_t v = mt.tmp[p++] & mask;
        out[o] = (int64_t)((uint64_t)low + v);
        o += (v <= r32);
      }
      mt.pos = p;
    }
    return;
  }
  const uint64_t mask = gen_mask(rng);
  for (int64_t i = 0; i < cnt; ++i) {
    uint64_t v;
    while ((v = (mt.next64() & mask)) > rng) {
    }
    out[i] = (int64_t)((uint64_t)low + v);
  }
}

template <int kIsa>
TW_INLINE int batch_body(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                         const int64_t* high, const int64_t* cnt, int64_t* out) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  int64_t o = 0;
  for (int32_t c = 0; c < n_calls;) {
    if (high[c] <= low[c]) {
      *pos = mt.pos;
      return 1;
    }
    // consecutive calls on the same range are one call of their summed size: the masked
    // rejection keeps no state between calls (SWR_divide's N calls per side: one fill each)
    int32_t c2 = c + 1;
    int64_t run = cnt[c];
    while (c2 < n_calls && low[c2] == low[c] && high[c2] == high[c]) run += cnt[c2++];
    randint_fill<kIsa>(mt, low[c], high[c], run, out + o);
    o += run;
    c = c2;
  }
  *pos = mt.pos;
  return 0;
}

template <int kIsa>
TW_INLINE void pairs_body(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz,
                          int64_t B, int64_t* ix, int64_t* iz) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int32_t s = 0; s < N; ++s) {
    randint_fill<kIsa>(mt, 0, kx, B, ix + (int64_t)s * B);
    randint_fill<kIsa>(mt, 0, kz, B, iz + (int64_t)s * B);
  }
  *pos = mt.pos;
}

int batch_generic(uint32_t* key, int32_t* pos, int32_t n, const int64_t* lo, const int64_t* hi,
                  const int64_t* cnt, int64_t* out) {
  return batch_body<0>(key, pos, n, lo, hi, cnt, out);
}
__attribute__((target("avx2,popcnt"))) int batch_avx2(uint32_t* key, int32_t* pos, int32_t n,
                                                      const int64_t* lo, const int64_t* hi,
                                                      const int64_t* cnt, int64_t* out) {
  return batch_body<1>(key, pos, n, lo, hi, cnt, out);
}
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) int batch_avx512(
    uint32_t* key, int32_t* pos, int32_t n, const int64_t* lo, const int64_t* hi,
    const int64_t* cnt, int64_t* out) {
  return batch_body<2>(key, pos, n, lo, hi, cnt, out);
}
void pairs_generic(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz, int64_t B,
                   int64_t* ix, int64_t* iz) {
  pairs_body<0>(key, pos, N, kx, kz, B, ix, iz);
}
__attribute__((target("avx2,popcnt"))) void pairs_avx2(uint32_t* key, int32_t* pos, int32_t N,
                                                       int64_t kx, int64_t kz, int64_t B,
                                                       int64_t* ix, int64_t* iz) {
  pairs_body<1>(key, pos, N, kx, kz, B, ix, iz);
}
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) void pairs_avx512(
    uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz, int64_t B, int64_t* ix,
    int64_t* iz) {
  pairs_body<2>(key, pos, N, kx, kz, B, ix, iz);
}

// RandomState.shuffle's index draws (legacy _shuffle_raw + random_interval): for i = n-1 down
// to 1, j[i] = the first v = next & mask(i) with v <= i (32-bit draws while i <= 2^32-1,
// 64-bit above).  Branch-free: every raw draw is written to j[i], i moves on only on accept.
// 8 raw draws at a time while the bound i is large: lane k is accepted iff v_k <= i - (accepts
// in lanes < k), so v <= i - 7 is a sure accept and v > i a sure reject; a batch of only sure
// lanes is left-packed and stored reversed at j[i-7 .. i] (j[i - r] = r-th accept; the lanes
// past the accepts land on lower slots that later draws overwrite).  Any unsure lane: the
// batch is left to the scalar loop.  Returns the new p (i updated).
template <typename J>
__attribute__((target("avx2,popcnt"))) inline int shuffle8_avx2(const uint32_t* tmp, int p,
                                                               uint32_t mask, int64_t lo,
                                                               int64_t& i, J* j) {
  const __m256i vm = _mm256_set1_epi32((int)mask);
  const __m256i sign = _mm256_set1_epi32((int)0x80000000u);
  const __m256i rev = _mm256_setr_epi32(7, 6, 5, 4, 3, 2, 1, 0);
  while (p + 8 <= kN && i - 8 > lo && i >= 8) {
    const __m256i v = _mm256_and_si256(_mm256_loadu_si256((const __m256i*)(tmp + p)), vm);
    const __m256i vs = _mm256_xor_si256(v, sign);
    const __m256i rej = _mm256_cmpgt_epi32(vs, _mm256_set1_epi32((int)((uint32_t)i ^ 0x80000000u)));
    const __m256i unsure = _mm256_andnot_si256(
        rej, _mm256_cmpgt_epi32(vs, _mm256_set1_epi32((int)((uint32_t)(i - 7) ^ 0x80000000u))));
    if (!_mm256_testz_si256(unsure, unsure)) break;
    const int acc = ~_mm256_movemask_ps(_mm256_castsi256_ps(rej)) & 0xFF;
    const __m256i packed = _mm256_permutevar8x32_epi32(
        v, _mm256_loadu_si256((const __m256i*)g_pack.idx[acc]));
    const __m256i r = _mm256_permutevar8x32_epi32(packed, rev);  // lane l = accept 7 - l
    if constexpr (sizeof(J) == 8) {
      _mm256_storeu_si256((__m256i*)(j + i - 7),
                          _mm256_cvtepu32_epi64(_mm256_castsi256_si128(r)));
      _mm256_storeu_si256((__m256i*)(j + i - 3),
                          _mm256_cvtepu32_epi64(_mm256_extracti128_si256(r, 1)));
    } else {
      _mm256_storeu_si256((__m256i*)(j + i - 7), r);
    }
    i -= __builtin_popcount((unsigned)acc);
    p += 8;
  }
  return p;
}

// the same with 16 lanes (sure accept v <= i - 15)
template <typename J>
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) inline int shuffle16_avx512(
    const uint32_t* tmp, int p, uint32_t mask, int64_t lo, int64_t& i, J* j) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i rev = _mm512_setr_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
  while (p + 16 <= kN && i - 16 > lo && i >= 16) {
    const __m512i v = _mm512_and_si512(_mm512_loadu_si512((const void*)(tmp + p)), vm);
    const __mmask16 rej = _mm512_cmpgt_epu32_mask(v, _mm512_set1_epi32((int)(uint32_t)i));
    const __mmask16 unsure =
        (__mmask16)(~rej & _mm512_cmpgt_epu32_mask(v, _mm512_set1_epi32((int)(uint32_t)(i - 15))));
    if (unsure) break;
    const __mmask16 acc = (__mmask16)~rej;
    const __m512i packed = _mm512_maskz_compress_epi32(acc, v);
    const __m512i r = _mm512_permutexvar_epi32(rev, packed);  // lane l = accept 15 - l
    if constexpr (sizeof(J) == 8) {
      _mm512_storeu_si512((void*)(j + i - 15),
                          _mm512_cvtepu32_epi64(_mm512_castsi512_si256(r)));
      _mm512_storeu_si512((void*)(j + i - 7),
                          _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(r, 1)));
    } else {
      _mm512_storeu_si512((void*)(j + i - 15), r);
    }
    i -= __builtin_popcount((unsigned)acc);
    p += 16;
  }
  return p;
}

// J = int64_t (the host swaps) or uint32_t (the device swaps: n <= 2^31, so 32-bit draws only).
// The draws for i = hi down to stop (stop >= 1; the whole shuffle: hi = n - 1, stop = 1): a
// shuffle drawn in consecutive ranges consumes the same words and makes the same draws as one
// call (the range end only lowers the loops' bound; the SIMD batches never store below it)
template <int kIsa, typename J>
void shuffle_draws(MT& mt, int64_t hi, int64_t stop, J* j) {
  int64_t i = hi;
  while (sizeof(J) == 8 && i >= stop && (uint64_t)i > 0xFFFFFFFFull) {
    const uint64_t mask = gen_mask((uint64_t)i);
    uint64_t v;
    while ((v = (mt.next64() & mask)) > (uint64_t)i) {
    }
    j[i--] = (J)v;
  }
  while (i >= stop) {
    const uint32_t mask = (uint32_t)gen_mask((uint64_t)i);
    // this mask serves i in (mask/2, mask]; the range ends below stop
    const int64_t lo = std::max<int64_t>((int64_t)(mask >> 1), stop - 1);
    if (mt.pos >= kN) generate_isa<kIsa>(mt);
    mt.temper_rest();
    int p = mt.pos;
    for (;;) {
      if (kIsa >= 2) p = shuffle16_avx512(mt.tmp, p, mask, lo, i, j);
      if (kIsa >= 1) p = shuffle8_avx2(mt.tmp, p, mask, lo, i, j);
      // scalar: until the block or the mask range ends, or (SIMD) 8 words have passed
      const int stop_p = kIsa ? (p + 8 < kN ? p + 8 : kN) : kN;
      while (p < stop_p && i > lo) {
        const uint32_t v = mt.tmp[p++] & mask;
        j[i] = (J)v;
        i -= (int64_t)(v <= (uint32_t)i);
      }
      if (p >= kN || i <= lo) break;
    }
    mt.pos = p;
  }
}

// the swaps of _shuffle_raw for items of `itemsize` bytes, i = n-1 down to 1, with the random
// side prefetched a few swaps ahead
void shuffle_apply(char* data, int64_t n, int64_t itemsize, const int64_t* j) {
  constexpr int64_t kAhead = 24;
  if (itemsize == 8) {
    uint64_t* a = (uint64_t*)data;
    for (int64_t i = n - 1; i >= 1; --i) {
      if (i - kAhead >= 1) __builtin_prefetch(a + j[i - kAhead], 1);
      const int64_t k = j[i];
      const uint64_t t = a[k];
      a[k] = a[i];
      a[i] = t;
    }
    return;
  }
  char buf[256];
  for (int64_t i = n - 1; i >= 1; --i) {
    if (i - kAhead >= 1) __builtin_prefetch(data + j[i - kAhead] * itemsize, 1);
    const int64_t k = j[i];
    if (k == i) continue;
    char* pk = data + k * itemsize;
    char* pi = data + i * itemsize;
    for (int64_t o = 0; o < itemsize; o += 256) {
      const int64_t c = itemsize - o < 256 ? itemsize - o : 256;
      memcpy(buf, pk + o, c);
      memcpy(pk + o, pi + o, c);
      memcpy(pi + o, buf, c);
    }
  }
}

template <typename J>
__attribute__((target("avx2,popcnt"))) void shuffle_draws_avx2(MT& mt, int64_t hi, int64_t stop,
                                                               J* j) {
  shuffle_draws<1>(mt, hi, stop, j);
}
template <typename J>
__attribute__((target("avx2,avx512f,avx512vl,popcnt,bmi2"))) void shuffle_draws_avx512(MT& mt,
                                                                                  int64_t hi,
                                                                                  int64_t stop,
                                                                                  J* j) {
  shuffle_draws<2>(mt, hi, stop, j);
}

// the draws for i = hi down to stop (the whole shuffle of n items: hi = n - 1, stop = 1)
template <typename J>
void shuffle_draws_isa(MT& mt, int64_t hi, int64_t stop, J* j, int isa) {
  if (isa == 2)
    shuffle_draws_avx512(mt, hi, stop, j);
  else if (isa == 1)
    shuffle_draws_avx2(mt, hi, stop, j);
  else
    shuffle_draws<0>(mt, hi, stop, j);
}

// grad_inc_block's draws straight into uint16 outputs (ranges <= 65536) with AVX-512 VBMI2:
// the masked words of a 16-lane batch are narrowed (vpmovdw), the accepted lanes compressed in
// a register (vpcompressw) and stored with a lane mask — no int64 widening and no narrowing pass
// afterwards.  Same words consumed, same values as fill_masked16.
__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) inline void
fill_masked16_u16(MT& mt, uint32_t mask, uint32_t r32, int64_t cnt, uint16_t* out) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  int64_t o = 0;
  while (o < cnt) {
    if (mt.pos >= kN) generate_isa<2>(mt);
    mt.temper_rest();
    int p = mt.pos;
    while (p < kN && o < cnt) {
      const int avail = kN - p;
      const __mmask16 lm = avail >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << avail) - 1u);
      const __m512i v = _mm512_and_si512(_mm512_maskz_loadu_epi32(lm, mt.tmp + p), vm);
      uint32_t acc = (uint32_t)_mm512_mask_cmple_epu32_mask(lm, v, vr);
      const int64_t rem = cnt - o;
      int na = __builtin_popcount(acc);
      int used = avail >= 16 ? 16 : avail;
      if (na >= rem) {  // the call ends inside this batch: at its rem-th accepted word
        if (na > rem) acc = _pdep_u32((1u << rem) - 1u, acc);
        na = (int)rem;
        used = 32 - __builtin_clz(acc);
      }
      const __m256i packed = _mm256_maskz_compress_epi16((__mmask16)acc, _mm512_cvtepi32_epi16(v));
      _mm256_mask_storeu_epi16((void*)(out + o), (__mmask16)((1u << na) - 1u), packed);
      o += na;
      p += used;
    }
    mt.pos = p;
  }
}

__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) void
pairs_u16_avx512(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz, int64_t B,
                 uint16_t* ix, uint16_t* iz) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int32_t s = 0; s < N; ++s) {
    for (int side = 0; side < 2; ++side) {
      const uint64_t rng = (uint64_t)((side ? kz : kx) - 1);
      uint16_t* o = (side ? iz : ix) + (int64_t)s * B;
      if (rng == 0) {  // randint(0, 1): no draw, all zeros (as randint_fill)
        for (int64_t i = 0; i < B; ++i) o[i] = 0;
      } else {
        fill_masked16_u16(mt, (uint32_t)gen_mask(rng), (uint32_t)rng, B, o);
      }
    }
  }
  *pos = mt.pos;
}

// fill_masked16_u16 with uint8 output (every value < 256): the same words consumed, the same
// values, a byte compress instead of a word compress.
__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) inline void
fill_masked16_u8(MT& mt, uint32_t mask, uint32_t r32, int64_t cnt, uint8_t* out) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  int64_t o = 0;
  while (o < cnt) {
    if (mt.pos >= kN) generate_isa<2>(mt);
    mt.temper_rest();
    int p = mt.pos;
    while (p < kN && o < cnt) {
      const int avail = kN - p;
      const __mmask16 lm = avail >= 16 ? (__mmask16)0xFFFF : (__mmask16)((1u << avail) - 1u);
      const __m512i v = _mm512_and_si512(_mm512_maskz_loadu_epi32(lm, mt.tmp + p), vm);
      uint32_t acc = (uint32_t)_mm512_mask_cmple_epu32_mask(lm, v, vr);
      const int64_t rem = cnt - o;
      int na = __builtin_popcount(acc);
      int used = avail >= 16 ? 16 : avail;
      if (na >= rem) {  // the call ends inside this batch: at its rem-th accepted word
        if (na > rem) acc = _pdep_u32((1u << rem) - 1u, acc);
        na = (int)rem;
        used = 32 - __builtin_clz(acc);
      }
      const __m128i packed = _mm_maskz_compress_epi8((__mmask16)acc, _mm512_cvtepi32_epi8(v));
      _mm_mask_storeu_epi8((void*)(out + o), (__mmask16)((1u << na) - 1u), packed);
      o += na;
      p += used;
    }
    mt.pos = p;
  }
}

// fill_masked16_u8 over 64 words per iteration: four 16-lane accept masks joined into one
// 64-bit mask, ONE popcount and end test per 64 words (the loop-carried chain mask -> popcount
// -> output offset is what bounds the 16-word form, tools/mb_mt.cpp), then four independent
// compress-stores at offsets from the partial popcounts.  Same words consumed, same values.
__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) inline void
fill_masked64_u8(MT& mt, uint32_t mask, uint32_t r32, int64_t cnt, uint8_t* out) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  int64_t o = 0;
  while (o < cnt) {
    if (mt.pos >= kN) generate_isa<2>(mt);
    mt.temper_rest();
    int p = mt.pos;
    while (p < kN && o < cnt) {
      const int w = kN - p < 64 ? kN - p : 64;  // words of this batch (the block's end)
      __m512i v[4];
      uint64_t acc = 0;
#pragma GCC unroll 4
      for (int g = 0; g < 4; ++g) {
        const int lanes = w - 16 * g;
        const __mmask16 lm = lanes >= 16  ? (__mmask16)0xFFFF
                             : lanes > 0 ? (__mmask16)((1u << lanes) - 1u)
                                         : (__mmask16)0;
        v[g] = _mm512_and_si512(_mm512_maskz_loadu_epi32(lm, mt.tmp + p + 16 * g), vm);
        acc |= (uint64_t)_mm512_mask_cmple_epu32_mask(lm, v[g], vr) << (16 * g);
      }
      const int64_t rem = cnt - o;
      int na = __builtin_popcountll(acc);
      int used = w;
      if (na >= rem) {  // the call ends inside this batch: at its rem-th accepted word
        if (na > rem) acc = _pdep_u64((1ull << rem) - 1ull, acc);  // rem < na <= 64
        na = (int)rem;
        used = 64 - __builtin_clzll(acc);
      }
      int off = 0;
#pragma GCC unroll 4
      for (int g = 0; g < 4; ++g) {
        const __mmask16 mg = (__mmask16)(acc >> (16 * g));
        const int cg = __builtin_popcount((unsigned)mg);
        const __m128i packed = _mm_maskz_compress_epi8(mg, _mm512_cvtepi32_epi8(v[g]));
        _mm_mask_storeu_epi8((void*)(out + o + off), (__mmask16)((1u << cg) - 1u), packed);
        off += cg;
      }
      o += na;
      p += used;
    }
    mt.pos = p;
  }
}

// fill_masked64_u8 with uint16 output (every value < 65536): SWR_divide's row draws for the
// replay loop's narrowed row tables.  Same words consumed, same values.
__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) inline void
fill_masked64_u16(MT& mt, uint32_t mask, uint32_t r32, int64_t cnt, uint16_t* out) {
  const __m512i vm = _mm512_set1_epi32((int)mask);
  const __m512i vr = _mm512_set1_epi32((int)r32);
  int64_t o = 0;
  while (o < cnt) {
    if (mt.pos >= kN) generate_isa<2>(mt);
    mt.temper_rest();
    int p = mt.pos;
    while (p < kN && o < cnt) {
      const int w = kN - p < 64 ? kN - p : 64;
      __m512i v[4];
      uint64_t acc = 0;
#pragma GCC unroll 4
      for (int g = 0; g < 4; ++g) {
        const int lanes = w - 16 * g;
        const __mmask16 lm = lanes >= 16  ? (__mmask16)0xFFFF
                             : lanes > 0 ? (__mmask16)((1u << lanes) - 1u)
                                         : (__mmask16)0;
        v[g] = _mm512_and_si512(_mm512_maskz_loadu_epi32(lm, mt.tmp + p + 16 * g), vm);
        acc |= (uint64_t)_mm512_mask_cmple_epu32_mask(lm, v[g], vr) << (16 * g);
      }
      const int64_t rem = cnt - o;
      int na = __builtin_popcountll(acc);
      int used = w;
      if (na >= rem) {
        if (na > rem) acc = _pdep_u64((1ull << rem) - 1ull, acc);
        na = (int)rem;
        used = 64 - __builtin_clzll(acc);
      }
      int off = 0;
#pragma GCC unroll 4
      for (int g = 0; g < 4; ++g) {
        const __mmask16 mg = (__mmask16)(acc >> (16 * g));
        const int cg = __builtin_popcount((unsigned)mg);
        const __m256i packed = _mm256_maskz_compress_epi16(mg, _mm512_cvtepi32_epi16(v[g]));
        _mm256_mask_storeu_epi16((void*)(out + o + off), (__mmask16)((1u << cg) - 1u), packed);
        off += cg;
      }
      o += na;
      p += used;
    }
    mt.pos = p;
  }
}

__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) int
batch_u16_avx512(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* high,
                 const int64_t* cnt, uint16_t* out) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  int64_t o = 0;
  for (int32_t c = 0; c < n_calls;) {
    int32_t c2 = c + 1;  // consecutive calls on one range: one fill (as batch_body)
    int64_t run = cnt[c];
    while (c2 < n_calls && high[c2] == high[c]) run += cnt[c2++];
    const uint64_t rng = (uint64_t)(high[c] - 1);
    if (rng == 0) {
      for (int64_t i = 0; i < run; ++i) out[o + i] = 0;
    } else {
      fill_masked64_u16(mt, (uint32_t)gen_mask(rng), (uint32_t)rng, run, out + o);
    }
    o += run;
    c = c2;
  }
  *pos = mt.pos;
  return 0;
}

__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) void
pairs_u8_avx512(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz, int64_t B,
                uint8_t* ix, uint8_t* iz) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int32_t s = 0; s < N; ++s) {
    for (int side = 0; side < 2; ++side) {
      const uint64_t rng = (uint64_t)((side ? kz : kx) - 1);
      uint8_t* o = (side ? iz : ix) + (int64_t)s * B;
      if (rng == 0) {  // randint(0, 1): no draw, all zeros (as randint_fill)
        for (int64_t i = 0; i < B; ++i) o[i] = 0;
      } else {
        fill_masked64_u8(mt, (uint32_t)gen_mask(rng), (uint32_t)rng, B, o);
      }
    }
  }
  *pos = mt.pos;
}

// SIMD level chosen once at run time: 2 AVX-512 (F + VL) + BMI2, 1 AVX2, 0 portable.
// TW_NP_RNG_SCALAR=1 forces the portable path, TW_NP_RNG_ISA=avx2 caps it at AVX2 (tests run
// every level against NumPy).
int isa_level() {
  static const int v = [] {
    const char* e = getenv("TW_NP_RNG_SCALAR");
    if (e && e[0] == '1') return 0;
    __builtin_cpu_init();
    if (!__builtin_cpu_supports("avx2") || !__builtin_cpu_supports("popcnt")) return 0;
    const char* cap = getenv("TW_NP_RNG_ISA");
    if (cap && strcmp(cap, "avx2") == 0) return 1;
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                   __builtin_cpu_supports("bmi2")
               ? 2
               : 1;
  }();
  return v;
}

// the uint16 pair draws above (AVX-512 level plus BW + VBMI2; TW_NP_RNG_ISA / _SCALAR caps
// apply through isa_level)
bool has_vbmi2() {
  static const bool v = isa_level() == 2 && __builtin_cpu_supports("avx512bw") &&
                        __builtin_cpu_supports("avx512vbmi2");
  return v;
}

}  // namespace

extern "C" {

// One batch of randint calls, in order: call c draws cnt[c] values in [low[c], high[c]) into
// out[off_c : off_c + cnt[c]] (off_c = running sum).  key/pos: the MT19937 state as returned by
// np.random.get_state() (advanced in place).  Returns 0, or 1 for an empty range (NumPy's
// ValueError "high <= low"), leaving the state where the failing call would have started.
int tw_np_randint_batch(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                        const int64_t* high, const int64_t* cnt, int64_t* out) {
  const int isa = isa_level();
  return isa == 2   ? batch_avx512(key, pos, n_calls, low, high, cnt, out)
         : isa == 1 ? batch_avx2(key, pos, n_calls, low, high, cnt, out)
                    : batch_generic(key, pos, n_calls, low, high, cnt, out);
}

// tw_np_randint_batch narrowed to uint16 for calls on [0, high) with high <= 65536 (SWR_divide's
// rows of the replay loop's narrowed row tables): the same words consumed, the same values.
// Returns 1 for a call outside that form (state untouched).
int tw_np_randint_batch_u16(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                            const int64_t* high, const int64_t* cnt, uint16_t* out) {
  for (int32_t c = 0; c < n_calls; ++c)
    if (low[c] != 0 || high[c] < 1 || high[c] > 65536 || cnt[c] < 0) return 1;
  if (has_vbmi2()) return batch_u16_avx512(key, pos, n_calls, high, cnt, out);
  static thread_local std::vector<int64_t> scratch;
  int64_t tot = 0;
  for (int32_t c = 0; c < n_calls; ++c) tot += cnt[c];
  scratch.resize((size_t)tot);
  const int rc = tw_np_randint_batch(key, pos, n_calls, low, high, cnt, scratch.data());
  if (rc) return rc;
  for (int64_t i = 0; i < tot; ++i) out[i] = (uint16_t)scratch[(size_t)i];
  return 0;
}

// grad_inc_block's draws for all N shards of one UN_split call (compute_stats.py:155-156):
// for s in 0..N-1: ix[s*B .. s*B+B) = randint(0, kx, B), then iz[s*B ..) = randint(0, kz, B).
int tw_np_randint_pairs(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz,
                        int64_t B, int64_t* ix, int64_t* iz) {
  if (kx <= 0 || kz <= 0) return 1;
  const int isa = isa_level();
  if (isa == 2)
    pairs_avx512(key, pos, N, kx, kz, B, ix, iz);
  else if (isa == 1)
    pairs_avx2(key, pos, N, kx, kz, B, ix, iz);
  else
    pairs_generic(key, pos, N, kx, kz, B, ix, iz);
  return 0;
}

// S consecutive steps of grad_inc_block's draws: out is (S, 2, N, B) int64, out[s][0] the
// step's X indices of all N shards and out[s][1] its Z indices (tw_np_randint_pairs per step).
int tw_np_randint_pairs_steps(uint32_t* key, int32_t* pos, int32_t S, int32_t N, int64_t kx,
                              int64_t kz, int64_t B, int64_t* out) {
  if (kx <= 0 || kz <= 0 || S < 0 || N < 0 || B < 0) return 1;
  const int64_t per = (int64_t)N * B;
  for (int32_t st = 0; st < S; ++st) {
    int64_t* o = out + (int64_t)st * 2 * per;
    const int rc = tw_np_randint_pairs(key, pos, N, kx, kz, B, o, o + per);
    if (rc) return rc;
  }
  return 0;
}

// The same S steps narrowed to uint16 (kx, kz <= 65536: every index < 65536), for a quarter
// of the bytes on the way to the device (the replay loop's H2D copy; tw_widen_u16 restores
// int64 there).  Each step is drawn into a thread-local int64 scratch, then narrowed.
int tw_np_randint_pairs_steps_u16(uint32_t* key, int32_t* pos, int32_t S, int32_t N, int64_t kx,
                                  int64_t kz, int64_t B, uint16_t* out) {
  if (kx <= 0 || kz <= 0 || kx > 65536 || kz > 65536 || S < 0 || N < 0 || B < 0) return 1;
  const int64_t per = (int64_t)N * B;
  if (has_vbmi2()) {
    for (int32_t st = 0; st < S; ++st) {
      uint16_t* o = out + (int64_t)st * 2 * per;
      pairs_u16_avx512(key, pos, N, kx, kz, B, o, o + per);
    }
    return 0;
  }
  static thread_local std::vector<int64_t> scratch;
  scratch.resize((size_t)(2 * per));
  for (int32_t st = 0; st < S; ++st) {
    const int rc = tw_np_randint_pairs(key, pos, N, kx, kz, B, scratch.data(),
                                       scratch.data() + per);
    if (rc) return rc;
    uint16_t* o = out + (int64_t)st * 2 * per;
    for (int64_t i = 0; i < 2 * per; ++i) o[i] = (uint16_t)scratch[(size_t)i];
  }
  return 0;
}

// The same S steps narrowed to uint8 (kx, kz <= 256): half the bytes of the uint16 form.
int tw_np_randint_pairs_steps_u8(uint32_t* key, int32_t* pos, int32_t S, int32_t N, int64_t kx,
                                 int64_t kz, int64_t B, uint8_t* out) {
  if (kx <= 0 || kz <= 0 || kx > 256 || kz > 256 || S < 0 || N < 0 || B < 0) return 1;
  const int64_t per = (int64_t)N * B;
  if (has_vbmi2()) {
    for (int32_t st = 0; st < S; ++st) {
      uint8_t* o = out + (int64_t)st * 2 * per;
      pairs_u8_avx512(key, pos, N, kx, kz, B, o, o + per);
    }
    return 0;
  }
  static thread_local std::vector<int64_t> scratch;
  scratch.resize((size_t)(2 * per));
  for (int32_t st = 0; st < S; ++st) {
    const int rc = tw_np_randint_pairs(key, pos, N, kx, kz, B, scratch.data(),
                                       scratch.data() + per);
    if (rc) return rc;
    uint8_t* o = out + (int64_t)st * 2 * per;
    for (int64_t i = 0; i < 2 * per; ++i) o[i] = (uint8_t)scratch[(size_t)i];
  }
  return 0;
}

// np.random.shuffle(x); np.random.shuffle(z) on C-contiguous arrays of nx / nz items of isx /
// isz bytes (rows of a 2-D array are items): the same draws from the same stream, the same
// swaps, the same final state.  x's draws come first; x's swaps then run on a second thread
// while z's draws and swaps run here.  jbuf: nx + nz int64 of scratch.  nz == 0 / z == NULL:
// x alone.
int tw_np_shuffle_pair(uint32_t* key, int32_t* pos, void* x, int64_t nx, int64_t isx, void* z,
                       int64_t nz, int64_t isz, int64_t* jbuf) {
  if (nx < 0 || nz < 0 || (nx > 1 && !x) || (nz > 1 && !z) || isx < 1 || isz < 1) return 2;
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  int64_t* jx = jbuf;
  int64_t* jz = jbuf + (nx > 0 ? nx : 0);
  const int isa = isa_level();
  auto draws = [&](int64_t n, int64_t* j) { shuffle_draws_isa(mt, n - 1, (int64_t)1, j, isa); };
  if (nx > 1) draws(nx, jx);
  std::thread tx;
  bool threaded = false;
  if (nx > 1) {
    if (nz > 1 && nx >= 65536) {
      tx = std::thread(shuffle_apply, (char*)x, nx, isx, (const int64_t*)jx);
      threaded = true;
    } else {
      shuffle_apply((char*)x, nx, isx, jx);
    }
  }
  if (nz > 1) {
    draws(nz, jz);
    shuffle_apply((char*)z, nz, isz, jz);
  }
  if (threaded) tx.join();
  *pos = mt.pos;
  return 0;
}

// The index draws of np.random.shuffle on n items (n <= 2^31) without the swaps: j[i] for
// i = n-1 down to 1 (j[0] untouched), as uint32, for the device swaps (devshuffle.hip).  The
// state advances exactly as the shuffle's would.
int tw_np_shuffle_draws32(uint32_t* key, int32_t* pos, int64_t n, uint32_t* j) {
  if (n < 0 || n > (1ll << 31) || (n > 1 && !j)) return 2;
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  if (n > 1) shuffle_draws_isa(mt, n - 1, (int64_t)1, j, isa_level());
  *pos = mt.pos;
  return 0;
}

// The same draws in consecutive ranges (the streamed last shuffle of the drop-in,
// _engine.DeviceShuffles.push_z_part): j[i] for i = hi down to lo (1 <= lo <= hi < n <= 2^31),
// the state advanced past them.  Ranges [hi_0 = n-1 .. lo_0], [lo_0 - 1 .. lo_1], ... down to 1
// make exactly tw_np_shuffle_draws32's draws.
int tw_np_shuffle_draws32_range(uint32_t* key, int32_t* pos, int64_t n, int64_t hi, int64_t lo,
                                uint32_t* j) {
  if (n < 2 || n > (1ll << 31) || lo < 1 || hi < lo || hi >= n || !j) return 2;
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  shuffle_draws_isa(mt, hi, lo, j, isa_level());
  *pos = mt.pos;
  return 0;
}

// Raw genrand_int32 stream (for tests).
int tw_np_mt_next32(uint32_t* key, int32_t* pos, int64_t cnt, uint32_t* out) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int64_t i = 0; i < cnt; ++i) out[i] = mt.next32();
  *pos = mt.pos;
  return 0;
}

}  // extern "C"
