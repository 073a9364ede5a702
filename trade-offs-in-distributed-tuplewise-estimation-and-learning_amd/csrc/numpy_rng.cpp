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
#include <stdint.h>
#include <string.h>

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

struct MT {
  uint32_t* key;  // caller-owned 624 words (NumPy's untempered state)
  int pos;
  uint32_t tmp[kN];  // tempered outputs of the current state block
  int tempered_upto = 0;  // tmp[0, tempered_upto) valid for the current block

  void generate() {
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
  inline void temper_rest() {
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

void randint_fill(MT& mt, int64_t low, int64_t high, int64_t cnt, int64_t* out) {
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
    // masked rejection, branch-free: every raw draw is written, the slot advances only when
    // the draw is accepted; raw draws come from a pre-tempered 624-word block
    const uint32_t mask = (uint32_t)gen_mask(rng);
    const uint32_t r32 = (uint32_t)rng;
    int64_t o = 0;
    while (o < cnt) {
      if (mt.pos >= kN) mt.generate();
      mt.temper_rest();
      int p = mt.pos;
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

}  // namespace

extern "C" {

// One batch of randint calls, in order: call c draws cnt[c] values in [low[c], high[c]) into
// out[off_c : off_c + cnt[c]] (off_c = running sum).  key/pos: the MT19937 state as returned by
// np.random.get_state() (advanced in place).  Returns 0, or 1 for an empty range (NumPy's
// ValueError "high <= low"), leaving the state where the failing call would have started.
int tw_np_randint_batch(uint32_t* key, int32_t* pos, int32_t n_calls, const int64_t* low,
                        const int64_t* high, const int64_t* cnt, int64_t* out) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  int64_t o = 0;
  for (int32_t c = 0; c < n_calls; ++c) {
    if (high[c] <= low[c]) {
      *pos = mt.pos;
      return 1;
    }
    randint_fill(mt, low[c], high[c], cnt[c], out + o);
    o += cnt[c];
  }
  *pos = mt.pos;
  return 0;
}

// grad_inc_block's draws for all N shards of one UN_split call (compute_stats.py:155-156):
// for s in 0..N-1: ix[s*B .. s*B+B) = randint(0, kx, B), then iz[s*B ..) = randint(0, kz, B).
int tw_np_randint_pairs(uint32_t* key, int32_t* pos, int32_t N, int64_t kx, int64_t kz,
                        int64_t B, int64_t* ix, int64_t* iz) {
  if (kx <= 0 || kz <= 0) return 1;
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int32_t s = 0; s < N; ++s) {
    randint_fill(mt, 0, kx, B, ix + (int64_t)s * B);
    randint_fill(mt, 0, kz, B, iz + (int64_t)s * B);
  }
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
