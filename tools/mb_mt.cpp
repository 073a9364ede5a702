// Host microbenchmark of the replay loop's NumPy-exact draws (csrc/numpy_rng.cpp, included
// whole so its internals are reachable): the C4 segment's uint8 pair draws per step, and the
// MT19937 block pieces alone — the AVX-512 twist, the baseline-ISA tempering loop
// (MT::temper_rest) and the explicit 16-lane tempering (temper_block16) — in ns per word.
// g++ -O3 -std=c++17 -pthread -o /tmp/mb_mt tools/mb_mt.cpp && /tmp/mb_mt   (host CPU only)
#include "../trade-offs-in-distributed-tuplewise-estimation-and-learning_amd/csrc/numpy_rng.cpp"

#include <chrono>
#include <cstdio>

// pairs_u8_avx512 with the 16-word compaction (fill_masked16_u8), for the A/B
__attribute__((target("avx2,avx512f,avx512vl,avx512bw,avx512vbmi2,popcnt,bmi2"))) static void
pairs_u8_16(uint32_t* key, int32_t* pos, int N, int64_t kx, int64_t kz, int64_t B, uint8_t* ix,
            uint8_t* iz) {
  MT mt;
  mt.key = key;
  mt.pos = *pos;
  for (int s = 0; s < N; ++s) {
    fill_masked16_u8(mt, (uint32_t)gen_mask(kx - 1), (uint32_t)(kx - 1), B, ix + s * B);
    fill_masked16_u8(mt, (uint32_t)gen_mask(kz - 1), (uint32_t)(kz - 1), B, iz + s * B);
  }
  *pos = mt.pos;
}

template <class F>
static double best_of(int reps, F f) {
  double best = 1e9;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
                              .count());
  }
  return best;
}

int main() {
  static uint32_t key[kN];
  for (int i = 0; i < kN; ++i) key[i] = 12345u * i + 7;
  int32_t pos = kN;
  const int S = 25, N = 100, B = 100;  // a 25-step C4 segment: kx = 91, kz = 7
  std::vector<uint8_t> out(S * 2 * N * B);
  const double t = best_of(50, [&] { tw_np_randint_pairs_steps_u8(key, &pos, S, N, 91, 7, B,
                                                                  out.data()); });
  printf("u8 pair draws      %7.2f us/step (64-word compaction, the product)\n", t / S * 1e6);
  std::vector<uint8_t> out2(S * 2 * N * B);
  pos = kN;
  const double t16 = best_of(50, [&] {
    for (int st = 0; st < S; ++st)
      pairs_u8_16(key, &pos, N, 91, 7, B, out2.data() + st * 2 * N * B,
                  out2.data() + st * 2 * N * B + N * B);
  });
  printf("u8 pair draws      %7.2f us/step (16-word compaction)\n", t16 / S * 1e6);
  // both forms from one state: the same bytes
  for (int i = 0; i < kN; ++i) key[i] = 777u * i + 3;
  pos = kN;
  tw_np_randint_pairs_steps_u8(key, &pos, S, N, 91, 7, B, out.data());
  for (int i = 0; i < kN; ++i) key[i] = 777u * i + 3;
  int32_t pos2 = kN;
  for (int st = 0; st < S; ++st)
    pairs_u8_16(key, &pos2, N, 91, 7, B, out2.data() + st * 2 * N * B,
                out2.data() + st * 2 * N * B + N * B);
  printf("same draws: %s\n", out == out2 && pos == pos2 ? "yes" : "NO");
  MT mt;
  mt.key = key;
  mt.pos = kN;
  uint32_t sink = 0;
  const int blocks = 1000;
  auto per_word = [&](auto f) { return best_of(20, [&] { for (int b = 0; b < blocks; ++b) f(); })
                                       / blocks / kN * 1e9; };
  printf("twist (16 lanes)   %7.2f ns/word\n", per_word([&] { twist_vec<16>(key); sink += key[3]; }));
  printf("temper_rest        %7.2f ns/word\n", per_word([&] {
           mt.tempered_upto = 0;
           mt.pos = 0;
           mt.temper_rest();
           sink += mt.tmp[5];
         }));
  printf("temper_block16     %7.2f ns/word\n", per_word([&] { temper_block16(key, mt.tmp); sink += mt.tmp[5]; }));
  printf("(sink %u)\n", sink);
  return 0;
}
