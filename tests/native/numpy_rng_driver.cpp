// Test driver (not product code): runs csrc/numpy_rng.cpp's C ABI from a text script so the
// host RNG restatement can be built and exercised under AddressSanitizer + UBSan
// (csrc/Makefile target `sanitize`, tests/test_sanitize.py), on the AVX2 and the portable paths.
//
// stdin:  mode ("batch" | "pairs" | "shuffle"), pos, 624 key words, then
//   batch: n_calls, then n_calls lines "low high cnt"
//   pairs: "N kx kz B"
//   shuffle: "nx nz": shuffles arange(nx) then arange(nz) (int64 items) in place
// stdout: the draws (one per line), then the final pos and the 624 key words.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

extern "C" int tw_np_randint_batch(uint32_t* key, int32_t* pos, int32_t n_calls,
                                   const int64_t* low, const int64_t* high, const int64_t* cnt,
                                   int64_t* out);
extern "C" int tw_np_randint_pairs(uint32_t* key, int32_t* pos, int32_t N, int64_t kx,
                                   int64_t kz, int64_t B, int64_t* ix, int64_t* iz);
extern "C" int tw_np_shuffle_pair(uint32_t* key, int32_t* pos, void* x, int64_t nx, int64_t isx,
                                  void* z, int64_t nz, int64_t isz, int64_t* jbuf);

int main() {
  char mode[16];
  int32_t pos;
  if (scanf("%15s %d", mode, &pos) != 2) return 2;
  std::vector<uint32_t> key(624);
  for (auto& k : key)
    if (scanf("%u", &k) != 1) return 2;
  std::vector<int64_t> out;
  int rc = 0;
  if (std::string(mode) == "batch") {
    int n;
    if (scanf("%d", &n) != 1) return 2;
    std::vector<int64_t> lo(n), hi(n), cnt(n);
    int64_t tot = 0;
    for (int c = 0; c < n; ++c) {
      if (scanf("%lld %lld %lld", (long long*)&lo[c], (long long*)&hi[c], (long long*)&cnt[c]) != 3)
        return 2;
      tot += cnt[c];
    }
    out.resize(tot);
    rc = tw_np_randint_batch(key.data(), &pos, n, lo.data(), hi.data(), cnt.data(), out.data());
  } else if (std::string(mode) == "shuffle") {
    long long nx, nz;
    if (scanf("%lld %lld", &nx, &nz) != 2) return 2;
    std::vector<int64_t> x(nx), z(nz), j(nx + nz + 1);
    for (long long i = 0; i < nx; ++i) x[i] = i;
    for (long long i = 0; i < nz; ++i) z[i] = i;
    rc = tw_np_shuffle_pair(key.data(), &pos, x.data(), nx, 8, z.data(), nz, 8, j.data());
    out.insert(out.end(), x.begin(), x.end());
    out.insert(out.end(), z.begin(), z.end());
  } else {
    long long N, kx, kz, B;
    if (scanf("%lld %lld %lld %lld", &N, &kx, &kz, &B) != 4) return 2;
    std::vector<int64_t> ix(N * B), iz(N * B);
    rc = tw_np_randint_pairs(key.data(), &pos, (int32_t)N, kx, kz, B, ix.data(), iz.data());
    for (long long s = 0; s < N; ++s) {  // NumPy's order: per shard ix block then iz block
      out.insert(out.end(), ix.begin() + s * B, ix.begin() + (s + 1) * B);
      out.insert(out.end(), iz.begin() + s * B, iz.begin() + (s + 1) * B);
    }
  }
  printf("%d\n", rc);
  for (int64_t v : out) printf("%lld\n", (long long)v);
  printf("%d\n", pos);
  for (uint32_t k : key) printf("%u\n", k);
  return 0;
}
