// go_rand.hpp -- Go's math/rand, the global source the reference seeds per experiment
// (pkg/simulator/core.go:115 rand.Seed(WorkloadTuningConfig.Seed)).
//
// Third-party algorithm outside /root/reference: the Go standard library (src/math/rand,
// rng.go + rand.go).  The seeded source is unchanged since Go 1.0, Shuffle/int31n since
// Go 1.10; go.mod:4 says go 1.15.  Restated from the published source:
//   rngSource.Seed     seedrand expansion XOR rngCooked        rng.go  Seed
//   rngSource.Uint64   additive lagged Fibonacci, len 607, tap 273
//   Rand.Int63/Uint32/Int31/Int/Int63n/Int31n/int31n/Intn/Float64/Perm/Shuffle   rand.go
// rngCooked is recomputed by tools/gen_go_rng_cooked.c (go_rng_cooked.inc).  Pinned by Go's
// published outputs for rand.Seed(1) (tests/test_go_rand.py) and, end to end, by the
// reference's per-seed expected_results rows.
#pragma once
#include <cstdint>
#include <vector>

namespace ksim_go {

static const int64_t kRngCooked[607] = {
#include "go_rng_cooked.inc"
};

class Rand {
 public:
  explicit Rand(int64_t seed) { Seed(seed); }

  void Seed(int64_t seed) {  // rng.go rngSource.Seed
    tap_ = 0;
    feed_ = kLen - kTap;
    draws_ = 0;
    seed = seed % kInt32Max;
    if (seed < 0) seed += kInt32Max;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < kLen; ++i) {
      x = seedrand(x);
      if (i >= 0) {
        uint64_t u = (uint64_t)(int64_t)x << 40;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x << 20;
        x = seedrand(x);
        u ^= (uint64_t)(int64_t)x;
        u ^= (uint64_t)kRngCooked[i];
        vec_[i] = u;
      }
    }
  }

  uint64_t Uint64() {  // rng.go rngSource.Uint64
    ++draws_;
    if (--tap_ < 0) tap_ += kLen;
    if (--feed_ < 0) feed_ += kLen;
    const uint64_t x = vec_[feed_] + vec_[tap_];
    vec_[feed_] = x;
    return x;
  }
  int64_t Int63() { return (int64_t)(Uint64() & kMask); }
  uint32_t Uint32() { return (uint32_t)(Int63() >> 31); }
  int32_t Int31() { return (int32_t)(Int63() >> 32); }
  int64_t Int() { const uint64_t u = (uint64_t)Int63(); return (int64_t)(u << 1 >> 1); }

  int64_t Int63n(int64_t n) {
    if (n <= 0) return -1;  // Go panics
    if ((n & (n - 1)) == 0) return Int63() & (n - 1);
    const int64_t max = (int64_t)((1ULL << 63) - 1 - (1ULL << 63) % (uint64_t)n);
    int64_t v = Int63();
    while (v > max) v = Int63();
    return v % n;
  }
  int32_t Int31n(int32_t n) {
    if (n <= 0) return -1;  // Go panics
    if ((n & (n - 1)) == 0) return Int31() & (n - 1);
    const int32_t max = (int32_t)((1U << 31) - 1 - (1U << 31) % (uint32_t)n);
    int32_t v = Int31();
    while (v > max) v = Int31();
    return v % n;
  }
  // rand.go int31n: Lemire's multiply-shift, used only by Shuffle
  int32_t int31n(int32_t n) {
    uint32_t v = Uint32();
    uint64_t prod = (uint64_t)v * (uint64_t)n;
    uint32_t low = (uint32_t)prod;
    if (low < (uint32_t)n) {
      const uint32_t thresh = (uint32_t)(-n) % (uint32_t)n;
      while (low < thresh) {
        v = Uint32();
        prod = (uint64_t)v * (uint64_t)n;
        low = (uint32_t)prod;
      }
    }
    return (int32_t)(prod >> 32);
  }
  int64_t Intn(int64_t n) {
    if (n <= 0) return -1;  // Go panics
    if (n <= kInt32Max) return Int31n((int32_t)n);
    return Int63n(n);
  }
  double Float64() {
    for (;;) {
      const double f = (double)Int63() / 9223372036854775808.0;
      if (f != 1.0) return f;
    }
  }
  std::vector<int> Perm(int n) {
    std::vector<int> m(n > 0 ? n : 0);
    for (int i = 0; i < n; ++i) {
      const int j = (int)Intn(i + 1);
      m[i] = m[j];
      m[j] = i;
    }
    return m;
  }
  template <class Swap>
  void Shuffle(int64_t n, Swap swap) {
    int64_t i = n - 1;
    for (; i > (1LL << 31) - 1 - 1; --i) swap(i, Int63n(i + 1));
    for (; i > 0; --i) swap(i, (int64_t)int31n((int32_t)(i + 1)));
  }

  // the source's state (the Random draw structure continues the stream on the device) and the
  // number of Uint64 draws since Seed
  void State(uint64_t* vec, int* tap, int* feed) const {
    for (int i = 0; i < kLen; ++i) vec[i] = vec_[i];
    *tap = tap_;
    *feed = feed_;
  }
  uint64_t Draws() const { return draws_; }

 private:
  static constexpr int kLen = 607, kTap = 273;
  static constexpr int64_t kInt32Max = 2147483647;
  static constexpr uint64_t kMask = (1ULL << 63) - 1;
  static int32_t seedrand(int32_t x) {  // x[n+1] = 48271 * x[n] mod (2^31 - 1)
    const int32_t a = 48271, q = 44488, r = 3399;
    const int32_t hi = x / q, lo = x % q;
    x = a * lo - r * hi;
    if (x < 0) x += (int32_t)kInt32Max;
    return x;
  }
  int tap_ = 0, feed_ = 0;
  uint64_t draws_ = 0;
  uint64_t vec_[kLen];
};

}  // namespace ksim_go
