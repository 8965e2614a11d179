/* gen_go_rng_cooked.c -- computes Go's math/rand rngCooked table (csrc/go_rng_cooked.inc).
 *
 * Go's seeded source (src/math/rand/rng.go, unchanged since Go 1.0) XORs its seed expansion
 * with rngCooked[607], "the state of the generator after 780e10 iterations" of the additive
 * lagged-Fibonacci generator x[n] = x[n-607] + x[n-273] (mod 2^64) started from srand(1) of
 * src/math/rand/gen_cooked.go.  The table itself is not in this image, so it is recomputed
 * here from that published recipe: 7.8e12 steps = 607*q + r, where 607 steps return the
 * feed/tap pointers to their start, so the state after 607*q steps is M^q * v0 with M the
 * 607x607 matrix of one lap (integer arithmetic mod 2^64), followed by r single steps.
 * About 3 s at -O3.  Pinned by Go's published outputs for rand.Seed(1)
 * (tests/test_go_rand.py).
 *
 * Usage: gen_go_rng_cooked > csrc/go_rng_cooked.inc
 */
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { LEN = 607, TAP = 273 };

static int32_t seedrand(int32_t x) { /* x[n+1] = 48271 * x[n] mod (2^31 - 1), Schrage */
  const int32_t a = 48271, q = 44488, r = 3399;
  const int32_t hi = x / q, lo = x % q;
  x = a * lo - r * hi;
  if (x < 0) x += 2147483647;
  return x;
}

static void mul(const uint64_t* a, const uint64_t* b, uint64_t* c) {
  memset(c, 0, sizeof(uint64_t) * LEN * LEN);
  for (int i = 0; i < LEN; ++i)
    for (int k = 0; k < LEN; ++k) {
      const uint64_t s = a[i * LEN + k];
      if (!s) continue;
      const uint64_t* br = b + (size_t)k * LEN;
      uint64_t* cr = c + (size_t)i * LEN;
      for (int j = 0; j < LEN; ++j) cr[j] += s * br[j];
    }
}

int main(void) {
  /* gen_cooked.go srand(1): 20 warm-up draws, then u = x<<20 ^ x'<<10 ^ x'' per entry */
  uint64_t v[LEN];
  int32_t x = 1;
  for (int i = -20; i < LEN; ++i) {
    x = seedrand(x);
    if (i >= 0) {
      uint64_t u = (uint64_t)(int64_t)x << 20;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x << 10;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x;
      v[i] = u;
    }
  }
  const size_t bytes = sizeof(uint64_t) * LEN * LEN;
  uint64_t *m = calloc(1, bytes), *p = calloc(1, bytes), *t = calloc(1, bytes);
  if (!m || !p || !t) return 1;
  for (int i = 0; i < LEN; ++i) m[i * LEN + i] = p[i * LEN + i] = 1;
  int tap = 0, feed = LEN - TAP;
  for (int s = 0; s < LEN; ++s) { /* one lap of vrand(): vec[feed] += vec[tap] */
    if (--tap < 0) tap += LEN;
    if (--feed < 0) feed += LEN;
    for (int j = 0; j < LEN; ++j) m[feed * LEN + j] += m[tap * LEN + j];
  }
  const uint64_t steps = 7800000000000ULL;
  uint64_t q = steps / LEN;
  const uint64_t r = steps % LEN;
  while (q) { /* p = M^q */
    if (q & 1) { mul(p, m, t); memcpy(p, t, bytes); }
    q >>= 1;
    if (q) { mul(m, m, t); memcpy(m, t, bytes); }
  }
  uint64_t w[LEN];
  for (int i = 0; i < LEN; ++i) {
    uint64_t s = 0;
    for (int j = 0; j < LEN; ++j) s += p[i * LEN + j] * v[j];
    w[i] = s;
  }
  tap = 0, feed = LEN - TAP;
  for (uint64_t s = 0; s < r; ++s) {
    if (--tap < 0) tap += LEN;
    if (--feed < 0) feed += LEN;
    w[feed] += w[tap];
  }
  printf("/* Go math/rand rngCooked[607] (src/math/rand/rng.go), recomputed by tools/gen_go_rng_cooked.c */\n");
  for (int i = 0; i < LEN; ++i) printf("%" PRId64 "LL,%s", (int64_t)w[i], (i % 4 == 3) ? "\n" : " ");
  printf("\n");
  free(m); free(p); free(t);
  return 0;
}
