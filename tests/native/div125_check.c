/* Test infrastructure (tests/test_div125.py): div125 (kubernetes-scheduler-simulator_amd/csrc/ksim_device.hpp)
 * -- x * RN(1/125), its exact remainder by an fma, one fma correction -- against IEEE division x / 125 for
 * every integer x in [0, 2^31) (the formula and the division are both odd in x).  Prints the mismatch
 * counts of the plain product and of the corrected form. */
#include <math.h>
#include <stdio.h>
#include <string.h>

int main(void) {
  const double c = 125.0, r = 1.0 / 125.0;
  long long bad_plain = 0, bad_fma = 0;
  for (long long x = 0; x < (1LL << 31); ++x) {
    const double xd = (double)x;
    const double q = xd / c;
    const double p = xd * r;
    const double e = fma(-p, c, xd);
    const double f = fma(e, r, p);
    bad_plain += memcmp(&q, &p, 8) != 0;
    bad_fma += memcmp(&q, &f, 8) != 0;
  }
  printf("%lld %lld\n", bad_plain, bad_fma);
  return 0;
}
