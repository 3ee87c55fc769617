/* markstein_check.c -- CPU check of the division used by the kernels (csrc/slgpu.hip div_rn):
 * q = RN(a/b) from y = RN(1/b) with two FMA corrections, against IEEE a/b, on random operands
 * from the ranges the kernels feed it (Otsu: a in [0, 255], b in (eps, 1]; rays: a = u - cx
 * over pixel coordinates, b = fx, and a = x or y over a norm b >= 1).
 *   gcc -O2 -o markstein_check tools/markstein_check.c -lm && ./markstein_check [samples]
 * Prints the mismatch count (expected 0) and exits non-zero on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double ud(void) { return (double)(xr() >> 11) * (1.0 / 9007199254740992.0); }

static double div_rn(double a, double b, double y) {
  const double q0 = a * y;
  const double q1 = fma(fma(-b, q0, a), y, q0);
  return fma(fma(-b, q1, a), y, q1);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000L;
  long bad = 0;
  for (long it = 0; it < n; ++it) {
    double a, b;
    switch (it % 4) {
      case 0: b = 1e-7 + ud() * (1.0 - 1e-7); a = ud() * 255.0; break;            /* Otsu mu1 */
      case 1: b = 1e-7 + ud(); a = ldexp(ud(), -(int)(xr() % 60)); break;         /* small numerators */
      case 2: b = 100.0 + ud() * 20000.0; a = (double)(xr() % 8192) - (ud() * 8192.0); break;  /* (u-cx)/fx */
      default: b = 1.0 + ud() * 30.0; a = (ud() - 0.5) * 2.0 * b; break;          /* x / norm */
    }
    const double y = 1.0 / b;
    if (div_rn(a, b, y) != a / b) ++bad;
  }
  printf("samples=%ld mismatches=%ld\n", n, bad);
  return bad != 0;
}
