/* Exhaustive check behind the kernel's Checker fast path (texture.rs:69-81):
 * for every float x with 2^-12 <= |x| < 65536, sign(libm sinf(x)) == (-1)^floor((double)x / pi),
 * and sinf(x) != 0; also reports min |sinf(x)| (no product of three can underflow to 0).
 * Build/run: gcc -O2 -fopenmp -ffp-contract=off sin_sign_check.c -lm && ./a.out */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(void) {
  const double INV_PI = 0.31830988618379067154;
  long long bad = 0, zero = 0;
  float minabs = 1.0f;
  uint32_t lo = 0x39800000u, hi = 0x47800000u; /* [2^-12, 65536): the kernel fast path */
#pragma omp parallel for reduction(+ : bad, zero) reduction(min : minabs) schedule(static, 1 << 16)
  for (long long b = lo; b < (long long)hi; ++b) {
    for (int sgn = 0; sgn < 2; ++sgn) {
      uint32_t u = (uint32_t)b | (sgn ? 0x80000000u : 0u);
      float x;
      memcpy(&x, &u, 4);
      float s = sinf(x);
      double k = floor((double)x * INV_PI);
      int neg = ((long long)k) & 1;
      if (s == 0.0f) zero++;
      else if ((s < 0.0f) != (neg != 0)) bad++;
      float a = fabsf(s);
      if (a < minabs) minabs = a;
    }
  }
  printf("mismatches %lld zeros %lld min|sinf| %g\n", bad, zero, minabs);
  return bad || zero ? 1 : 0;
}
