/* Exhaustive proof behind the kernel's Checker decision (texture.rs:69-81:
 * sinf(f x) * sinf(f y) * sinf(f z) < 0 with Rust's f32::sin = the platform libm, glibc here).
 * Over EVERY finite float x (both signs) it checks against glibc's sinf:
 *   fast range  2^-12 <= |x| < 65536: sign(sinf x) == (-1)^floor((double)x / pi) (the kernel's
 *               double-precision fast path), == rtw::pi_parity too, and sinf x != 0;
 *   large range |x| >= 65536:        sign(sinf x) == rtw::pi_parity(|x|) (exact integer
 *               reduction, csrc/rtw_checker.h) and sinf x != 0;
 *   tiny range  0 < |x| < 2^-12:     sinf x == x bit for bit (the kernel multiplies the x's);
 * and reports min |sinf x| over |x| >= 2^-12 (a product of three such factors cannot underflow).
 * TEST INFRASTRUCTURE.  Build/run (tests/test_checker_proof.py does):
 *   g++ -O2 -fopenmp -ffp-contract=off sin_sign_check.cpp -o sin_sign_check && ./sin_sign_check */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../raytracer-weekend_amd/csrc/rtw_checker.h"

int main(int argc, char** argv) {
  const double INV_PI = 0.31830988618379067154;
  long long bad_fast = 0, bad_large = 0, bad_tiny = 0, zero = 0, bad_parity = 0;
  float minabs = 1.0f;
  /* argv[1] = stride (1 = exhaustive; the CPU test suite samples with a prime stride) */
  const long long stride = argc > 1 ? atoll(argv[1]) : 1;
  const uint32_t TINY = 0x39800000u, BIG = 0x47800000u, INF = 0x7F800000u;
#pragma omp parallel for reduction(+ : bad_fast, bad_large, bad_tiny, zero, bad_parity) reduction(min : minabs) \
    schedule(dynamic, 1 << 12)
  for (long long b = 1; b < (long long)INF; b += stride) {
    for (int sgn = 0; sgn < 2; ++sgn) {
      const uint32_t u = (uint32_t)b | (sgn ? 0x80000000u : 0u);
      float x;
      memcpy(&x, &u, 4);
      const float s = sinf(x);
      if ((uint32_t)b < TINY) {
        if (memcmp(&s, &x, 4) != 0) bad_tiny++;
        continue;
      }
      if (s == 0.0f) { zero++; continue; }
      const float a = fabsf(s);
      if (a < minabs) minabs = a;
      const int neg_sin = s < 0.0f;
      const int neg_par = (int)(rtw::pi_parity(fabsf(x)) ^ (uint32_t)(x < 0.0f));
      if ((uint32_t)b < BIG) {
        const int k_odd = (int)(((long long)floor((double)x * INV_PI)) & 1);
        if (neg_sin != k_odd) bad_fast++;
        if (neg_sin != neg_par) bad_parity++;
      } else if (neg_sin != neg_par) {
        bad_large++;
      }
    }
  }
  printf("fast-range mismatches %lld, pi_parity mismatches (fast range) %lld, large-range mismatches %lld, "
         "tiny sinf(x) != x %lld, zeros %lld, min|sinf| (|x| >= 2^-12) %g, stride %lld\n",
         bad_fast, bad_parity, bad_large, bad_tiny, zero, minabs, stride);
  return bad_fast || bad_parity || bad_large || bad_tiny || zero ? 1 : 0;
}
