// rtw_checker.h — exact sign of sin(x) for every finite float, shared by the gfx950 kernel
// (Checker::value, texture.rs:69-81) and the exhaustive proof oracle/tools/sin_sign_check.c.
//
// sign(sin a) for a > 0 is the parity of floor(a / pi).  For a = M 2^E (M a 24-bit integer)
// the parity is (M & A_E & 1) ^ (floor(M f_E) & 1), where 1/pi 2^E = A_E + f_E; f_E is taken to
// 96 bits from a table of 1/pi (computed with integer Machin arithmetic), so floor(M f_E) is
// exact unless a / pi lies within 2^-72 of an integer, which no float does (the proof tool checks
// every float against glibc's sinf).  Plain 32/64-bit integer arithmetic: host and device alike.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#define RTW_HD static inline
#endif

namespace rtw {

// T[0] holds the weights 2^31 .. 2^0 of 1/pi (zero); T[k] (k >= 1) the weights 2^(31-32k) .. 2^(-32k).
constexpr uint32_t INV_PI_T[12] = {0u,          0x517CC1B7u, 0x27220A94u, 0xFE13ABE8u, 0xFA9A6EE0u, 0x6DB14ACCu,
                                   0x9E21C820u, 0xFF28B1D5u, 0xEF5DE2B0u, 0xDB92371Du, 0x2126E970u, 0u};
RTW_HD uint32_t inv_pi_word(int k) { return (k >= 0 && k < 12) ? INV_PI_T[k] : 0u; }
// 32 bits of T starting at bit index b (index 0 = weight 2^31)
RTW_HD uint32_t inv_pi_bits32(int b) {
  const int q = b >> 5, s = b & 31;
  const uint32_t hi = inv_pi_word(q), lo = inv_pi_word(q + 1);
  return s ? (hi << s) | (lo >> (32 - s)) : hi;
}

// parity of floor(a / pi) for finite a >= 0 (1 = sin(a) < 0)
RTW_HD uint32_t pi_parity(float a) {
  if (!(a >= 3.0f)) return 0u;  // a < 3 < pi (or NaN): floor(a / pi) = 0
  uint32_t u;
  memcpy(&u, &a, 4);
  const uint32_t M = (u & 0x7FFFFFu) | 0x800000u;  // a >= 3 is normal
  const int E = (int)((u >> 23) & 0xFFu) - 150;      // a = M 2^E, E in [-22, 104]
  const int b0 = 32 + E;                             // first fraction bit of (1/pi) 2^E
  const uint32_t a_bit = (inv_pi_bits32(31 + E) >> 31) & 1u;
  const uint32_t F2 = inv_pi_bits32(b0), F1 = inv_pi_bits32(b0 + 32), F0 = inv_pi_bits32(b0 + 64);
  const uint64_t p0 = (uint64_t)M * F0;
  const uint64_t p1 = (uint64_t)M * F1 + (p0 >> 32);
  const uint64_t p2 = (uint64_t)M * F2 + (p1 >> 32);
  return ((M & a_bit) ^ (uint32_t)(p2 >> 32)) & 1u;
}

}  // namespace rtw
