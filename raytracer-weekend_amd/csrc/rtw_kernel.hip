// rtw_kernel.hip — gfx950 path-tracing megakernel and the device half of the C-ABI.
//
// Hot path restated (reference raytracer_weekend_lib/src/):
//   Raytracer::render / sample_pixel (lib.rs:57-95)   -> one work unit per path (pixel, sample); the samples
//                                                        of a pixel are summed in sample order afterwards
//   sample_ray (lib.rs:97-117)                          -> iterative bounce loop, L = T * terminal
//   [Box<dyn Hittable>]::hit (hittable/mod.rs:57-69)    -> 4-wide BVH walk (or the flat list), min t,
//                                                        ties -> the larger DFS key
//   Material::scatter / emitted (material.rs, light_source.rs), Texture::value (texture.rs,
//   image_texture.rs), Camera::get_ray (camera.rs:66-74)
//
// Numerics: compiled with -ffp-contract=off and IEEE div/sqrt (hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt), so every primitive test, scatter and the
// throughput product are bit-identical to the oracle's iterative integrator.  Divisions that
// share a divisor use Markstein's correction from an exact reciprocal (rcp_rn, proven over every
// float on the device).  Only the BVH culling uses FMA / rcp approximations, and it is
// conservative (padded boxes + slack), so it changes which nodes are visited, never the answer.
//
// Kernel structure: path_kernel is PERSISTENT -- the grid is the resident capacity,
// and each wave draws path ids from a global queue (RenderArgs::batch per atomic: 1024 in the
// 1024-lane LDS-node and the list-mode kernels, 2048 elsewhere; knob RTW_BATCH) into an LDS pool, hands
// them to its idle lanes by ballot + mbcnt prefix (64 consecutive ids = one sample of one 8x8 tile), and
// loops: regenerate -> trace_begin (the always-tested list) -> trace_run (resumable BVH4 walk with
// postponed leaves; returns once quota16/16 of the lanes are done) -> shade.  A finished path writes
// its radiance to an ordered sample buffer that reduce_kernel sums per pixel in sample order.
// Variants (pick_kernel): feature-specialised instantiations; the LDS-node kernel for sphere worlds whose
// tree fits (the whole node table in LDS, sorted-push walk over 16-bit child codes; by default 1024-lane
// workgroups, 2 per CU at 8 waves/SIMD, with the paths' T / depth / id in LDS rows: DESIGN.md §3); the
// global-node kernels (256-lane workgroups, 32-bit LDS stack) for meshes, with half-precision nodes
// (DevNode4h) for large trees; BVH-less list-mode kernels for <= 32 primitives.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>

#include "../../include/rtw.h"
#include "rtw_checker.h"
#include "rtw_scene.hpp"

namespace rtw {
namespace dev {

// Compile-time switches.  The product build sets none of them.  Only these remain, and none changes a
// result: RTW_NT_SAMPLES (0 = the sample buffer written / read with plain accesses; an A/B knob) and the
// COUNT-build diagnostics RTW_LANE_DIAG / RTW_UNI_DIAG (node-loop lane states) and RTW_SHADE_DIAG (shading
// sub-phase timers; each replaces the COUNT build's sub_cycles).  RTW_DIAG_ONE_TRIP (a timing diagnostic that is
// NOT the reference's distribution) refuses to compile unless RTW_ALLOW_NON_REFERENCE is set as well, so no
// product build can carry it.  Round 3's equivalence switches (sphere-root / unit() reciprocals, the
// precomputed Dielectric ratios, start_path's LDS operands, select-form rect tests) are the only code now;
// the dropped experiments (round 3's per-rect-guarded chain reciprocals, the xoroshiro64+ output) are deleted.
#if defined(RTW_DIAG_ONE_TRIP) && !defined(RTW_ALLOW_NON_REFERENCE)
#error "RTW_DIAG_ONE_TRIP changes the sampled distribution (not the reference's): diagnostic builds only"
#endif
#if defined(RTW_DIAG_FAR) && !defined(RTW_ALLOW_NON_REFERENCE)
#error "RTW_DIAG_FAR removes parts of the far-origin walk (timing diagnostic): diagnostic builds only"
#endif
#if defined(RTW_DIAG_NO_STORE) && !defined(RTW_ALLOW_NON_REFERENCE)
#error "RTW_DIAG_NO_STORE drops the sample stores (the image is not computed): diagnostic builds only"
#endif
#if defined(RTW_RNG_PLUS) || defined(RTW_RECT_RCP) || defined(RTW_SPH_RCP) || defined(RTW_FAST_RCP) || \
    defined(RTW_DIEL_PRE) || defined(RTW_START_LDS) || defined(RTW_RECT_SELECT)
#error "removed compile-time switch (round 4): the kernel has one code path for it"
#endif

constexpr float TMIN = 0.001f;  // lib.rs:102
constexpr int BLOCK = 256;
// LDS traversal-stack entries per lane (+ 1 scratch row).  At the 5 waves/SIMD the default
// variants are register-allocated for, 160 KB of LDS per CU holds 5 blocks of 256 lanes x 25 rows;
// a tree whose worst-case push bound (Flat::stack_need) is deeper keeps the excess in HBM
// (RenderArgs::spill).  STACK_LDS (33 rows) is for the 4-waves/SIMD tuning variants.
constexpr int STACK_LDS = 32;
constexpr int STACK_LDS5 = 24;
// Deep-tree variants (mesh scenes): 31 rows x 256 lanes x 4 B x 5 blocks = 158,720 B <= 160 KiB, so a
// push bound up to 30 (cow 25, monument 30) stays in LDS at 5 waves/SIMD without the spill path.
constexpr int STACK_DEEP5 = 30;

struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 scale(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 divs(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Correctly rounded f32 sqrt for x in [2^-96, inf): the backend's own expansion of sqrtf (v_sqrt_f32,
// then the +-1 ulp residual corrections) without its small-input scaling and special-value fix-up,
// which select the unscaled, uncorrected result for exactly these inputs -- the same bits, 7 fewer
// VALU ops.  tests/test_gpu_parity.py checks it against IEEE sqrt on the device.
__device__ __forceinline__ float sqrt_rn_big(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
  const float sup = __uint_as_float(__float_as_uint(s) + 1u);
  const float s1 = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
  return __builtin_fmaf(-sup, s, x) > 0.0f ? sup : s1;
}
__device__ __forceinline__ float sqrt_rn(float x) {  // = sqrtf(x) for every x
  float r = sqrt_rn_big(x);
  if (__builtin_expect(!(x >= 0x1p-96f && x < INFINITY), 0)) r = sqrtf(x);
  return r;
}
#ifndef RTW_NT_SAMPLES
#define RTW_NT_SAMPLES 1  // the sample buffer written with non-temporal stores
#endif
__device__ __forceinline__ bool near_zero(V3 a) {                                   // vec3.rs:133-138
  return fabsf(a.x) < 1e-8f && fabsf(a.y) < 1e-8f && fabsf(a.z) < 1e-8f;
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }  // :140-142
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float eta) {                                  // :144-151
  float cos_t = fminf(dot(neg(uv), n), 1.0f);
  V3 perp = scale(add(uv, scale(n, cos_t)), eta);
  float k = -sqrtf(fabsf(1.0f - len2(perp)));
  return add(perp, scale(n, k));
}
__device__ __forceinline__ V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

// ---- RNG: xoroshiro64* per path (state s0 | s1 << 32, never 0) seeded by
// splitmix64(splitmix64(seed) ^ (j << 48 | i << 32 | sample)); rand 0.9 float conversions
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t xoro_seed(uint64_t h) { return h ? h : 0x9E3779B97F4A7C15ull; }
// one 32-bit multiply + 5 shift/rotate/xor ops per draw (the round-1 PCG32 step was a 64-bit
// multiply: 3 quarter-rate VALU ops)
__device__ __forceinline__ uint32_t rng_next(uint64_t& s) {
  uint32_t s0 = (uint32_t)s, s1 = (uint32_t)(s >> 32);
  const uint32_t result = s0 * 0x9E3779BBu;
  s1 ^= s0;
  s0 = __builtin_amdgcn_alignbit(s0, s0, 6) ^ s1 ^ (s1 << 9);  // rotl(s0, 26)
  s1 = __builtin_amdgcn_alignbit(s1, s1, 19);                   // rotl(s1, 13)
  s = ((uint64_t)s1 << 32) | s0;
  return result;
}
// (u >> 9) | 0x3F800000 (= 1.0f's bits: the float in [1, 2) with u's top 23 bits as mantissa) in one
// v_alignbit_b32: the low word of the 64-bit (0x7F : u) >> 9.  Inline asm: the compiler turns the builtin
// back into a shift and an or (two VALU ops per draw in the rejection loops).  AB = false keeps the shift and
// the or: the asm statement changed the triangle kernels' register allocation (MI355X A/B,
// profiles/r03/experiments r03t: jumpy +0.6%, cornell +1.0%, cow -2.4%, monument -1.2%), so only the
// sphere and list-mode kernels use it (the same split as start_path's LDS operands, SLDS).
template <bool AB>
__device__ __forceinline__ uint32_t one_mant23(uint32_t u) {
  if constexpr (!AB) return (u >> 9) | 0x3F800000u;
  uint32_t r;
  asm("v_alignbit_b32 %0, %1, %2, 9" : "=v"(r) : "s"(0x7Fu), "v"(u));
  return r;
}
__device__ __forceinline__ float gen_f32(uint64_t& s) {  // rand Standard<f32>
  return (float)(rng_next(s) >> 8) * (1.0f / 16777216.0f);
}
template <bool AB>
__device__ __forceinline__ float gen_range(uint64_t& s, float lo, float hi, float sc) {
  // UniformFloat::sample_single with sc = hi - lo precomputed (kernel-uniform: stays in an SGPR)
  for (;;) {
    float v01 = __uint_as_float(one_mant23<AB>(rng_next(s))) - 1.0f;
    float r = v01 * sc + lo;
    if (r < hi) return r;
    sc = __uint_as_float(__float_as_uint(sc) - 1u);
  }
}
// gen_range(s, -1, 1) without the retry loop: v12 = 1 + m 2^-23 (m < 2^23), and
// (v12 - 1) * 2 + -1 = 2 v12 - 3 = (m - 2^22) 2^-22 is exact in both forms and at most 1 - 2^-22 < 1,
// so the retry never fires (checked for every m in tests/test_oracle_kat.py::test_pm1_never_retries)
// and one exact fma gives the oracle's bits.
template <bool AB>
__device__ __forceinline__ float gen_pm1(uint64_t& s) {
  const float v12 = __uint_as_float(one_mant23<AB>(rng_next(s)));
  return __builtin_fmaf(v12, 2.0f, -3.0f);
}
template <bool AB>
__device__ __forceinline__ V3 rand_in_unit_sphere(uint64_t& s) {  // vec3.rs:101-108
  for (;;) {
    float x = gen_pm1<AB>(s);
    float y = gen_pm1<AB>(s);
    float z = gen_pm1<AB>(s);
    V3 p = mk(x, y, z);
#ifdef RTW_DIAG_ONE_TRIP  // timing diagnostic only (not the reference's distribution): no rejection tail
    return p;
#endif
    if (len2(p) < 1.0f) return p;
  }
}
template <bool AB>
__device__ __forceinline__ V3 rand_in_unit_disk(uint64_t& s) {  // vec3.rs:124-131
  for (;;) {
    float x = gen_pm1<AB>(s);
    float y = gen_pm1<AB>(s);
    V3 p = mk(x, y, 0.0f);
    if (len2(p) < 1.0f) return p;
  }
}

// ---- f32 transcendentals, correctly rounded: evaluated in double with polynomials of error
// < 2^-60 and rounded once (the oracle's §libm restates the same algorithm; tests pin GPU ==
// oracle == (float)glibc-double).  Only IEEE double + - * / sqrt floor: no FMA contraction
// (-ffp-contract=off), so the bits are the oracle's.
__device__ __forceinline__ double ln_core(double m) {  // 2 atanh((m-1)/(m+1)), m in [sqrt(1/2), sqrt(2)]
  const double s = (m - 1.0) / (m + 1.0), z = s * s;
  double p = 1.0 / 23.0;
  p = p * z + 1.0 / 21.0; p = p * z + 1.0 / 19.0; p = p * z + 1.0 / 17.0; p = p * z + 1.0 / 15.0;
  p = p * z + 1.0 / 13.0; p = p * z + 1.0 / 11.0; p = p * z + 1.0 / 9.0; p = p * z + 1.0 / 7.0;
  p = p * z + 1.0 / 5.0; p = p * z + 1.0 / 3.0; p = p * z + 1.0;
  return 2.0 * s * p;
}
__device__ __forceinline__ float dev_log10f(float x) {  // f32::log10
  if (x != x) return x;
  if (x == 0.0f) return -INFINITY;
  if (x < 0.0f) return NAN;
  if (isinf(x)) return x;
  const uint64_t u = (uint64_t)__double_as_longlong((double)x);
  int e = (int)((u >> 52) & 0x7ff) - 1023;
  double m = __longlong_as_double((long long)((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
  if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
  const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  const double INV_LN10 = 0.43429448190325182765;
  const double lnx = ((double)e * LN2_HI + ln_core(m)) + (double)e * LN2_LO;
  return (float)(lnx * INV_LN10);
}
__device__ __forceinline__ double sin_core(double r) {
  const double z = r * r;
  double p = -1.0 / 1307674368000.0;
  p = p * z + 1.0 / 6227020800.0; p = p * z - 1.0 / 39916800.0; p = p * z + 1.0 / 362880.0;
  p = p * z - 1.0 / 5040.0; p = p * z + 1.0 / 120.0; p = p * z - 1.0 / 6.0;
  return r + r * z * p;
}
__device__ __forceinline__ double cos_core(double r) {
  const double z = r * r;
  double p = 1.0 / 20922789888000.0;
  p = p * z - 1.0 / 87178291200.0; p = p * z + 1.0 / 479001600.0; p = p * z - 1.0 / 3628800.0;
  p = p * z + 1.0 / 40320.0; p = p * z - 1.0 / 720.0; p = p * z + 1.0 / 24.0; p = p * z - 0.5;
  return 1.0 + z * p;
}
__device__ __forceinline__ float dev_sinf(float x) {  // f32::sin
  if (x != x || x == 0.0f) return x;  // keeps the sign of zero
  if (isinf(x)) return NAN;
  const double d = x;
  const double TWO_OVER_PI = 6.36619772367581382433e-01;
  const double P1 = 1.57079632673412561417e+00, P2 = 6.07710050650619224932e-11, P3 = 2.02226624879595063154e-21;
  const double k = floor(d * TWO_OVER_PI + 0.5);
  const double r = ((d - k * P1) - k * P2) - k * P3;
  const double q = k - 4.0 * floor(k * 0.25);
  const double v = q == 0.0 ? sin_core(r) : (q == 1.0 ? cos_core(r) : (q == 2.0 ? -sin_core(r) : -cos_core(r)));
  return (float)v;
}
__device__ __forceinline__ double atan_core(double t) {  // |t| <= tan(pi/16)
  const double z = t * t;
  double p = -1.0 / 29.0;
  p = p * z + 1.0 / 27.0; p = p * z - 1.0 / 25.0; p = p * z + 1.0 / 23.0; p = p * z - 1.0 / 21.0;
  p = p * z + 1.0 / 19.0; p = p * z - 1.0 / 17.0; p = p * z + 1.0 / 15.0; p = p * z - 1.0 / 13.0;
  p = p * z + 1.0 / 11.0; p = p * z - 1.0 / 9.0; p = p * z + 1.0 / 7.0; p = p * z - 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  return t - t * z * p;
}
__device__ __forceinline__ double atan01(double a) {  // 0 <= a <= 1
  const double T1 = 0.19891236737965800691, T3 = 0.66817863791929891999, C1 = 0.41421356237309504880;
  const double PI_8 = 0.39269908169872415481, PI_4 = 0.78539816339744830962;
  if (a <= T1) return atan_core(a);
  if (a <= T3) return PI_8 + atan_core((a - C1) / (1.0 + a * C1));
  return PI_4 + atan_core((a - 1.0) / (1.0 + a));
}
__device__ __forceinline__ double atan2_pos(double y, double x) {  // y > 0 finite, x finite non-zero
  const double PI = 3.14159265358979323846, PI_2 = 1.57079632679489661923;
  const double ax = fabs(x);
  const double r = y <= ax ? atan01(y / ax) : PI_2 - atan01(ax / y);
  return x < 0.0 ? PI - r : r;
}
__device__ __forceinline__ float dev_atan2f(float y, float x) {  // f32::atan2, C99 Annex F special cases
  const double PI = 3.14159265358979323846, PI_2 = 1.57079632679489661923, PI_4 = 0.78539816339744830962;
  if (x != x || y != y) return x + y;
  const bool sx = signbit(x), sy = signbit(y);
  double r;
  if (y == 0.0f) r = sx ? PI : 0.0;
  else if (isinf(x)) r = isinf(y) ? (sx ? 3.0 * PI_4 : PI_4) : (sx ? PI : 0.0);
  else if (x == 0.0f || isinf(y)) r = PI_2;
  else r = atan2_pos(fabs((double)y), (double)x);
  return (float)(sy ? -r : r);
}
__device__ __forceinline__ float dev_acosf(float x) {  // f32::acos = atan2(sqrt((1-x)(1+x)), x)
  if (x != x) return x;
  if (!(fabsf(x) <= 1.0f)) return NAN;
  const double d = x, s = sqrt((1.0 - d) * (1.0 + d));
  if (s == 0.0) return d > 0.0 ? 0.0f : (float)3.14159265358979323846;
  return (float)atan2_pos(s, d);
}

struct Ray { V3 o, d; float time; };

// ---- wrapper chains (transformations.rs:23-38, :115-135): world ray -> object ray
// Wave-uniform loads of scene tables through the constant address space: the backend emits scalar
// loads (s_load, scalar cache) instead of 64-lane vector loads of one address, which kept the
// vector-memory units of the list-mode kernel busy (cornell-box: TA 94%, TD 99%).  Reads only: the
// kernel never writes the scene tables.
template <class T>
__device__ __forceinline__ T uload(const T* p) {
  if constexpr (sizeof(T) == 16) {  // HIP vector types: load the native 4 x 32-bit vector
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 v = *(const __attribute__((address_space(4))) u4*)(p);
    T t;
    __builtin_memcpy(&t, &v, 16);
    return t;
  } else {
    return *(const __attribute__((address_space(4))) T*)(p);
  }
}

// a wrapper op's kind (op.x holds (float)IO_TRANSLATE or (float)IO_ROTY, rtw_flatten.cpp) compared as bits: an
// integer compare, which a kernel-uniform op does on the scalar unit (a float compare is a VALU op plus an exec and)
__device__ __forceinline__ bool op_is(float x, uint32_t kind) { return __float_as_uint(x) == __float_as_uint((float)kind); }

template <bool UNI = false>
__device__ __forceinline__ Ray to_local(const DevInst* in, Ray r) {
  const uint32_t n = UNI ? uload(&in->nops) : in->nops;
  for (uint32_t k = 0; k < n; ++k) {
    const float4* opp = reinterpret_cast<const float4*>(in->op[k]);
    const float4 op = UNI ? uload(opp) : *opp;
    if (op_is(op.x, IO_TRANSLATE)) {
      r.o = sub(r.o, mk(op.y, op.z, op.w));
    } else {
      const float s = op.y, c = op.z;
      r.o = mk(c * r.o.x - s * r.o.z, r.o.y, s * r.o.x + c * r.o.z);
      r.d = mk(c * r.d.x - s * r.d.z, r.d.y, s * r.d.x + c * r.d.z);
    }
  }
  return r;
}

// RN(x / b) from y = RN(1 / b) by Markstein's correction (q0 = RN(x y) is within an ulp of x / b, the
// residual r = x - q0 b is exact in one fma, and RN(q0 + r y) = RN(x / b); Markstein 1990, no
// underflow or overflow): the camera's u, v divisions (lib.rs:84-85), whose divisors w - 1, h - 1 are
// integers in [1, 65535] and dividends 0 or in [2^-24, 65536), with y computed exactly on the host.
// Three VALU ops instead of the ~10 of an IEEE division; tests/test_gpu_parity.py checks it against
// IEEE division on the device.
__device__ __forceinline__ float div_by_recip(float x, float b, float y) {
  const float q0 = x * y;
  const float r = __builtin_fmaf(-q0, b, x);
  return __builtin_fmaf(r, y, q0);
}
// RN(1 / b) in three VALU ops: the hardware reciprocal (v_rcp_f32, within 1 ulp) refined by one Newton
// step with an exact residual, e = 1 - b y0 (fma), y1 = RN(y0 + e y0).  Equal to the IEEE quotient 1.0f / b
// for every b with |b| in [2^-126, 2^126] (normal b whose reciprocal is normal): checked on the device over
// all 2^32 bit patterns (rtw_diag_sweep 0, tests/test_gpu_parity.py), which is the proof, since v_rcp_f32
// is a fixed function of its input.  Callers guard the range (rcp_rn_ok) and divide otherwise.
__device__ __forceinline__ float rcp_rn_fast(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y0, 1.0f);
  return __builtin_fmaf(e, y0, y0);
}
__device__ __forceinline__ bool rcp_rn_ok(float b) {
  const float ab = fabsf(b);
  return ab >= 0x1p-126f && ab <= 0x1p126f;
}
__device__ __forceinline__ float rcp_rn(float b) {  // = 1.0f / b for every b
  float y = rcp_rn_fast(b);
  if (__builtin_expect(!rcp_rn_ok(b), 0)) y = 1.0f / b;
  return y;
}
// RN(x / b) from y = RN(1 / b) with the range guard of the sphere roots: Markstein's correction is the IEEE
// quotient wherever b is in [2^-60, 2^60] and |x| < 2^64 and the quotient is normal, and below 2^-126 both
// are tiny (< TMIN); other lanes divide.
__device__ __forceinline__ bool recip_div_ok(float b) {
  const float ab = fabsf(b);
  return ab >= 0x1p-60f && ab <= 0x1p60f;
}
__device__ __forceinline__ float div_rcp(float x, float b, float y, bool b_ok) {
  float t = div_by_recip(x, b, y);
  if (__builtin_expect(!(b_ok && fabsf(x) < 0x1p64f), 0)) t = x / b;
  return t;
}
// vec3.rs:85-87 unit_vector: a / |a|.  |a| = sqrt_rn (IEEE sqrt); the three divisions share the divisor, so
// one rcp_rn and three corrections; |a.k| <= |a| needs no numerator guard.
__device__ __forceinline__ V3 unit(V3 a) {
  const float s = sqrt_rn(len2(a));
  const float y = rcp_rn_fast(s);
  V3 r = mk(div_by_recip(a.x, s, y), div_by_recip(a.y, s, y), div_by_recip(a.z, s, y));
  if (__builtin_expect(!recip_div_ok(s), 0)) r = divs(a, s);
  return r;
}

// ---- candidate t of one primitive (independent of t_max; -1 = miss)
// rad2 = radius * radius (precomputed for moving spheres; the same f32 product)
__device__ __forceinline__ float cand_sphere(const Ray& r, V3 c, float rad2) {  // spherical.rs:26-44
  V3 oc = sub(r.o, c);
  float a = len2(r.d);
  float hb = dot(oc, r.d);
  float cc = len2(oc) - rad2;
  float disc = hb * hb - a * cc;
  if (disc < 0.0f) return -1.0f;  // spherical.rs:32: a NaN discriminant goes on (a NaN root, a hit in list mode)
  float sq = sqrtf(disc);
  float root = (-hb - sq) / a;
  if (root < TMIN) root = (-hb + sq) / a;  // root1 > t_max implies root2 > t_max
  return root;
}
// The same test with the ray's a = |d|^2 and y = RN(1 / a) computed once per traversal (SphRcp): each
// root is Markstein's correction div_by_recip (3 VALU) instead of an IEEE division (~10).  Equal to
// the IEEE quotient whenever a is in [2^-60, 2^60] and |numerator| < 2^64 (then the quotient is finite,
// and wherever it is normal the correction is exact; below 2^-126 both are < TMIN); other lanes divide.
struct SphRcp { float a, ya; bool ok; };
__device__ __forceinline__ SphRcp sph_rcp(const Ray& r) {
  SphRcp q;
  q.a = len2(r.d);
  q.ya = rcp_rn_fast(q.a);  // = 1.0f / a inside the guarded range below (outside it sph_div divides)
  q.ok = q.a >= 0x1p-60f && q.a <= 0x1p60f;
  return q;
}
__device__ __forceinline__ float sph_div(float n, const SphRcp& q) {
  float t = div_by_recip(n, q.a, q.ya);
  if (__builtin_expect(!(q.ok && fabsf(n) < 0x1p64f), 0)) t = n / q.a;
  return t;
}
__device__ __forceinline__ float cand_sphere_rcp(const Ray& r, V3 c, float rad2, const SphRcp& q) {
  V3 oc = sub(r.o, c);
  float hb = dot(oc, r.d);
  float cc = len2(oc) - rad2;
  float disc = hb * hb - q.a * cc;
  if (!(disc >= 0.0f)) return -1.0f;
  float sq = sqrt_rn(disc);
  float root = sph_div(-hb - sq, q);
  if (root < TMIN) root = sph_div(-hb + sq, q);
  return root;
}
// spherical.rs:117-123 over the flattened layout q0 = (c0, r*r), q1 = (c1 - c0, r), q2 = (t0, t1)
// (rtw_flatten.cpp).  For the shutter [+0, 1] (aux = 1) the fraction (time - 0) / (1 - 0) is `time`
// exactly: when every moving sphere of the scene has it (DevScene::msphere_unit, a kernel-uniform
// branch) the IEEE division and the q2 load are skipped; otherwise each prim's t0, t1 are used.
__device__ __forceinline__ V3 center_at(float4 q0, float4 q1, const float4* P, uint32_t unit_shutter, float time) {
  float frac = time;
  if (!unit_shutter) {
    const float4 q2 = P[2];
    frac = (time - q2.x) / (q2.y - q2.x);
  }
  return add(mk(q0.x, q0.y, q0.z), scale(mk(q1.x, q1.y, q1.z), frac));
}
template <int AXIS, bool SEL = false>  // 0 XY, 1 XZ, 2 YZ — rectangular.rs:33-41, :84-92, :135-143
__device__ __forceinline__ float cand_rect(const Ray& r, const float* q0, float k) {
  const float o_k = AXIS == 0 ? r.o.z : (AXIS == 1 ? r.o.y : r.o.x);
  const float d_k = AXIS == 0 ? r.d.z : (AXIS == 1 ? r.d.y : r.d.x);
  const float o_a = AXIS == 2 ? r.o.y : r.o.x, d_a = AXIS == 2 ? r.d.y : r.d.x;
  const float o_b = AXIS == 0 ? r.o.y : r.o.z, d_b = AXIS == 0 ? r.d.y : r.d.z;
  float t = (k - o_k) / d_k;
  if constexpr (SEL) {
    // the same decisions as selects (x, y have no side effects): no exec-mask branches in the list loop
    const float x = o_a + t * d_a;
    const float y = o_b + t * d_b;
    const bool out = (t < TMIN) | (x < q0[0]) | (x > q0[1]) | (y < q0[2]) | (y > q0[3]);
    return out ? -1.0f : t;
  }
  if (t < TMIN) return -1.0f;
  float x = o_a + t * d_a;
  float y = o_b + t * d_b;
  if (x < q0[0] || x > q0[1] || y < q0[2] || y > q0[3]) return -1.0f;
  return t;
}
struct TriUV { float t, u, v; };
__device__ __forceinline__ TriUV tri_solve(const Ray& r, const float* q) {  // triangular.rs:98-118
  V3 a = mk(q[0], q[1], q[2]), ab = mk(q[3], q[4], q[5]), ac = mk(q[6], q[7], q[8]);
  V3 n = mk(q[9], q[10], q[11]);
  float det = -dot(r.d, n);
  float inv = rcp_rn(det);  // triangular.rs:105 `1.0 / determinant`, the IEEE reciprocal
  V3 ao = sub(r.o, a);
  V3 aoxd = cross(ao, r.d);
  TriUV o;
  o.u = dot(ac, aoxd) * inv;
  o.v = -dot(ab, aoxd) * inv;
  o.t = dot(ao, n) * inv;
  return o;
}
__device__ __forceinline__ float cand_tri(const Ray& r, const float* q) {
  TriUV s = tri_solve(r, q);
  if (s.t < TMIN) return -1.0f;
  if (!(s.t >= 0.0f && s.u >= 0.0f && s.v >= 0.0f && (s.u + s.v) <= 1.0f)) return -1.0f;
  return s.t;
}
__device__ __forceinline__ float cand_tri_uv(const Ray& r, const float* q, float& u, float& v) {
  TriUV s = tri_solve(r, q);
  u = s.u;
  v = s.v;
  if (s.t < TMIN) return -1.0f;
  if (!(s.t >= 0.0f && s.u >= 0.0f && s.v >= 0.0f && (s.u + s.v) <= 1.0f)) return -1.0f;
  return s.t;
}

struct Best {
  float t;
  uint32_t key;
  int32_t prim;
  float u, v;  // a triangle winner's barycentrics (tri_solve's, triangular.rs:109-112): the hit record reuses them
};

// ConstantMedium::hit (volumes.rs:37-78) in the order-independent form the oracle defines (K_MEDIUM):
// boundary entry / exit by the reference's own hit routines with t in (-inf, inf) and
// (rec1 + 0.0001, inf), distance test against the unclipped exit, and the draw from a sub-stream
// keyed by (segment state, leaf key).  -1 = no hit.
template <uint32_t FEAT>
__device__ __forceinline__ float cand_medium(const DevScene& S, const Ray& lr, const float4* P, uint32_t key,
                                          uint32_t inner, uint64_t seg) {
  const float4 q0v = P[0], q1v = P[1], q2v = P[2];
  const Ray br = ((FEAT & F_INST) && inner) ? to_local(S.insts + inner, lr) : lr;
  float r1, r2;
  if (q2v.y == 0.0f) {  // Sphere boundary: spherical.rs:18-60 twice
    const V3 oc = sub(br.o, mk(q0v.x, q0v.y, q0v.z));
    const float a = len2(br.d), hb = dot(oc, br.d), cc = len2(oc) - q0v.w * q0v.w;
    const float disc = hb * hb - a * cc;
    if (disc < 0.0f) return -1.0f;
    const float sq = sqrtf(disc);
    const float root1 = (-hb - sq) / a, root2 = (-hb + sq) / a;
    float rt = root1;
    if (rt < -INFINITY || INFINITY < rt) {
      rt = root2;
      if (rt < -INFINITY || INFINITY < rt) return -1.0f;
    }
    r1 = rt;
    const float lo = r1 + 0.0001f;
    rt = root1;
    if (rt < lo || INFINITY < rt) {
      rt = root2;
      if (rt < lo || INFINITY < rt) return -1.0f;
    }
    r2 = rt;
  } else {  // Cuboid boundary: its six rects (rectangular.rs:177-240) as a closest-hit list, twice
    const float p0[3] = {q0v.x, q0v.y, q0v.z}, p1[3] = {q1v.x, q1v.y, q1v.z};
    const float o[3] = {br.o.x, br.o.y, br.o.z}, d[3] = {br.d.x, br.d.y, br.d.z};
    float ts[6];
    bool inb[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int axis = k >> 1;  // XY, XY, XZ, XZ, YZ, YZ; k on z / y / x, far side first
      const int kx = axis == 0 ? 2 : (axis == 1 ? 1 : 0), ax = axis == 2 ? 1 : 0, bx = axis == 0 ? 1 : 2;
      const float kk = (k & 1) ? p0[kx] : p1[kx];
      const float t = (kk - o[kx]) / d[kx];
      const float x = o[ax] + t * d[ax], y = o[bx] + t * d[bx];
      ts[k] = t;
      inb[k] = !(x < p0[ax] || x > p1[ax] || y < p0[bx] || y > p1[bx]);
    }
    float closest = INFINITY;
    bool any = false;
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (inb[k] && !(ts[k] < -INFINITY || ts[k] > closest)) { closest = ts[k]; any = true; }
    if (!any) return -1.0f;
    r1 = closest;
    const float lo = r1 + 0.0001f;
    closest = INFINITY;
    any = false;
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (inb[k] && !(ts[k] < lo || ts[k] > closest)) { closest = ts[k]; any = true; }
    if (!any) return -1.0f;
    r2 = closest;
  }
  float t1 = fmaxf(r1, TMIN);
  if (t1 >= r2) return -1.0f;
  t1 = fmaxf(t1, 0.0f);
  const float len = sqrtf(len2(lr.d));
  const float dist = (r2 - t1) * len;
  uint64_t g = xoro_seed(splitmix64(seg ^ splitmix64((uint64_t)key)));
  const float hd = q2v.x * dev_log10f(gen_f32(g));
  if (hd > dist) return -1.0f;
  return t1 + hd / len;
}

// COUNT build only: wave-level SIMD utilisation.  Adds 1 to cnt[wave_slot] for the first
// active lane (one per wave execution) and the wave's active-lane count to cnt[lane_slot].
__device__ __forceinline__ void simd_tick(uint32_t* cnt, int wave_slot, int lane_slot) {
  const uint64_t m = __ballot(1);
  if ((uint32_t)__lane_id() == (uint32_t)(__ffsll((long long)m) - 1)) {
    cnt[wave_slot] += 1;
    cnt[lane_slot] += (uint32_t)__popcll(m);
  }
}

// The sphere-only kernels' branch-free 32-B test (q0 = (c0, r^2), q1 = (c1 - c0, key bits); see test_prim)
__device__ __forceinline__ void test_sphere32(const DevScene& S, uint32_t pi, float4 q0v, float4 q1v, const Ray& wr,
                                              Best& b, const SphRcp* rq) {
  const float4* P = reinterpret_cast<const float4*>(S.prims + pi);
  const V3 c = center_at(q0v, q1v, P, S.msphere_unit, wr.time);
  const float t = rq ? cand_sphere_rcp(wr, c, q0v.w, *rq) : cand_sphere(wr, c, q0v.w);
  const uint32_t key = __float_as_uint(q1v.w);
  if (t >= TMIN && t < INFINITY && (t < b.t || (t == b.t && key > b.key))) {
    b.t = t;
    b.key = key;
    b.prim = (int32_t)pi;
  }
}

// List-mode kernels (F_LIST): a winner whose t is NaN (an in-plane hit, see rect_list_test) is carried with best
// t = +inf and this bit in its index (list worlds have few prims); trace_begin hands it on with t = NaN
constexpr int32_t RECT_NAN_HIT = 0x40000000;

// LOCAL: `wr` already is the prim's object-space ray (the caller caches it per wrapper chain)
// UNI: pi is wave-uniform (the always list): scalar loads (uload)
template <bool COUNT, uint32_t FEAT, bool LOCAL = false, bool UNI = false>
__device__ __forceinline__ void test_prim(const DevScene& S, uint32_t pi, const Ray& wr, Best& b,
                                          uint32_t* cnt, uint64_t seg, const SphRcp* rq = nullptr) {
  const float4* P = reinterpret_cast<const float4*>(S.prims + pi);
  // sphere-only worlds: a static sphere is tested as a moving one with c1 - c0 = 0 (c0 + time * 0 is
  // c0 up to the sign of a zero coordinate, which changes neither the decision nor t: the zero only
  // reaches hb, whose sign matters only when every term and sqrt(disc) vanish, a root of +-0 that
  // fails t >= 0.001 either way), so one branch-free test reads q0 = (c0, r^2) and q1 = (c1 - c0,
  // key bits) -- 32 B, no type dispatch
  constexpr bool SPH_ONLY = (FEAT & (F_RECT | F_TRI | F_MEDIUM | F_INST)) == 0 && (FEAT & (F_SPHERE | F_MSPHERE));
  if constexpr (SPH_ONLY && !COUNT) {
    const float4 q0v = UNI ? uload(P) : P[0];
    const float4 q1v = UNI ? uload(P + 1) : P[1];
    test_sphere32(S, pi, q0v, q1v, wr, b, rq);
    return;
  }
  // every 16-B part the scene's primitive kinds may need is loaded up front, in one round trip:
  // loading the geometry only after the type was known cost two more dependent trips per test
  const uint4 meta = UNI ? uload(reinterpret_cast<const uint4*>(P + 3)) : *reinterpret_cast<const uint4*>(P + 3);
  const float4 q0v = UNI ? uload(P) : P[0];
  constexpr bool NEED_Q1 = (FEAT & (F_MSPHERE | F_TRI | F_RECT)) != 0, NEED_Q2 = (FEAT & F_TRI) != 0;
  const float4 q1v = NEED_Q1 ? (UNI ? uload(P + 1) : P[1]) : q0v;
  const float4 q2v = NEED_Q2 ? (UNI ? uload(P + 2) : P[2]) : q0v;
  const uint32_t type = meta.x & 0xffu, inst = meta.x >> 8;
  // rect tests and the accept as selects instead of exec-mask branches (RTW_RECT_SELECT) in the kernels
  // without triangles: cornell-800 +6.7%; the triangle kernels lost 0.6-1.4% (profiles/r03/experiments, u1)
  constexpr bool SEL = !(FEAT & F_TRI);
  // object-space ray of the prim's wrapper chain; in BVH leaves recomputed per test (a few
  // flops) rather than cached, which keeps 8 VGPRs free for occupancy
  Ray lr = wr;
  if (!LOCAL && (FEAT & F_INST) && inst) {
    if (inst == S.uni_inst)  // transformations.rs:23-38 with the kernel-uniform offset: no dependent loads
      lr.o = sub(wr.o, mk(S.uni_off[0], S.uni_off[1], S.uni_off[2]));
    else
      lr = to_local<UNI>(S.insts + inst, wr);
  }
  float q0[4] = {q0v.x, q0v.y, q0v.z, q0v.w};
  float t = -1.0f, tu = 0.0f, tv = 0.0f;
  if ((FEAT & F_SPHERE) && type == PT_SPHERE) {
    t = cand_sphere(lr, mk(q0[0], q0[1], q0[2]), q0[3]);  // q0.w = r * r (flattener, the same f32 product)
  } else if ((FEAT & F_MSPHERE) && type == PT_MSPHERE) {
    t = cand_sphere(lr, center_at(q0v, q1v, P, S.msphere_unit, lr.time), q0v.w);
  } else if ((FEAT & F_TRI) && type == PT_TRI) {
    const float q[12] = {q0v.x, q0v.y, q0v.z, q0v.w, q1v.x, q1v.y, q1v.z, q1v.w, q2v.x, q2v.y, q2v.z, q2v.w};
    t = cand_tri_uv(lr, q, tu, tv);
  } else if ((FEAT & F_MEDIUM) && type == PT_MEDIUM) {
    t = cand_medium<FEAT>(S, lr, P, meta.y, meta.w, seg);
  } else if (FEAT & F_RECT) {
    const float k = q1v.x;
    if (type == PT_RECT_XY) t = cand_rect<0, SEL>(lr, q0, k);
    else if (type == PT_RECT_XZ) t = cand_rect<1, SEL>(lr, q0, k);
    else if (type == PT_RECT_YZ) t = cand_rect<2, SEL>(lr, q0, k);
  }
  if (COUNT) { cnt[1]++; if (type < 6u) cnt[2 + type]++; simd_tick(cnt, 10, 11); }  // media: total only
  if constexpr ((FEAT & F_LIST) != 0) {
    // list mode tests in DFS-key order: the reference's own fold (hittable/mod.rs:57-69) with its comparisons,
    // which a NaN candidate passes (rectangular.rs:33-41, spherical.rs:32-43): best NaN behaves as best +inf
    // (RECT_NAN_HIT); a later object wins ties by order
    const bool acc = !(t < TMIN) & !(t > b.t);
    const bool tnan = t != t;
    b.t = acc ? (tnan ? INFINITY : t) : b.t;
    b.key = acc ? meta.y : b.key;
    b.prim = acc ? ((int32_t)pi | (tnan ? RECT_NAN_HIT : 0)) : b.prim;
    if (FEAT & F_TRI) {
      b.u = acc ? tu : b.u;
      b.v = acc ? tv : b.v;
    }
    return;
  }
  // hittable/mod.rs:61-65: accept t <= closest_so_far; a later object (larger key) wins ties
  if constexpr (SEL) {
    const bool acc = (t >= TMIN) & (t < INFINITY) & ((t < b.t) | ((t == b.t) & (meta.y > b.key)));
    b.t = acc ? t : b.t;
    b.key = acc ? meta.y : b.key;
    b.prim = acc ? (int32_t)pi : b.prim;
  } else if (t >= TMIN && t < INFINITY && (t < b.t || (t == b.t && meta.y > b.key))) {
    b.t = t;
    b.key = meta.y;
    b.prim = (int32_t)pi;
    if (FEAT & F_TRI) {
      b.u = tu;
      b.v = tv;
    }
  }
}

// A BVH leaf triangle when every leaf is a triangle of one wrapper chain (DevScene::bvh_tri): `lr` is
// already the chain's object-space ray, no type dispatch; the 48 B of geometry in three loads, and the
// tie key (DevPrim::key) only for a candidate at or below the best t (triangular.rs:97-138).
template <bool COUNT>
__device__ __forceinline__ void test_tri_leaf(const DevScene& S, uint32_t pi, const Ray& lr, Best& b, uint32_t* cnt) {
  const float4* P = reinterpret_cast<const float4*>(S.prims + pi);
  const float4 q0v = P[0], q1v = P[1], q2v = P[2];
  const float q[12] = {q0v.x, q0v.y, q0v.z, q0v.w, q1v.x, q1v.y, q1v.z, q1v.w, q2v.x, q2v.y, q2v.z, q2v.w};
  float u, v;
  const float t = cand_tri_uv(lr, q, u, v);
  if (COUNT) { cnt[1]++; cnt[2 + PT_TRI]++; simd_tick(cnt, 10, 11); }
  if (t >= TMIN && t < INFINITY && t <= b.t) {  // hittable/mod.rs:61-65, the key read only here
    const uint32_t key = reinterpret_cast<const uint4*>(P + 3)->y;
    if (t < b.t || key > b.key) {
      b.t = t;
      b.key = key;
      b.prim = (int32_t)pi;
      b.u = u;
      b.v = v;
    }
  }
}

// Conservative slab test on a padded box (culling only; never decides a hit).
__device__ __forceinline__ bool slab_test(float lx, float ly, float lz, float hx, float hy, float hz,
                                          V3 inv, V3 ood, float tmax_c, float& tnear) {
  float tx0 = __builtin_fmaf(lx, inv.x, -ood.x), tx1 = __builtin_fmaf(hx, inv.x, -ood.x);
  float ty0 = __builtin_fmaf(ly, inv.y, -ood.y), ty1 = __builtin_fmaf(hy, inv.y, -ood.y);
  float tz0 = __builtin_fmaf(lz, inv.z, -ood.z), tz1 = __builtin_fmaf(hz, inv.z, -ood.z);
  float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
  float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax_c));
  tnear = tn;
  return tn <= tf;
}

// Resumable closest-hit query.  A traversal can be suspended between two leaf phases and
// resumed in a later iteration of the path loop, so a wave does not wait for its slowest ray:
// trace_run returns as soon as `quota` lanes are done and the rest continue next time.
struct TraceState {
  Best b;
  int32_t node;  // node4 to visit next, -1 = none
  int32_t pend;  // parked leaf word ~(first << 3 | count), 0 = none
  int32_t sp;    // LDS stack depth
  bool on;       // a traversal is in progress
};

// The list-mode loop of rect worlds (cornell-box: the F_BOXES | F_LIST kernel), rectangular.rs:27-57, :78-108,
// :129-159 for every rect, hittable/mod.rs:57-69 over them.  It walks the always list as runs of one wrapper
// chain and one kind (DevScene::lgroups): per chain the object-space ray, per run one specialised loop, so a rect
// costs no chain check and no type dispatch -- the scalar unit, which one CU's four SIMDs share, had become the
// limit of this loop (~35 SALU per rect against 17 VALU, profiles/r05/experiments).
// Fast path (wave-uniform, per chain): the division (k - o_k) / d_k is Markstein's correction from
// y_k = RN(1 / d_k) (rcp_rn_fast, exact in [2^-126, 2^126]; 3 VALU instead of the IEEE division's 11), the IEEE
// quotient whenever |d_k| is in [2^-60, 2^60] and |k - o_k| < 2^64 (|k| < 2^62 for every rect, DevScene::rect_fast;
// |o_k| < 2^62 per lane): then nothing over- or underflows unless |quotient| < 2^-42, where both are < TMIN and
// rejected alike (Markstein 1990; div_by_recip).  There t, the hit point's x, y are finite or +-inf, and the
// reference's tests `t >= TMIN`, `t <= best` and `!(x < a0 || x > a1)` are med3(v, lo, hi) == v (lo <= hi holds:
// TMIN <= best always, a0 <= a1 for every rect, DevScene::rect_fast): 3 med3, 3 subtractions, one max3 and one
// compare instead of 6 compares and 5 scalar ands.  A chain where any lane of the wave is outside that range runs the reference's IEEE
// division and compares (slow path).  The list is in DFS-key order, so a later rect wins a tie: accept t <= best
// (no key compare; bt starts at the reference's t_max = inf: a fast-path t is finite).  VERDICT r4 item 3.
template <int AXIS, bool FAST>
__device__ __forceinline__ void rect_list_test(const Ray& lr, V3 y, float4 q0, float k, uint32_t pi, float& bt,
                                               int32_t& bp) {
  const float o_k = AXIS == 0 ? lr.o.z : (AXIS == 1 ? lr.o.y : lr.o.x);
  const float d_k = AXIS == 0 ? lr.d.z : (AXIS == 1 ? lr.d.y : lr.d.x);
  const float y_k = AXIS == 0 ? y.z : (AXIS == 1 ? y.y : y.x);
  const float o_a = AXIS == 2 ? lr.o.y : lr.o.x, d_a = AXIS == 2 ? lr.d.y : lr.d.x;
  const float o_b = AXIS == 0 ? lr.o.y : lr.o.z, d_b = AXIS == 0 ? lr.d.y : lr.d.z;
  const float num = k - o_k;
  bool acc;
  if constexpr (FAST) {
    const float t = div_by_recip(num, d_k, y_k);
    const float x = o_a + t * d_a;
    const float yy = o_b + t * d_b;
    // the three tests as one: each med3 equals its value exactly when in range, so the largest |med3 - value| is 0 exactly
    // when all pass (t finite; x, y finite or +-inf, and +-inf lies outside the rect's finite bounds, rect_fast: inf, a
    // rejection as the reference's).  One compare, no scalar ands (+2 VALU, -2 SALU per rect: cornell-800 +1.5%, r05z)
    const float m1 = __builtin_amdgcn_fmed3f(t, TMIN, bt), m2 = __builtin_amdgcn_fmed3f(x, q0.x, q0.y);
    const float m3 = __builtin_amdgcn_fmed3f(yy, q0.z, q0.w);
    acc = fmaxf(fmaxf(fabsf(m1 - t), fabsf(m2 - x)), fabsf(m3 - yy)) == 0.0f;
    bt = acc ? t : bt;
    bp = acc ? (int32_t)pi : bp;
  } else {
    // the reference's own comparisons, rejections that a NaN passes (rectangular.rs:33-41): a ray in the
    // rect's plane (d_k = 0, k - o_k = 0: a Lambertian bounce whose direction lost its normal component) has
    // t = 0 / 0 and hits.  The reference's best is then NaN, under which every later rect whose own test passes
    // wins -- exactly as under best = +inf -- so bt keeps +inf (never NaN: the fast path's med3 needs an ordered
    // bound) and bp carries RECT_NAN_HIT; trace_rect_list hands the winner on with t = NaN.
    const float t = num / d_k;
    const float x = o_a + t * d_a;
    const float yy = o_b + t * d_b;
    const bool out = (x < q0.x) | (x > q0.y) | (yy < q0.z) | (yy > q0.w);
    acc = !(t < TMIN) & !(t > bt) & !out;
    const bool tnan = t != t;
    bt = acc ? (tnan ? INFINITY : t) : bt;
    bp = acc ? ((int32_t)pi | (tnan ? RECT_NAN_HIT : 0)) : bp;
  }
}

// one run of rects of one kind (AXIS) and chain: the whole 64-B record in one scalar load (s_load_dwordx16)
template <bool COUNT, int AXIS, bool FAST>
__device__ __forceinline__ void rect_list_run(const DevScene& S, uint32_t first, uint32_t count, const Ray& lr, V3 y,
                                              float& bt, int32_t& bp, uint32_t* cnt) {
  // the 5 dwords a test reads (a0, a1, b0, b1, k) as one s_load_dwordx8 per 64-B record (not the whole record as
  // s_load_dwordx16): both records of a trip fit the SGPRs at once, so their loads share one wait (cornell-800 +1.1%,
  // r05z2)
  typedef uint32_t u8v __attribute__((ext_vector_type(8)));
  const __attribute__((address_space(4))) u8v* P = (const __attribute__((address_space(4))) u8v*)(S.prims + first);
  auto one = [&](const u8v& rec, uint32_t k) {
    const float4 q0 = make_float4(__uint_as_float(rec[0]), __uint_as_float(rec[1]), __uint_as_float(rec[2]),
                                  __uint_as_float(rec[3]));
    rect_list_test<AXIS, FAST>(lr, y, q0, __uint_as_float(rec[4]), first + k, bt, bp);
    if (COUNT) { cnt[1]++; cnt[2 + PT_RECT_XY + AXIS]++; simd_tick(cnt, 10, 11); }
  };
  uint32_t k = 0;
  const __attribute__((address_space(4))) u8v* Pk = P;
  for (; k + 1u < count; k += 2u, Pk += 4) {  // two rects per trip (a Cuboid's runs are pairs)
    const u8v r0 = Pk[0], r1 = Pk[2];
    one(r0, k);
    one(r1, k + 1u);
  }
  if (k < count) {
    const u8v rl = Pk[0];
    one(rl, k);
  }
}

// a whole Cuboid (GK_BOX6): its xy, xz and yz pairs back to back, no run dispatch between them
template <bool COUNT, bool FAST>
__device__ __forceinline__ void rect_box6_run(const DevScene& S, uint32_t first, const Ray& lr, V3 y, float& bt,
                                              int32_t& bp, uint32_t* cnt) {
  rect_list_run<COUNT, 0, FAST>(S, first, 2u, lr, y, bt, bp, cnt);
  rect_list_run<COUNT, 1, FAST>(S, first + 2u, 2u, lr, y, bt, bp, cnt);
  rect_list_run<COUNT, 2, FAST>(S, first + 4u, 2u, lr, y, bt, bp, cnt);
}

template <bool COUNT>
__device__ __forceinline__ void trace_rect_list(const DevScene& S, const Ray& r, Best& best, uint32_t* cnt) {
  float bt = INFINITY;  // lib.rs:102 t_max
  int32_t bp = -1;
  uint32_t cur = 0xFFFFFFFFu;
  Ray lr = r;
  V3 y = mk(0.f, 0.f, 0.f);
  bool fast = false;
  for (uint32_t g = 0; g < S.n_lgroups; ++g) {
    const uint4 G = uload(reinterpret_cast<const uint4*>(S.lgroups + g));  // (first, count, instance, kind)
    if (G.z != cur) {  // wave-uniform
      cur = G.z;
      lr = r;
      if (cur) {  // a Cuboid's rotate_y + translate: both ops' loads at once, one wait (to_local's ops in order;
                  // cornell-800 +0.8%, r05z10)
        const DevInst* I = S.insts + cur;
        const uint32_t n = uload(&I->nops);
        const float4 op0 = uload(reinterpret_cast<const float4*>(I->op[0]));
        const float4 op1 = uload(reinterpret_cast<const float4*>(I->op[1]));
        auto apply = [&](const float4& op) {
          if (op_is(op.x, IO_TRANSLATE)) {
            lr.o = sub(lr.o, mk(op.y, op.z, op.w));
          } else {
            const float sn = op.y, c = op.z;
            lr.o = mk(c * lr.o.x - sn * lr.o.z, lr.o.y, sn * lr.o.x + c * lr.o.z);
            lr.d = mk(c * lr.d.x - sn * lr.d.z, lr.d.y, sn * lr.d.x + c * lr.d.z);
          }
        };
        if (n >= 1u) apply(op0);
        if (n >= 2u) apply(op1);
        for (uint32_t k = 2; k < n; ++k) apply(uload(reinterpret_cast<const float4*>(I->op[k])));
      }
      y = mk(rcp_rn_fast(lr.d.x), rcp_rn_fast(lr.d.y), rcp_rn_fast(lr.d.z));
      // the fast path's ranges (|d_k| in [2^-60, 2^60], |o_k| < 2^62), tested stricter on sums (a NaN or infinite
      // component makes its sum fail; a sum within the bound bounds each term): three compares instead of nine and
      // two scalar ands instead of eight (cornell-800 +1.9%, r05z7); a stricter test only sends more lanes to the
      // IEEE path
      const float dmin = fminf(fminf(fabsf(lr.d.x), fabsf(lr.d.y)), fabsf(lr.d.z));
      const float dsum = (fabsf(lr.d.x) + fabsf(lr.d.y)) + fabsf(lr.d.z);
      const float osum = (fabsf(lr.o.x) + fabsf(lr.o.y)) + fabsf(lr.o.z);
      const bool ok = (dmin >= 0x1p-60f) & (dsum <= 0x1p60f) & (osum < 0x1p62f);
      fast = S.rect_fast && __ballot(!ok) == 0;
    }
    if (fast) {
      if (G.w == GK_BOX6) rect_box6_run<COUNT, true>(S, G.x, lr, y, bt, bp, cnt);
      else if (G.w == PT_RECT_XY) rect_list_run<COUNT, 0, true>(S, G.x, G.y, lr, y, bt, bp, cnt);
      else if (G.w == PT_RECT_XZ) rect_list_run<COUNT, 1, true>(S, G.x, G.y, lr, y, bt, bp, cnt);
      else rect_list_run<COUNT, 2, true>(S, G.x, G.y, lr, y, bt, bp, cnt);
    } else {
      if (G.w == GK_BOX6) rect_box6_run<COUNT, false>(S, G.x, lr, y, bt, bp, cnt);
      else if (G.w == PT_RECT_XY) rect_list_run<COUNT, 0, false>(S, G.x, G.y, lr, y, bt, bp, cnt);
      else if (G.w == PT_RECT_XZ) rect_list_run<COUNT, 1, false>(S, G.x, G.y, lr, y, bt, bp, cnt);
      else rect_list_run<COUNT, 2, false>(S, G.x, G.y, lr, y, bt, bp, cnt);
    }
  }
  // an in-plane hit won (RECT_NAN_HIT; bp < 0 = no hit): the reference's t is NaN
  const bool nan_hit = bp >= 0 && (bp & RECT_NAN_HIT) != 0;
  best.t = nan_hit ? __builtin_nanf("") : bt;
  best.prim = nan_hit ? (bp & ~RECT_NAN_HIT) : bp;
}

// ---- far-origin rays (round 6; rtw_flatten.cpp's header)
// The BVH's sphere leaves are padded for origins within D0 of every BVH point.  From farther away (a path bouncing
// inside the r = 1000 ground sphere: ~5% of jumpy-balls' segments) the reference's f32 sphere test "hits" a sphere
// up to delta(D) outside it (its cancellation grows with D²), and its flat list finds such a hit wherever it lies.
// trace_begin tests the BVH box grown by delta(D) first -- almost every far ray misses it and skips the BVH -- and
// the rest (~5e-5 of jumpy-balls' segments) walk the tree here with every box grown by delta(D): a stack walk over
// the f32 node table (order never changes the answer: closest t, ties to the larger key) that descends into the
// nearest child hit, the lane's own LDS stack column as its stack (its main walk has not started), each hit leaf's
// primitives tested in turn.  A push past the column (never for a tree whose stack bound fits it) sends the lane
// through every BVH primitive.  Inlined into the main kernels, where the segment starts (profiles/r06/experiments:
// a far-path kernel that replayed the few paths needing it cost the same at 1080p but added its tail, one path's
// latency, to every frame: configs[0] -30%).
// The DevFar record, DEVFAR_BACK bytes before the prim table, re-derived at each use (the asm hides the pointer's
// provenance): otherwise the compiler hoists its ~20 kernel-uniform values into SGPRs held across the whole path
// loop, which spilled other SGPRs into VGPR lanes (v_readlane / v_writelane in the hot loop: jumpy-1080p -7%)
__device__ __forceinline__ const DevFar* far_record(const DevScene& S) {
  const char* p = reinterpret_cast<const char*>(S.prims);
  asm volatile("" : "+s"(p));
  return reinterpret_cast<const DevFar*>(p - DEVFAR_BACK);
}
__device__ __forceinline__ float far_inv(float d) {  // trace_run's reciprocal (culling only)
  const float dd = fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d);
  return __builtin_amdgcn_rcpf(dd);
}
template <bool COUNT, uint32_t FEAT, int STACK, int BLK, bool C16, int NCAP>
__device__ void trace_far(const DevScene& S, const Ray& r, Best& b, float delta, uint16_t* stk16, int32_t* stk,
                          uint32_t* cnt, uint64_t seg, uint32_t* err, const float4* lnodes) {
  const DevFar* const FR = far_record(S);
  // the f32 node table: the workgroup's LDS copy in the LDS-node kernels, else global memory
  const char* const NB = NCAP > 0 ? reinterpret_cast<const char*>(lnodes)
                                  : reinterpret_cast<const char*>(S.prims) - uload(&FR->nodes_back);
  const uint32_t n_bvh = uload(&FR->n_bvh);
  const V3 inv = mk(far_inv(r.d.x), far_inv(r.d.y), far_inv(r.d.z));
  const V3 ood = mk(r.o.x * inv.x, r.o.y * inv.y, r.o.z * inv.z);
  // every box grown by delta: its near plane delta |inv| earlier, its far plane delta |inv| later
  const V3 bn = mk(-ood.x - delta * fabsf(inv.x), -ood.y - delta * fabsf(inv.y), -ood.z - delta * fabsf(inv.z));
  const V3 bf = mk(-ood.x + delta * fabsf(inv.x), -ood.y + delta * fabsf(inv.y), -ood.z + delta * fabsf(inv.z));
  const uint32_t nx = inv.x < 0.f ? 16u : 0u, ny = (inv.y < 0.f ? 16u : 0u) + 32u, nz = (inv.z < 0.f ? 16u : 0u) + 64u;
  const uint32_t fx = nx ^ 16u, fy = ny ^ 16u, fz = nz ^ 16u;
  int32_t node = 0, sp = 0;
  bool over = false;
  for (uint32_t guard = 0;; ++guard) {
    if (node < 0) {
      if (sp == 0) break;
      --sp;
      node = C16 ? (int32_t)stk16[sp * BLK] : stk[sp * BLK];
    }
    if (guard >= (1u << 20)) {  // a corrupt tree (cycle): end the walk and report, as trace_run does
      *err = 1u;
      b.prim = -2;
      return;
    }
    if (COUNT) cnt[0]++;
    const uint32_t nb = (uint32_t)node << 7;  // sizeof(DevNode4)
    const float4 qnx = *reinterpret_cast<const float4*>(NB + (nb + nx)), qfx = *reinterpret_cast<const float4*>(NB + (nb + fx));
    const float4 qny = *reinterpret_cast<const float4*>(NB + (nb + ny)), qfy = *reinterpret_cast<const float4*>(NB + (nb + fy));
    const float4 qnz = *reinterpret_cast<const float4*>(NB + (nb + nz)), qfz = *reinterpret_cast<const float4*>(NB + (nb + fz));
    // 16-bit codes (0 = empty) or the 32-bit child words (0 = empty: the root is nobody's child)
    const uint4 cw = *reinterpret_cast<const uint4*>(NB + (nb + (C16 ? 112u : 96u)));
    const float tmax_c = __builtin_fmaf(b.t, 1.0e-5f, b.t) + 1.0e-5f;
    const float NX[4] = {qnx.x, qnx.y, qnx.z, qnx.w}, FX[4] = {qfx.x, qfx.y, qfx.z, qfx.w};
    const float NY[4] = {qny.x, qny.y, qny.z, qny.w}, FY[4] = {qfy.x, qfy.y, qfy.z, qfy.w};
    const float NZ[4] = {qnz.x, qnz.y, qnz.z, qnz.w}, FZ[4] = {qfz.x, qfz.y, qfz.z, qfz.w};
    const uint32_t W[4] = {cw.x, cw.y, cw.z, cw.w};
    uint32_t hits = 0;
    // the nearest internal child hit is walked next (the others pushed): the leaves met first shrink best t
    float tnear = INFINITY;
    int kn = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float tn = fmaxf(fmaxf(fmaxf(__builtin_fmaf(NX[k], inv.x, bn.x), __builtin_fmaf(NY[k], inv.y, bn.y)),
                                   __builtin_fmaf(NZ[k], inv.z, bn.z)), 0.0f);
      const float tf = fminf(fminf(fminf(__builtin_fmaf(FX[k], inv.x, bf.x), __builtin_fmaf(FY[k], inv.y, bf.y)),
                                   __builtin_fmaf(FZ[k], inv.z, bf.z)), tmax_c);
      const bool h = W[k] != 0u && tn <= tf;
      hits |= h ? 1u << k : 0u;
      const bool inner = C16 ? (W[k] & 0x8000u) == 0u : (int32_t)W[k] >= 0;
      const bool nearer = h && inner && tn < tnear;
      tnear = nearer ? tn : tnear;
      kn = nearer ? k : kn;
    }
    node = kn < 0 ? -1 : (int32_t)(kn == 0 ? W[0] : (kn == 1 ? W[1] : (kn == 2 ? W[2] : W[3])));
    hits &= kn < 0 ? hits : ~(1u << kn);
    while (hits) {
      const int k = __builtin_ctz(hits);
      hits &= hits - 1u;
      const uint32_t w = k == 0 ? W[0] : (k == 1 ? W[1] : (k == 2 ? W[2] : W[3]));
      if (C16 ? (w & 0x8000u) != 0u : (int32_t)w < 0) {  // a leaf: its primitives now
        const uint32_t v = C16 ? w & 0xFFFFu : ~w;
        const uint32_t first = C16 ? (v >> 2) & 0x1FFFu : v >> 3, n = C16 ? (v & 3u) + 1u : v & 7u;
        for (uint32_t q = 0; q < n; ++q) test_prim<COUNT, FEAT>(S, first + q, r, b, cnt, seg);
      } else if (sp < STACK) {
        if constexpr (C16) stk16[sp * BLK] = (uint16_t)w;
        else stk[sp * BLK] = (int32_t)w;
        ++sp;
      } else {
        over = true;  // the subtree is covered by the flat pass below
      }
    }
  }
  if (over)
    for (uint32_t pi = 0; pi < n_bvh; ++pi) test_prim<COUNT, FEAT>(S, pi, r, b, cnt, seg);
}

// Kernel variants that carry the far-origin path: BVH walks that may test spheres.  Not the mesh kernels (F_MESHES):
// a mesh world with spheres in its BVH (DevScene::far_check without bvh_tri) runs the generic kernel instead
// (pick_kernel), since even unexecuted the far code cost cow-1080p 0.6% and monument-4k 0.3% (r06)
constexpr bool far_kernel_feat(uint32_t feat) {
  return !(feat & F_LIST) && (feat & (F_SPHERE | F_MSPHERE | F_MEDIUM)) && feat != F_MESHES;
}
// C16: the kernel's LDS stack holds 16-bit entries (the LDS-node and S16 walks), else 32-bit ones (stk); trace_far
// borrows the lane's column.  A lane whose segment needs the far-origin walk takes it here, instead of the main walk.
template <bool COUNT, uint32_t FEAT, int STACK = 1, int BLK = BLOCK, bool C16 = false, int NCAP = 0>
__device__ __forceinline__ void trace_begin(const DevScene& S, const Ray& r, TraceState& ts, uint32_t* cnt,
                                            uint64_t seg, uint16_t* stk16 = nullptr, int32_t* stk = nullptr,
                                            uint32_t* err = nullptr, const float4* lnodes = nullptr) {
  ts.b = Best{INFINITY, 0u, -1, 0.0f, 0.0f};
  // list-mode worlds of rects only (the F_BOXES | F_LIST kernel)
  constexpr bool RECT_LIST = (FEAT & F_LIST) && (FEAT & F_RECT) && !(FEAT & (F_SPHERE | F_MSPHERE | F_TRI | F_MEDIUM));
  if constexpr (RECT_LIST) {
    trace_rect_list<COUNT>(S, r, ts.b, cnt);
  } else if (FEAT & F_INST) {
    // the always list is wave-uniform and in DFS order, so a wrapper chain's prims are adjacent
    // (a Cuboid's 6 sides): transform the ray once per chain instead of once per prim
    uint32_t cur = 0;
    Ray lr = r;
    // the always-tested prims are the last n_always of the prim table, in order (rtw_flatten.cpp appends them
    // after the BVH's): their indices need no load from S.always, so a prim's record loads do not wait on one
    // (cornell-800 +4.7%: 18 prims per segment; cow +1.5%, monument +0.6%; experiments a1)
    const uint32_t a0 = S.n_prims - S.n_always;
    for (uint32_t k = 0; k < S.n_always; ++k) {
      const uint32_t pi = a0 + k;
      const uint32_t inst = uload(&S.prims[pi].type_inst) >> 8;
      if (inst != cur) {
        lr = inst ? to_local<true>(S.insts + inst, r) : r;
        cur = inst;
      }
      test_prim<COUNT, FEAT, true, true>(S, pi, lr, ts.b, cnt, seg);
    }
  } else {
    constexpr bool SPH_ONLY = (FEAT & (F_RECT | F_TRI | F_MEDIUM | F_INST)) == 0 && (FEAT & (F_SPHERE | F_MSPHERE));
    SphRcp rq;
    if constexpr (SPH_ONLY) rq = sph_rcp(r);
    // (the loaded index here: the computed one made the sphere kernels 1.1% slower, experiments a1)
    for (uint32_t k = 0; k < S.n_always; ++k)
      test_prim<COUNT, FEAT, false, true>(S, uload(S.always + k), r, ts.b, cnt, seg, SPH_ONLY ? &rq : nullptr);
  }
  if constexpr ((FEAT & F_LIST) && !RECT_LIST) {  // an in-plane (NaN) winner: the reference's t is NaN
    const bool nan_hit = ts.b.prim >= 0 && (ts.b.prim & RECT_NAN_HIT) != 0;
    ts.b.t = nan_hit ? __builtin_nanf("") : ts.b.t;
    ts.b.prim = nan_hit ? (ts.b.prim & ~RECT_NAN_HIT) : ts.b.prim;
  }
  // far-origin rays (above): the BVH box grown by delta(D) over [0, best], then trace_far for the few that reach it;
  // neither takes the main walk
  bool walk = true;
#if defined(RTW_DIAG_FAR)  // timing diagnostic: 1 = no far check (pads only), 2 = far lanes skip the BVH, 3 = no far walk
                          // (the slab test's result unused: removed), 5 = the slab test kept, no far walk
  constexpr int DF = RTW_DIAG_FAR;
#else
  constexpr int DF = 0;
#endif
  constexpr bool FAR = DF != 1 && far_kernel_feat(FEAT);
  if constexpr (FAR) {
    if (S.far_check) {  // kernel-uniform
      const float4* const FR = reinterpret_cast<const float4*>(far_record(S));
      const float4 mid = uload(FR), half = uload(FR + 1);  // (mid, d2), (half, q)
      const float tx = fabsf(r.o.x - mid.x) + half.x;
      const float ty = fabsf(r.o.y - mid.y) + half.y;
      const float tz = fabsf(r.o.z - mid.z) + half.z;
      const float D2 = tx * tx + ty * ty + tz * tz;  // the farthest corner of the BVH box, squared
      const bool far = D2 > mid.w;
      if (__any(far)) {
        bool need = false;
        float delta = 0.0f;
        if (far && DF != 2) {
          const float4 lo = uload(FR + 2), hi = uload(FR + 3), e = uload(FR + 4);  // (lo, q0), (hi, s), (s0, l, l0)
          // D from v_sqrt_f32 (1 ulp) rounded up; delta grows with D
          const float D = __builtin_amdgcn_sqrtf(D2) * 1.000001f;
          delta = fminf(half.w * D2 + lo.w, hi.w * D + e.x) + (e.y * D + e.z);
          // the BVH box grown by delta, centred: |p - mid| <= half + delta per axis, over [0, best].  Raw reciprocals:
          // a zero direction component gives +-inf planes (the axis unconstrained, or a miss), and a NaN (0 * inf: the
          // origin exactly on a grown plane, the ray in it) drops out of fminf / fmaxf as a miss -- correct, since the
          // spurious-hit region lies strictly inside the grown box (delta has 1% to spare)
          const float ix = __builtin_amdgcn_rcpf(r.d.x), iy = __builtin_amdgcn_rcpf(r.d.y), iz = __builtin_amdgcn_rcpf(r.d.z);
          const float ox = r.o.x - mid.x, oy = r.o.y - mid.y, oz = r.o.z - mid.z;
          const float hx = half.x + delta, hy = half.y + delta, hz = half.z + delta;
          const float ax = (-hx - ox) * ix, bx = (hx - ox) * ix, ay = (-hy - oy) * iy, by = (hy - oy) * iy;
          const float az = (-hz - oz) * iz, bz = (hz - oz) * iz;
          const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
          const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)),
                                 fminf(fmaxf(az, bz), __builtin_fmaf(ts.b.t, 1.0e-5f, ts.b.t) + 1.0e-5f));
          need = tn <= tf;
        }
        walk = !far;
        if (DF == 5) asm volatile("" ::"v"((uint32_t)need));  // timing diagnostic: the test kept, no far walk
        if (DF != 3 && DF != 5 && __builtin_expect(__any(need), 0))
          if (need) trace_far<COUNT, FEAT, STACK, BLK, C16, NCAP>(S, r, ts.b, delta, stk16, stk, cnt, seg, err, lnodes);
      }
    }
  }
  // the root (or none) made opaque here: hoisted out of the path loop, the compiler kept it in a VGPR across the
  // whole loop and spilled it.  Triangle kernels (the mesh walk): as a scalar, since the 7-wave walk spilled even
  // the opaque VGPR copy to scratch (one reload per segment; s1)
  int32_t root = S.n_nodes ? 0 : -1;
  if constexpr ((FEAT & F_TRI) != 0) {
    root = __builtin_amdgcn_readfirstlane(root);
    asm volatile("" : "+s"(root));
  } else {
    asm volatile("" : "+v"(root));
  }
  ts.node = walk ? root : -1;
  ts.pend = 0;
  ts.sp = 0;
  ts.on = true;
}

// while-while walk of the 4-wide BVH with postponed leaves (Aila & Laine 2009): phase 1 visits
// internal nodes (nearest hit child next, the other hit children pushed); a lane that reaches a
// leaf parks it (one slot; further leaves go on the stack) and keeps walking speculatively until
// every lane of the wave holds a leaf or has run dry; phase 2 tests all parked leaves together.
// NCAP > 0: the whole node table is in the workgroup's LDS (`lnodes`, copied at kernel start), so
// the 7 node loads of a visit are ds_read_b128s instead of vector-memory loads (TA/TD were 89/98%
// busy on jumpy-balls with the nodes in L1/L2).
//
// NCAP > 0 also switches to the sorted-push walk over 16-bit stack entries (`stk16`, rows of BLK
// halfwords) of the nodes' 16-bit child codes (DevNode4::code: internal = node4 index, leaf =
// 0x8000 | first << 2 | (count - 1)), and a visit
//   * keys every hit child as (its entry distance's float bits, top 16) | code, a miss as 0,
//   * sorts the 4 keys descending (10 min/max) and writes all four codes to stack rows sp..sp+3
//     (one address, constant offsets; rows past the new top are scratch: Flat::stack_need4),
//   * walks into the nearest hit child (the smallest non-zero key) and keeps the others pushed,
//     farthest deepest; a nearest leaf is parked, or stays pushed if the parking slot is taken.
// It replaces the per-child nearest / push bookkeeping of the 32-bit walk (a visit: 97 -> 91 VALU,
// 44 of them the slab tests) and halves the stack's LDS.
// Which nodes are visited in which order never changes the answer (closest hit, ties to the
// larger key, over every leaf not culled).
// HN: the walk reads the half-precision node table (DevNode4h: 4 loads / 64 B per visit instead of 7 / 112 B)
#ifndef RTW_MESH_ROOT
#define RTW_MESH_ROOT 5  // node4s of the S16 mesh walk's LDS copy of the tree top (trace_run ROOT; 0 = none, 1 = root)
#endif
#ifndef RTW_SRING
#define RTW_SRING 1  // path starts made a ring of 64 at a time (path_kernel SRING; 0 = each lane's own, for A/B)
#endif
#ifndef REGEN_RING
#define REGEN_RING 2  // regen_min of the kernels with the start ring
#endif
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2_t as_h2(uint32_t u) { return __builtin_bit_cast(half2_t, u); }

// S16: the global-node walk keeps 16-bit stack entries (the nodes' 16-bit codes, sign-extended: leaves < 0)
// in the uint16 column `stk16`, half the LDS of the 32-bit stack (RTW_MESH_S16: more workgroups per CU)
template <bool COUNT, int STACK, bool SPILL, uint32_t FEAT, int BLK, int NCAP, bool HN = false, bool S16 = false>
__device__ void trace_run(const DevScene& S, const Ray& r, TraceState& ts, int32_t* stk, int32_t* spill,
                          uint32_t spill_lanes, uint32_t* cnt, uint32_t quota, uint32_t leaf_thr, uint64_t seg,
                          uint32_t* err, uint64_t* tph, const float4* lnodes, uint16_t* stk16) {
  constexpr bool K16 = NCAP > 0;
  constexpr bool CODES = K16 || HN || S16;  // leaves are 16-bit codes (the 32-bit walk keeps them sign-extended)
  constexpr bool SPH_ONLY = (FEAT & (F_RECT | F_TRI | F_MEDIUM | F_INST)) == 0 && (FEAT & (F_SPHERE | F_MSPHERE));
  SphRcp rq;  // once per call: the sphere roots' divisor and its reciprocal
  if constexpr (SPH_ONLY) rq = sph_rcp(r);
  // triangle-only BVH (DevScene::bvh_tri): the leaves' common object-space ray, once per call
  Ray tri_ray = r;
  if constexpr ((FEAT & F_TRI) != 0) {
    if (S.bvh_tri && (FEAT & F_INST) && S.tri_inst) {
      if (S.tri_inst == S.uni_inst) tri_ray.o = sub(r.o, mk(S.uni_off[0], S.uni_off[1], S.uni_off[2]));
      else tri_ray = to_local<true>(S.insts + S.tri_inst, r);
    }
  }
  // COUNT: tph[0] += wave-cycles in the node loop (phase 1), tph[1] += in the leaf tests (phase 2)
  uint64_t tm = COUNT ? __builtin_amdgcn_s_memtime() : 0;
  // Waves walking the tree issue before waves shading or regenerating (the path kernel drops the
  // priority again when trace_run returns).  MI355X A/B (profiles/r02/experiments, s1/s2): jumpy
  // +1.7%, cow +1.6%, monument +0.7%; shading first, node-load issue first or graded levels were
  // slower or equal.
  // The LDS-node kernel (NCAP > 0, node loads from LDS) is 0.6% faster without it (experiments, p2).
  if constexpr (NCAP == 0) __builtin_amdgcn_s_setprio(2);
  auto tick = [&](int k) {
    if (COUNT) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      tph[k] += t - tm;
      tm = t;
    }
  };
  auto safe_inv = [](float d) {
    float dd = fabsf(d) > 1e-20f ? d : copysignf(1e-20f, d);
    return __builtin_amdgcn_rcpf(dd);
  };
  const V3 inv = mk(safe_inv(r.d.x), safe_inv(r.d.y), safe_inv(r.d.z));
  const V3 ood = mk(r.o.x * inv.x, r.o.y * inv.y, r.o.z * inv.z);
  // near / far plane byte offsets inside DevNode4 by the ray's direction signs (32-bit offsets
  // from the uniform table base: the loads take the SGPR-base + VGPR-offset form)
  const uint32_t nx = inv.x < 0.f ? 16u : 0u, ny = (inv.y < 0.f ? 16u : 0u) + 32u, nz = (inv.z < 0.f ? 16u : 0u) + 64u;
  const uint32_t fx = nx ^ 16u, fy = ny ^ 16u, fz = nz ^ 16u;
  const char* const NB = NCAP > 0 ? reinterpret_cast<const char*>(lnodes)
                                  : (HN ? reinterpret_cast<const char*>(S.hnodes) : reinterpret_cast<const char*>(S.nodes));
  // ROOT (the S16 half-node mesh walk): lanes at the root or one of its children (breadth-first ids 0..4) visit it
  // from the workgroup's LDS copy of those five node4s (lnodes) before the loop, twice, so a segment's first two
  // visits cost no vector-memory loads (the mesh kernels are bound on the vector-memory data path, TD: ~2 of
  // monument's 5.6 visits per ray).  monument-4k +0.7%, cow-1080p +0.5-0.7% (profiles/r06/experiments rt5); the
  // same in the loop itself (t1: the tree's top from LDS at every visit) lost 6%: a visit whose lanes straddle the
  // table's edge runs both load paths, and the branch breaks up the loop's load clause.  17 node4s, three levels: -3.6%.
  constexpr bool ROOT = HN && S16 && NCAP == 0 && RTW_MESH_ROOT > 0;
  constexpr int32_t NROOT = RTW_MESH_ROOT;  // node4s in the LDS copy: 1 = the root, 5 = the root and its children
#pragma unroll
  for (int lv = 0; lv < (ROOT ? (NROOT > 1 ? 2 : 1) : 0); ++lv) {
    if (__any(ts.node >= 0 && ts.node < NROOT)) {
      if (ts.node >= 0 && ts.node < NROOT) {
        const char* const TB = reinterpret_cast<const char*>(lnodes) + (uint32_t)ts.node * 112u;
        const uint4 px = *reinterpret_cast<const uint4*>(TB + nx);
        const uint4 py = *reinterpret_cast<const uint4*>(TB + ny);
        const uint4 pz = *reinterpret_cast<const uint4*>(TB + nz);
        const uint4 cq = *reinterpret_cast<const uint4*>(TB + 96u);
        const half2_t oxy = as_h2(cq.z), oz = as_h2(cq.w);
        const V3 bs = mk(__builtin_fmaf((float)oxy.x, inv.x, -ood.x), __builtin_fmaf((float)oxy.y, inv.y, -ood.y),
                         __builtin_fmaf((float)oz.x, inv.z, -ood.z));
        const uint32_t PQ[3][4] = {{px.x, px.y, px.z, px.w}, {py.x, py.y, py.z, py.w}, {pz.x, pz.y, pz.z, pz.w}};
        float NA[3][4], FA[3][4];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const half2_t n01 = as_h2(PQ[q][0]), n23 = as_h2(PQ[q][1]), f01 = as_h2(PQ[q][2]), f23 = as_h2(PQ[q][3]);
          NA[q][0] = (float)n01.x; NA[q][1] = (float)n01.y; NA[q][2] = (float)n23.x; NA[q][3] = (float)n23.y;
          FA[q][0] = (float)f01.x; FA[q][1] = (float)f01.y; FA[q][2] = (float)f23.x; FA[q][3] = (float)f23.y;
        }
        const int32_t CW[4] = {(int32_t)(int16_t)(cq.x & 0xFFFFu), (int32_t)cq.x >> 16, (int32_t)(int16_t)(cq.y & 0xFFFFu),
                               (int32_t)cq.y >> 16};
        if (COUNT) {
          cnt[0]++;
          cnt[14] += (CW[0] != 0) + (CW[1] != 0) + (CW[2] != 0) + (CW[3] != 0);
        }
        const float tmax_c = __builtin_fmaf(ts.b.t, 1.0e-5f, ts.b.t) + 1.0e-5f;
        int32_t next = -1, bk = -1;
        float best = INFINITY;
        bool hit[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // conservative slab test (culling only), as in the loop below
          const float a0 = __builtin_fmaf(NA[0][k], inv.x, bs.x), b0 = __builtin_fmaf(NA[1][k], inv.y, bs.y);
          const float c0 = __builtin_fmaf(NA[2][k], inv.z, bs.z);
          const float d0 = __builtin_fmaf(FA[0][k], inv.x, bs.x), e0 = __builtin_fmaf(FA[1][k], inv.y, bs.y);
          const float f0 = __builtin_fmaf(FA[2][k], inv.z, bs.z);
          const float tn = fmaxf(fmaxf(fmaxf(a0, b0), c0), 0.0f);
          hit[k] = tn <= fminf(fminf(fminf(d0, e0), f0), tmax_c);
          const bool in = hit[k] & (CW[k] >= 0) & (tn < best);
          best = in ? tn : best;
          bk = in ? k : bk;
          next = in ? CW[k] : next;
        }
        int32_t pend = ts.pend, sp = ts.sp;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool leaf_take = hit[k] & (CW[k] < 0) & (pend == 0);
          pend = leaf_take ? CW[k] : pend;
          const bool pk = hit[k] & (k != bk) & !leaf_take;
          stk16[sp * BLK] = (uint16_t)CW[k];
          sp += pk ? 1 : 0;
        }
        ts.pend = pend;
        ts.sp = sp;
        ts.node = next;
      }
    }
  }
  // every wave must drain: a corrupt tree (a cycle) ends the walk instead of hanging the GPU, and
  // sets the device's host-mapped error word (RenderArgs::err), which the host turns into RTW_EINVAL
  // at the next render call, rtw_render_status, rtw_path_kernel_times or a stats read
  constexpr uint32_t GUARD = 1u << 20;
  uint32_t guard = 0;
  for (; guard < GUARD; ++guard) {
    uint32_t g2 = 0;
    for (; g2 < GUARD; ++g2) {
      if constexpr (K16) {  // refill: pop a code (internal node, or a leaf if the parking slot is free)
        const bool can = ts.node < 0 && ts.sp > 0;
        const int32_t top = can ? (int32_t)stk16[(ts.sp - 1) * BLK] : 0;
        const bool leaf = (top & 0x8000) != 0;
        const bool popn = can && !leaf;
        const bool popl = can && leaf && ts.pend == 0;
        ts.node = popn ? top : ts.node;
        ts.pend = popl ? top : ts.pend;
        ts.sp -= (popn || popl) ? 1 : 0;
      } else {  // refill from the stack: an internal node, or a parked leaf if the slot is free
        const bool can = ts.node < 0 && ts.sp > 0;
        int32_t top = 0;
        if (can) {
          const int32_t i = ts.sp - 1;
          if constexpr (S16) {
            top = (int32_t)(int16_t)stk16[i * BLK];
          } else {
            top = stk[(SPILL ? min(i, STACK) : i) * BLK];
            if (SPILL && i >= STACK) top = spill[(size_t)(i - STACK) * spill_lanes];  // rare
          }
        }
        const bool popn = can && top >= 0;
        const bool popl = can && top < 0 && ts.pend == 0;
        ts.node = popn ? top : ts.node;
        ts.pend = popl ? top : ts.pend;
        ts.sp -= (popn || popl) ? 1 : 0;
      }
#ifdef RTW_LANE_DIAG
      if (COUNT) {  // lane states per node-loop iteration (diagnostic build): all, descending, parked, done
        const uint64_t bd = __ballot(ts.node >= 0), bp = __ballot(ts.node < 0 && ts.pend != 0);
        const uint64_t bn = __ballot(ts.node < 0 && ts.pend == 0 && ts.sp == 0);
        tph[3] += 64;  // per lane (the wave-uniform values are added by every lane: ratios are unaffected)
        tph[4] += (uint64_t)__popcll(bd);
        tph[5] += (uint64_t)__popcll(bp);
        tph[6] += (uint64_t)__popcll(bn);
      }
#endif
      if (!__any(ts.node >= 0 && ts.pend == 0)) break;
      // enough lanes hold a postponed leaf with nothing left to descend: test the leaves now instead of
      // waiting until no lane can descend (Aila & Laine's rule).  leaf_thr = 3/16 of the wave's lanes
      // (knob RTW_LEAF16), measured on MI355X against 1..16/16: monument +8%, cow +0.6%, jumpy -0.4%
      if ((uint32_t)__popcll(__ballot(ts.node < 0 && ts.pend != 0)) >= leaf_thr) break;
#ifdef RTW_UNI_DIAG
      if (COUNT) {  // diagnostic build: wave-level visits whose visiting lanes share the node (and octant)
        const uint64_t vis = __ballot(ts.node >= 0);
        const int src = (int)__ffsll((long long)vis) - 1;
        const int32_t n0 = __shfl(ts.node, src, 64);
        const uint32_t oct = nx | ny | nz, o0 = (uint32_t)__shfl((int)oct, src, 64);
        const bool un = __ballot(ts.node >= 0 && ts.node != n0) == 0;
        const bool uo = __ballot(ts.node >= 0 && (ts.node != n0 || oct != o0)) == 0;
        tph[3] += 1;
        tph[4] += uo ? 1 : 0;
        tph[5] += un ? 1 : 0;
        tph[6] += (uint64_t)__popcll(vis);
      }
#endif
      if (ts.node >= 0) {
        float NX[4], FX[4], NY[4], FY[4], NZ[4], FZ[4];
        int32_t CW[4];
        V3 bs;  // plane t = plane * inv + bs per axis
        if constexpr (HN) {
          // DevNode4h: per axis ONE 16-B load at offset 0 / 16 by direction sign = (near x4, far x4) as f16
          // offsets; then codes + origin.  t = off * inv + (origin * inv - o * inv): every product and
          // sum a v_fma_mix_f32 on the f16 halves.  The f16 boxes contain the f32 ones (outward rounding).
          const uint32_t nb = (uint32_t)ts.node * 112u;  // sizeof(DevNode4h)
          const uint4 px = *reinterpret_cast<const uint4*>(NB + (nb + nx));
          const uint4 py = *reinterpret_cast<const uint4*>(NB + (nb + ny));
          const uint4 pz = *reinterpret_cast<const uint4*>(NB + (nb + nz));
          const uint4 cq = *reinterpret_cast<const uint4*>(NB + (nb + 96u));
          const half2_t oxy = as_h2(cq.z), oz = as_h2(cq.w);
          bs = mk(__builtin_fmaf((float)oxy.x, inv.x, -ood.x), __builtin_fmaf((float)oxy.y, inv.y, -ood.y),
                  __builtin_fmaf((float)oz.x, inv.z, -ood.z));
          const uint32_t P[3][4] = {{px.x, px.y, px.z, px.w}, {py.x, py.y, py.z, py.w}, {pz.x, pz.y, pz.z, pz.w}};
          float* const NA[3] = {NX, NY, NZ};
          float* const FA[3] = {FX, FY, FZ};
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            const half2_t n01 = as_h2(P[a][0]), n23 = as_h2(P[a][1]), f01 = as_h2(P[a][2]), f23 = as_h2(P[a][3]);
            NA[a][0] = (float)n01.x; NA[a][1] = (float)n01.y; NA[a][2] = (float)n23.x; NA[a][3] = (float)n23.y;
            FA[a][0] = (float)f01.x; FA[a][1] = (float)f01.y; FA[a][2] = (float)f23.x; FA[a][3] = (float)f23.y;
          }
          if constexpr (K16) {  // the codes as they are
            CW[0] = (int32_t)(cq.x & 0xFFFFu); CW[1] = (int32_t)(cq.x >> 16);
            CW[2] = (int32_t)(cq.y & 0xFFFFu); CW[3] = (int32_t)(cq.y >> 16);
          } else {  // sign-extended: internal >= 0, leaf < 0, as the 32-bit walk's child words
            CW[0] = (int32_t)(int16_t)(cq.x & 0xFFFFu); CW[1] = (int32_t)cq.x >> 16;
            CW[2] = (int32_t)(int16_t)(cq.y & 0xFFFFu); CW[3] = (int32_t)cq.y >> 16;
          }
        } else {
          const uint32_t nb = (uint32_t)ts.node << 7;  // sizeof(DevNode4); n_nodes < 2^25 (flatten)
          constexpr uint32_t CWO = (K16 || S16) ? 112u : 96u;  // child codes (K16, S16) or child words
          const float4 qnx = *reinterpret_cast<const float4*>(NB + (nb + nx));
          const float4 qfx = *reinterpret_cast<const float4*>(NB + (nb + fx));
          const float4 qny = *reinterpret_cast<const float4*>(NB + (nb + ny));
          const float4 qfy = *reinterpret_cast<const float4*>(NB + (nb + fy));
          const float4 qnz = *reinterpret_cast<const float4*>(NB + (nb + nz));
          const float4 qfz = *reinterpret_cast<const float4*>(NB + (nb + fz));
          const int4 cw = *reinterpret_cast<const int4*>(NB + (nb + CWO));
          bs = neg(ood);
          NX[0] = qnx.x; NX[1] = qnx.y; NX[2] = qnx.z; NX[3] = qnx.w; FX[0] = qfx.x; FX[1] = qfx.y; FX[2] = qfx.z; FX[3] = qfx.w;
          NY[0] = qny.x; NY[1] = qny.y; NY[2] = qny.z; NY[3] = qny.w; FY[0] = qfy.x; FY[1] = qfy.y; FY[2] = qfy.z; FY[3] = qfy.w;
          NZ[0] = qnz.x; NZ[1] = qnz.y; NZ[2] = qnz.z; NZ[3] = qnz.w; FZ[0] = qfz.x; FZ[1] = qfz.y; FZ[2] = qfz.z; FZ[3] = qfz.w;
          if constexpr (S16 && !K16) {  // 16-bit codes, sign-extended: internal >= 0, leaf < 0
            CW[0] = (int32_t)(int16_t)cw.x; CW[1] = (int32_t)(int16_t)cw.y;
            CW[2] = (int32_t)(int16_t)cw.z; CW[3] = (int32_t)(int16_t)cw.w;
          } else {
            CW[0] = cw.x; CW[1] = cw.y; CW[2] = cw.z; CW[3] = cw.w;
          }
        }
        if (COUNT) {
          cnt[0]++;
          simd_tick(cnt, 8, 9);
          cnt[14] += (CW[0] != 0) + (CW[1] != 0) + (CW[2] != 0) + (CW[3] != 0);  // child word 0 = empty slot
        }
        const float tmax_c = __builtin_fmaf(ts.b.t, 1.0e-5f, ts.b.t) + 1.0e-5f;
        float tn[4];
        bool hit[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // conservative slab test (culling only)
          const float a = __builtin_fmaf(NX[k], inv.x, bs.x), b = __builtin_fmaf(NY[k], inv.y, bs.y);
          const float c = __builtin_fmaf(NZ[k], inv.z, bs.z);
          const float d = __builtin_fmaf(FX[k], inv.x, bs.x), e = __builtin_fmaf(FY[k], inv.y, bs.y);
          const float f = __builtin_fmaf(FZ[k], inv.z, bs.z);
          tn[k] = fmaxf(fmaxf(fmaxf(a, b), c), 0.0f);
          hit[k] = tn[k] <= fminf(fminf(fminf(d, e), f), tmax_c);
        }
        if constexpr (K16) {
          // pin the child codes in registers: otherwise the compiler sinks each child's LDS read under
          // its `hit` branch (4 dependent read round trips per visit)
          int32_t cwv[4] = {CW[0], CW[1], CW[2], CW[3]};
          asm volatile("" : "+v"(cwv[0]), "+v"(cwv[1]), "+v"(cwv[2]), "+v"(cwv[3]));
          uint32_t key[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) key[k] = hit[k] ? ((__float_as_uint(tn[k]) & 0xFFFF0000u) | (uint32_t)cwv[k]) : 0u;
          const uint32_t a0 = max(key[0], key[1]), b0 = min(key[0], key[1]);
          const uint32_t c0 = max(key[2], key[3]), d0 = min(key[2], key[3]);
          const uint32_t s0 = max(a0, c0), x0 = min(a0, c0), y0 = max(b0, d0), s3 = min(b0, d0);
          const uint32_t s1 = max(x0, y0), s2 = min(x0, y0);
          uint16_t* w = stk16 + ts.sp * BLK;  // rows sp .. sp + 3 (ds_write_b16 stores the code bits)
          w[0] = (uint16_t)s0;
          w[BLK] = (uint16_t)s1;
          w[2 * BLK] = (uint16_t)s2;
          w[3 * BLK] = (uint16_t)s3;
          const bool m1 = s1 != 0u, m2 = s2 != 0u, m3 = s3 != 0u;
          const uint32_t near = m3 ? s3 : (m2 ? s2 : (m1 ? s1 : s0));
          const int32_t code = (int32_t)(near & 0xFFFFu);
          const bool any = s0 != 0u, leaf = (code & 0x8000) != 0;
          const bool park = any && leaf && ts.pend == 0;
          // pushed: the hits but the nearest (h - 1), + the nearest leaf if it cannot be parked
          ts.sp += (int32_t)m1 + (int32_t)m2 + (int32_t)m3 + ((any && leaf && !park) ? 1 : 0);
          ts.pend = park ? code : ts.pend;
          ts.node = (any && !leaf) ? code : -1;
          continue;
        }
        // nearest hit internal child -> next node; the other hit children -> stack / parked slot
        int32_t next = -1;
        float best = INFINITY;
        int bk = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool in = hit[k] & (CW[k] >= 0) & (tn[k] < best);  // bitwise: no branches
          best = in ? tn[k] : best;
          bk = in ? k : bk;
          next = in ? CW[k] : next;
        }
        int32_t pend = ts.pend;
        uint32_t push = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool leaf_take = hit[k] & (CW[k] < 0) & (pend == 0);
          pend = leaf_take ? CW[k] : pend;
          push |= (hit[k] & (k != bk) & !leaf_take) ? (1u << k) : 0u;
        }
        ts.pend = pend;
        int32_t sp = ts.sp;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool pk = (push >> k) & 1u;
          // branch-free: a child that is not pushed is written where the next push (or nothing)
          // lands, i.e. at or above the final top, never below it.  Rows 0..STACK exist; with
          // SPILL, row STACK is scratch and entries from STACK up live in HBM (sp < stack_need).
          if constexpr (S16) {
            stk16[sp * BLK] = (uint16_t)CW[k];
          } else {
            stk[(SPILL ? min(sp, STACK) : sp) * BLK] = CW[k];
            if (SPILL && pk && sp >= STACK) spill[(size_t)(sp - STACK) * spill_lanes] = CW[k];  // rare
          }
          sp += pk ? 1 : 0;
        }
        ts.sp = sp;
        ts.node = next;
      }
    }
    if (g2 == GUARD) break;
    tick(0);
    if (ts.pend != 0) {  // phase 2
      const uint32_t v = CODES ? (uint32_t)ts.pend & 0xFFFFu : ~(uint32_t)ts.pend;
      const int32_t first = CODES ? (int32_t)((v >> 2) & 0x1FFFu) : (int32_t)(v >> 3);
      const int32_t n = CODES ? (int32_t)(v & 3u) + 1 : (int32_t)(v & 7u);
      if ((FEAT & F_TRI) && S.bvh_tri) {  // kernel-uniform: every leaf is a triangle of one wrapper chain
        for (int32_t k = 0; k < n; ++k) test_tri_leaf<COUNT>(S, (uint32_t)(first + k), tri_ray, ts.b, cnt);
      } else {
        for (int32_t k = 0; k < n; ++k)
          test_prim<COUNT, FEAT>(S, (uint32_t)(first + k), r, ts.b, cnt, seg, SPH_ONLY ? &rq : nullptr);
      }
      ts.pend = 0;
    }
    tick(1);
    const uint64_t done = __ballot(ts.node < 0 && ts.sp == 0);
    if (done == __ballot(1) || (uint32_t)__popcll(done) >= quota) return;
  }
  *err = 1u;  // a guard tripped: end this traversal (miss) and report (a vector store to host memory)
  ts.b.prim = -2;  // the path kernel drains the grid (see its miss branch)
  ts.node = -1;
  ts.sp = 0;
  ts.pend = 0;
}

// ---- hit record of the winner (hittable/mod.rs:32-48 at every level)
struct Rec { V3 p, n; float u, v; bool front; uint32_t mat; };
__device__ __forceinline__ void face(Rec& h, V3 dir, V3 outward) {
  h.front = dot(dir, outward) < 0.0f;
  h.n = h.front ? outward : neg(outward);
}
__device__ __forceinline__ void sphere_uv(V3 p, float& u, float& v) {  // spherical.rs:62-77
  const float PI = 3.14159265358979323846f;
  float theta = dev_acosf(-p.y);
  float phi = dev_atan2f(-p.z, p.x) + PI;
  u = phi / (2.0f * PI);
  v = theta / PI;
}

template <uint32_t FEAT>
__device__ Rec hit_record(const DevScene& S, const Ray& wr, const Best& b, uint32_t shade_kind) {
  // Triangle kernels: the meta word first, then only the geometry the winner's type needs (a triangle
  // needs none: its barycentrics come from its test, Best::u / v; cow +4%).  Other kernels load the whole
  // record in one round trip (a dependent geometry load cost jumpy 2.3%, profiles/r03/experiments b2).
  const float4* PP = reinterpret_cast<const float4*>(S.prims + b.prim);
  const uint4 meta = *reinterpret_cast<const uint4*>(PP + 3);
  float4 g0, g1, g2;
  if constexpr (!(FEAT & F_TRI)) {
    g0 = PP[0];
    g1 = PP[1];
    g2 = PP[2];
  }
  auto geo = [&](int k) -> float4 {
    if constexpr (!(FEAT & F_TRI)) return k == 0 ? g0 : (k == 1 ? g1 : g2);
    else return PP[k];
  };
  const uint32_t type = meta.x & 0xffu, inst = meta.x >> 8;
  const DevInst* I = S.insts + inst;
  const bool uni = (FEAT & F_INST) && inst && inst == S.uni_inst;  // one Translation, offset uniform
  Ray lr = wr;
  // Chains of at most two wrappers (a Cuboid's .rotate_y().translate(): cornell-box, the book-2 scenes), in the
  // kernels without triangles: the header and both ops in three independent loads and the directions after each op
  // kept for the unwinding below, instead of the generic loops' chain of dependent loads and per-level recomputation
  // (the same f32 operations).
  bool short_chain = false;
  uint32_t nops = 0;
  float4 op0 = make_float4(0.f, 0.f, 0.f, 0.f), op1 = op0;
  V3 d0 = wr.d, d1 = wr.d;  // the ray direction inside wrapper 0 (after op 0) and wrapper 1 (after ops 0, 1)
  auto apply_op = [](float4 op, Ray& r) {  // transformations.rs:23-28 / :115-135, as to_local
    if (op_is(op.x, IO_TRANSLATE)) {
      r.o = sub(r.o, mk(op.y, op.z, op.w));
    } else {
      const float s = op.y, c = op.z;
      r.o = mk(c * r.o.x - s * r.o.z, r.o.y, s * r.o.x + c * r.o.z);
      r.d = mk(c * r.d.x - s * r.d.z, r.d.y, s * r.d.x + c * r.d.z);
    }
  };
  if (uni) {
    lr.o = sub(wr.o, mk(S.uni_off[0], S.uni_off[1], S.uni_off[2]));
  } else if ((FEAT & F_INST) && inst) {
    nops = I->nops;
    op0 = *reinterpret_cast<const float4*>(I->op[0]);
    op1 = *reinterpret_cast<const float4*>(I->op[1]);
    short_chain = !(FEAT & F_TRI) && nops <= 2u;  // (the mesh kernels' registers are spoken for: generic path)
    if (short_chain) {
      apply_op(op0, lr);
      d0 = lr.d;
      if (nops == 2u) apply_op(op1, lr);
      d1 = lr.d;
    } else {
      lr = to_local(I, wr);
    }
  }
  const float t = b.t;
  Rec h;
  h.mat = meta.z;
  h.u = 0.0f;
  h.v = 0.0f;
  V3 outward;
  h.p = add(lr.o, scale(lr.d, t));  // ray.rs:25-27
  if (((FEAT & F_SPHERE) && type == PT_SPHERE) || ((FEAT & F_MSPHERE) && type == PT_MSPHERE)) {
    const float4 q0 = geo(0), q1 = geo(1), q2 = geo(2);
    V3 c = type == PT_SPHERE ? mk(q0.x, q0.y, q0.z) : center_at(q0, q1, PP, S.msphere_unit, lr.time);
    const float rad = q2.z;  // r (q0.w holds r * r)
    // spherical.rs:49 (p - c) / r by the corrections from RN(1 / r), computed once by the flattener (q2.w)
    const V3 pc = sub(h.p, c);
    const bool ok = recip_div_ok(rad);
    outward = mk(div_rcp(pc.x, rad, q2.w, ok), div_rcp(pc.y, rad, q2.w, ok), div_rcp(pc.z, rad, q2.w, ok));
    if ((FEAT & F_UV) && (shade_kind & (1u << 12))) sphere_uv(outward, h.u, h.v);
  } else if ((FEAT & F_TRI) && type == PT_TRI) {
    const TriUV s{b.t, b.u, b.v};  // tri_solve's values from the winning test (the same ray and operands)
    const DevTriShade& sh = S.tshade[b.prim];  // indexed like prims[] (rtw_flatten.cpp)
    float w = 1.0f - s.u - s.v;  // triangular.rs:315-323
    outward = add(add(scale(ld3(sh.n), w), scale(ld3(sh.n + 3), s.u)), scale(ld3(sh.n + 6), s.v));
    h.u = (w * sh.uv[0] + s.u * sh.uv[2]) + s.v * sh.uv[4];
    h.v = (w * sh.uv[1] + s.u * sh.uv[3]) + s.v * sh.uv[5];
  } else if ((FEAT & F_MEDIUM) && type == PT_MEDIUM) {  // volumes.rs:62-77: no face-normal logic
    outward = mk(1.0f, 0.0f, 0.0f);
  } else {
    const int axis = (int)type - PT_RECT_XY;
    const float x = axis == 2 ? h.p.y : h.p.x;
    const float y = axis == 0 ? h.p.y : h.p.z;
    const float4 q0 = geo(0);
    h.u = (x - q0.x) / (q0.y - q0.x);
    h.v = (y - q0.z) / (q0.w - q0.z);
    outward = axis == 0 ? mk(0.f, 0.f, 1.f) : (axis == 1 ? mk(0.f, 1.f, 0.f) : mk(1.f, 0.f, 0.f));
  }
  if ((FEAT & F_MEDIUM) && type == PT_MEDIUM) {
    h.n = outward;
    h.front = true;
  } else {
    face(h, lr.d, outward);
  }
  if (uni) {  // transformations.rs:29-37: p + offset, face normal against the world ray
    h.p = add(h.p, mk(S.uni_off[0], S.uni_off[1], S.uni_off[2]));
    face(h, wr.d, h.n);
  } else if ((FEAT & F_INST) && inst && short_chain) {  // unwind inner -> outer (transformations.rs:29-37, :137-147)
    auto unwind_op = [&](float4 op, V3 dk) {
      if (op_is(op.x, IO_TRANSLATE)) {
        h.p = add(h.p, mk(op.y, op.z, op.w));
        face(h, dk, h.n);
      } else {
        const float s = op.y, c = op.z;
        V3 p = mk(c * h.p.x + s * h.p.z, h.p.y, -s * h.p.x + c * h.p.z);
        V3 n = mk(c * h.n.x + s * h.n.z, h.n.y, -s * h.n.x + c * h.n.z);
        h.p = p;
        face(h, dk, n);
      }
    };
    if (nops == 2u) unwind_op(op1, d1);
    if (nops >= 1u) unwind_op(op0, d0);
  } else if ((FEAT & F_INST) && inst) {  // unwind wrappers inner -> outer (transformations.rs:29-37, :137-147)
    for (int k = (int)I->nops - 1; k >= 0; --k) {
      V3 dk = wr.d;  // direction as seen inside wrapper k = after ops 0..k
      for (int q = 0; q <= k; ++q) {
        const float4 op = *reinterpret_cast<const float4*>(I->op[q]);
        if (op_is(op.x, IO_ROTY)) dk = mk(op.z * dk.x - op.y * dk.z, dk.y, op.y * dk.x + op.z * dk.z);
      }
      const float4 op = *reinterpret_cast<const float4*>(I->op[k]);
      if (op_is(op.x, IO_TRANSLATE)) {
        h.p = add(h.p, mk(op.y, op.z, op.w));
        face(h, dk, h.n);
      } else {
        const float s = op.y, c = op.z;
        V3 p = mk(c * h.p.x + s * h.p.z, h.p.y, -s * h.p.x + c * h.p.z);
        V3 n = mk(c * h.n.x + s * h.n.z, h.n.y, -s * h.n.x + c * h.n.z);
        h.p = p;
        face(h, dk, n);
      }
    }
  }
  return h;
}

// Checker::value's decision (texture.rs:69-81) is `sinf(fx) * sinf(fy) * sinf(fz) < 0` with glibc's
// sinf.  oracle/tools/sin_sign_check.cpp proves over EVERY finite float (tests/test_checker_proof.py):
// sign(sinf x) = parity of floor(x / pi), by the double-precision product for 2^-12 <= |x| < 65536
// and by the exact integer reduction rtw::pi_parity for |x| >= 65536; sinf x == x for |x| < 2^-12;
// |sinf x| >= 3.2e-9 for |x| >= 2^-12 (no product of three such factors underflows).  So the
// decision is the XOR of the factors' signs, except that NaN / inf / 0 factors give "even" and a
// product that underflows to zero is "even".  Underflow needs a tiny factor: it is decided from the
// product of the tiny factors alone (|sin| of the others taken as 1), exact unless that product is
// below 2^-120 / 3.2e-9^k (some |f x| < ~1e-20): that corner alone is not pinned.
__device__ __forceinline__ bool checker_odd_slow(float fx, float fy, float fz) {
  const float f[3] = {fx, fy, fz};
  uint32_t neg = 0;
  float tiny = 1.0f;  // left-to-right product of the tiny factors (sinf x == x there)
#pragma unroll 1
  for (int k = 0; k < 3; ++k) {  // cold path: one copy of the reduction, not three
    const float x = f[k], ax = fabsf(x);
    if (x != x || isinf(x) || x == 0.0f) return false;  // NaN or +-0 product: `< 0` is false
    if (ax < 0x1p-12f) tiny = tiny * ax;
    neg ^= (ax < 0x1p-12f ? 0u : pi_parity(ax)) ^ (x < 0.0f ? 1u : 0u);
  }
  return neg != 0 && tiny != 0.0f;
}
__device__ __forceinline__ bool checker_odd(float fx, float fy, float fz) {
  const float ax = fabsf(fx), ay = fabsf(fy), az = fabsf(fz);
  const float lo = 0x1p-12f, hi = 65536.0f;
  if (ax >= lo && ax < hi && ay >= lo && ay < hi && az >= lo && az < hi) {
    const double INV_PI = 0.31830988618379067154;
    const int k = (int)floor((double)fx * INV_PI) + (int)floor((double)fy * INV_PI) + (int)floor((double)fz * INV_PI);
    return (k & 1) != 0;
  }
  return checker_odd_slow(fx, fy, fz);
}

// ---- Perlin noise (perlin.rs:50-122), same operation order as the oracle's perlin_noise
__device__ __forceinline__ int64_t f32_as_i64(float x) {  // Rust `as i64`: saturating, NaN -> 0
  if (x != x) return 0;
  if (x >= 9223372036854775807.0f) return INT64_MAX;
  if (x <= -9223372036854775808.0f) return INT64_MIN;
  return (int64_t)x;
}
__device__ __forceinline__ float perlin_noise(const DevPerlin& P, V3 p) {
  const V3 fl = mk(floorf(p.x), floorf(p.y), floorf(p.z));
  const uint32_t bx = (uint32_t)f32_as_i64(fl.x), by = (uint32_t)f32_as_i64(fl.y), bz = (uint32_t)f32_as_i64(fl.z);
  const V3 w = sub(p, fl);
  const V3 f = mul(mul(w, w), sub(mk(3.0f, 3.0f, 3.0f), scale(w, 2.0f)));  // filter_hermit
  float accum = 0.0f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t hsh = (uint32_t)P.perm[0][(bx + i) & 255u] ^ (uint32_t)P.perm[1][(by + j) & 255u] ^
                             (uint32_t)P.perm[2][(bz + k) & 255u];
        const float4 g = *reinterpret_cast<const float4*>(P.g[hsh]);
        const V3 c = mk((float)i, (float)j, (float)k);
        const V3 wv = sub(f, c);
        const V3 bl = add(mul(c, f), mul(sub(mk(1.f, 1.f, 1.f), c), sub(mk(1.f, 1.f, 1.f), f)));
        const float bf = bl.x * bl.y * bl.z;
        accum += bf * dot(mk(g.x, g.y, g.z), wv);
      }
  return accum;
}
__device__ __forceinline__ float perlin_turbulence(const DevPerlin& P, V3 p, int depth) {  // perlin.rs:78-91
  float accum = 0.0f, weight = 1.0f;
#pragma unroll 1
  for (int d = 0; d < depth; ++d) {
    accum += weight * perlin_noise(P, p);
    weight *= 0.5f;
    p = scale(p, 2.0f);
  }
  return fabsf(accum);
}

// image_texture.rs:34-52 over RGBX8 texels (rtw_flatten.cpp): one aligned 4-byte load
__device__ __forceinline__ V3 image_texel(const DevScene& S, uint32_t off, uint32_t tw, uint32_t th, float u, float v) {
  float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
  float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
  float vv = 1.0f - vc;
  float fi = uu * (float)tw, fj = vv * (float)th;
  uint32_t i = (fi != fi || fi <= 0.0f) ? 0u : (fi >= 4294967295.0f ? 0xFFFFFFFFu : (uint32_t)fi);
  uint32_t j = (fj != fj || fj <= 0.0f) ? 0u : (fj >= 4294967295.0f ? 0xFFFFFFFFu : (uint32_t)fj);
  i = i > tw - 1 ? tw - 1 : i;
  j = j > th - 1 ? th - 1 : j;
  const uint32_t px = *reinterpret_cast<const uint32_t*>(S.texels + off + ((size_t)j * tw + i) * 4);
  const float sc = 1.0f / 255.0f;
  return mk((float)(px & 0xffu) * sc, (float)((px >> 8) & 0xffu) * sc, (float)((px >> 16) & 0xffu) * sc);
}

// ---- textures (texture.rs:56-81, :89-104; image_texture.rs:34-52)
template <uint32_t FEAT>
__device__ V3 tex_value(const DevScene& S, uint32_t id, float u, float v, V3 p) {
  for (int guard = 0; guard < 64; ++guard) {
    const DevTex& t = S.texs[id];
    if (t.type == TT_SOLID) return ld3(t.c);
    if ((FEAT & F_CHECKER) && t.type == TT_CHECKER) {
      id = checker_odd(t.freq * p.x, t.freq * p.y, t.freq * p.z) ? t.odd : t.even;
      continue;
    }
    if ((FEAT & F_IMAGE) && t.type == TT_IMAGE) return image_texel(S, t.off, t.w, t.h, u, v);
    if ((FEAT & F_NOISE) && t.type == TT_NOISE) {  // texture.rs:89-95
      const float tb = perlin_turbulence(S.perlins[t.off], p, 7);
      const float sv = 0.5f * (1.0f + dev_sinf(t.freq * p.z + 10.0f * tb));
      return mk(sv, sv, sv);
    }
    if ((FEAT & F_UVDEBUG) && t.type == TT_UVDEBUG) return mk(u, v, 0.0f);  // UVDebug
    break;
  }
  return mk(0.f, 0.f, 0.f);
}

__device__ __forceinline__ float reflectance(float cosine, float r0) {  // material.rs:108-112, r0 precomputed (DevShade::a)
  float x = 1.0f - cosine;
  float x2 = x * x;
  return r0 + (1.0f - r0) * (x * (x2 * x2));  // powi(5) as LLVM expands it
}

// ---- the persistent path kernel
//
// Work unit = one path (pixel, sample).  Path id p (within a pass) = (slot*spp + s)*64 + l:
// slot = tile slot, s = sample, l = lane-in-tile, so the 64 paths a wave draws together
// are one sample of one 8x8 tile (coherent camera rays).  Waves are persistent: whenever
// lanes finish a path, the wave hands them new ids from a per-wave pool (ballot + mbcnt
// prefix), refilled from a global counter BATCH ids at a time, so lanes stay busy and the
// grid drains with a one-path tail.  Each finished path writes L to the ordered sample
// buffer (path-major RGB, 12 B per path in HBM); reduce_kernel then sums each pixel's samples in
// sample order — exactly lib.rs:83-87's `pixel_color += sample_ray(..)` sequence.
// Path ids a wave takes per returning atomic on the global queue word (path_kernel SHARD: eight).  Every wave of
// the grid hits that word: at 256 ids per atomic, short-path scenes spent most of their time behind it
// (MI355X, RTW_BATCH sweep: cow-1080p 19.0k -> 30.1k Mrays/s, monument-4k 12.8k -> 17.0k, jumpy-1080p
// 19.4k -> 20.4k at 2048); the tail this leaves is one batch per wave (~0.1 ms).  Knob RTW_BATCH.
constexpr uint32_t BATCH = 2048;

struct PathState {
  Ray ray;
  V3 T;
  uint64_t rng;
  uint32_t pid;  // path id within the pass (a pass holds at most 2^32 paths, max_pass_paths)
  uint32_t depth;
};

// floor(n / d) for 32-bit n and d >= 2 from M = UINT64_MAX / d + 1 (Lemire, Kaser & Kurz 2019,
// "Faster remainder by direct computation"): hi64(M * n) in two 32-bit multiplies instead of the
// ~25-instruction runtime u32 division; checked exhaustively for 12 divisors over every n and for
// 1e8 random pairs on the host.
__device__ __forceinline__ uint32_t fastdiv(uint32_t n, uint64_t M) {
  const uint64_t t = (uint64_t)(uint32_t)(M >> 32) * n + __umulhi((uint32_t)M, n);
  return (uint32_t)(t >> 32);
}

// readfirstlane of a 64-bit value.  The builtin returns a signed int: each half must go through
// uint32_t before widening, or a low half >= 2^31 sign-extends over the high half (path ids of a
// pass above 2^31 — monument-4k's 2^32-path passes — became huge and wrote outside the buffer).
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  return ((uint64_t)hi << 32) | lo;
}

// start_path's kernel-uniform operands (camera, frame and tile geometry, seeds): copied into LDS once per
// workgroup and re-read at every regeneration, instead of living in SGPRs across the whole path loop,
// where the list-mode and sphere kernels had to spill them into VGPR lanes (every reload a v_readlane).
struct StartArgs {
  DevCamera cam;
  float fw1, fh1, rw1, rh1, time_span;
  uint32_t w, h, spp, max_depth, tiles_x, slot_base, tile_first, tile_stride;
  uint64_t spp_magic, tiles_x_magic, seed_hash;
  const uint32_t* tile_ids;
};
__device__ __forceinline__ void fill_start_args(const RenderArgs& a, StartArgs& o) {
  o.cam = a.cam;
  o.fw1 = a.fw1; o.fh1 = a.fh1; o.rw1 = a.rw1; o.rh1 = a.rh1; o.time_span = a.time_span;
  o.w = a.w; o.h = a.h; o.spp = a.spp; o.max_depth = a.max_depth; o.tiles_x = a.tiles_x;
  o.slot_base = a.slot_base; o.tile_first = a.tile_first; o.tile_stride = a.tile_stride;
  o.spp_magic = a.spp_magic; o.tiles_x_magic = a.tiles_x_magic; o.seed_hash = a.seed_hash;
  o.tile_ids = a.tile_ids;
}

// LST_BLK > 0: also store T = 1, depth and the path id in the lane's LDS state rows (path_kernel LST), here
// where the values are made (carried to the caller, they were spilled)
template <bool FROM_LDS, int LST_BLK = 0, int LST_ROW = 0, bool AB = FROM_LDS>
__device__ __forceinline__ bool start_path(const StartArgs& a, uint64_t pid, PathState& st, uint16_t* lst = nullptr) {
  if constexpr (FROM_LDS) asm volatile("" ::: "memory");  // read the LDS copy here: no loop-invariant register copies
  const uint32_t hi = (uint32_t)(pid >> 6), l = (uint32_t)pid & 63u;
  const uint32_t slot = a.spp > 1u ? fastdiv(hi, a.spp_magic) : hi, s = hi - slot * a.spp;
  const uint32_t gslot = a.slot_base + slot;
  const uint32_t tile = a.tile_ids ? a.tile_ids[gslot] : a.tile_first + gslot * a.tile_stride;
  const uint32_t ty = a.tiles_x > 1u ? fastdiv(tile, a.tiles_x_magic) : tile;
  const uint32_t i = (tile - ty * a.tiles_x) * 8u + (l & 7u), row = ty * 8u + (l >> 3);
  if (i >= a.w || row >= a.h) return false;
  const uint32_t j = a.h - 1u - row;
  const DevCamera& C = a.cam;
  uint64_t rng = xoro_seed(splitmix64(a.seed_hash ^ (((uint64_t)j << 48) | ((uint64_t)i << 32) | s)));
  // lib.rs:84-86 + camera.rs:66-74
  const float u = div_by_recip((float)i + gen_f32(rng), a.fw1, a.rw1);
  const float v = div_by_recip((float)j + gen_f32(rng), a.fh1, a.rh1);
  const V3 rd = scale(rand_in_unit_disk<AB>(rng), C.lens_radius);
  const V3 off = add(scale(ld3(C.u), rd.x), scale(ld3(C.v), rd.y));
  st.ray.o = add(ld3(C.origin), off);
  st.ray.d = sub(sub(add(add(ld3(C.llc), scale(ld3(C.horizontal), u)), scale(ld3(C.vertical), v)), ld3(C.origin)),
                 off);
  st.ray.time = gen_range<AB>(rng, C.time0, C.time1, a.time_span);
  st.rng = rng;
  st.T = mk(1.f, 1.f, 1.f);
  st.depth = a.max_depth;
  st.pid = (uint32_t)pid;
  if constexpr (LST_BLK > 0) {
    const uint32_t v[5] = {0x3F800000u, 0x3F800000u, 0x3F800000u, a.max_depth, (uint32_t)pid};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      lst[(LST_ROW + 2 * k) * LST_BLK] = (uint16_t)v[k];
      lst[(LST_ROW + 2 * k + 1) * LST_BLK] = (uint16_t)(v[k] >> 16);
    }
  }
  return true;
}

// BLK: workgroup size (256, or 512 for the LDS-node variants: one copy of the node table serves 8
// waves).  NCAP: capacity of the LDS node table in node4s (0 = nodes read from global memory).
template <bool COUNT, int STACK, bool SPILL, int OCC, uint32_t FEAT, int BLK = BLOCK, int NCAP = 0, bool HN = false,
          bool S16 = false>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void path_kernel(RenderArgs a) {
  // + 1: trace_run's branch-free push.  LDS-node variants use 16-bit entries, STACK rows (window included);
  // S16 (global nodes, 16-bit entries): STACK + 1 rows of 16 bits
  __shared__ int32_t stk_all[(NCAP > 0 || S16) ? 1 : (STACK + 1) * BLK];
  // LST: 10 more 16-bit rows after the stack hold the path state (below)
  // (the S16 mesh walk too: its 16-bit stack column has STACK + 1 rows, the state rows follow them)
  constexpr int LST_ROWS = ((NCAP > 0 && BLK == 1024) || S16) ? 10 : 0;
  constexpr int LST_ROW0 = STACK + (S16 ? 1 : 0);
  __shared__ uint16_t stk16_all[NCAP > 0 ? (STACK + LST_ROWS) * BLK : (S16 ? (STACK + 1 + LST_ROWS) * BLK : 1)];
  constexpr uint32_t NODE_Q = HN ? 7u : 8u;  // 16-B quads per node (DevNode4h / DevNode4)
  // (the S16 half-node mesh walk: the root node only, trace_run ROOT)
  constexpr bool ROOT_LDS = HN && S16 && NCAP == 0 && RTW_MESH_ROOT > 0;
  __shared__ float4 nodes_lds[NCAP > 0 ? NCAP * NODE_Q : (ROOT_LDS ? RTW_MESH_ROOT * NODE_Q : 1)];
  if constexpr (NCAP > 0) {  // the host launches this variant only when Flat::codes16 and n_nodes <= NCAP
    const float4* g = HN ? reinterpret_cast<const float4*>(a.scene.hnodes) : reinterpret_cast<const float4*>(a.scene.nodes);
    for (uint32_t k = threadIdx.x; k < a.scene.n_nodes * NODE_Q; k += BLK) nodes_lds[k] = g[k];
  }
  if constexpr (ROOT_LDS) {
    const uint32_t nq = min(a.scene.n_nodes, (uint32_t)RTW_MESH_ROOT) * NODE_Q;
    if (threadIdx.x < nq) nodes_lds[threadIdx.x] = reinterpret_cast<const float4*>(a.scene.hnodes)[threadIdx.x];
  }
  // start_path's operands from LDS in the sphere and list-mode variants (their SGPR spills, and every
  // reload a v_readlane: cornell-800 +6%, jumpy +0.8%) and in the 6 / 7-wave mesh walk (S16): at 80 VGPRs its
  // SGPRs overflowed into VGPR lanes and 28 B per lane of scratch; with the LDS copy 12 B: monument-4k +4.5%,
  // cow-1080p +6.7% (profiles/r05/experiments, m1).  The 5-wave mesh variants keep the kernel arguments (their
  // paths regenerate every ~2 segments: 5-7% slower with the LDS reads in round 3).  The one-alignbit draws (AB)
  // stay with the sphere and list-mode kernels (the triangle kernels' register allocation lost 1-2% with them).
  constexpr bool AB = !(FEAT & F_TRI);
  constexpr bool SLDS = AB || S16;
  __shared__ StartArgs start_lds[SLDS ? 1 : 0 + 1];
  StartArgs sa_reg;
  if constexpr (SLDS) {
    if (threadIdx.x == 0) fill_start_args(a, start_lds[0]);
  } else {
    fill_start_args(a, sa_reg);
  }
  const StartArgs& SA = SLDS ? start_lds[0] : sa_reg;
  __syncthreads();
  uint16_t* stk16 = stk16_all + threadIdx.x;
  int32_t* stk = stk_all + threadIdx.x;
  int32_t* spill = a.spill + (size_t)blockIdx.x * BLK + threadIdx.x;  // unused unless spill_depth > 0
  const uint32_t lane = threadIdx.x & 63u;
  // LST (1024-lane LDS-node workgroups, 2 per CU: half the node-table copies of 512-lane ones): a path's
  // throughput, remaining depth and id live in LDS, not VGPRs.  At 8 waves / SIMD (64 VGPRs) the compiler
  // spilled exactly these to scratch (a scratch load / store per use in every shading pass: ~40% of the
  // kernel's vector-memory instructions and ~23 GB of HBM write-back per jumpy-1080p frame)
  // Each 32-bit value is two 16-bit rows of the lane's stack column (rows STACK.. STACK + 9: T.x, T.y, T.z,
  // depth, id), addressed from the stack pointer with constant offsets: separate per-lane LDS pointers were
  // loop-invariant VGPRs, which the compiler spilled in turn.
  constexpr bool LST = LST_ROWS > 0;
  auto lst_st = [&](int k, uint32_t v) {
    stk16[(LST_ROW0 + 2 * k) * BLK] = (uint16_t)v;
    stk16[(LST_ROW0 + 2 * k + 1) * BLK] = (uint16_t)(v >> 16);
  };
  auto lst_ld = [&](int k) -> uint32_t {
    return (uint32_t)stk16[(LST_ROW0 + 2 * k) * BLK] | ((uint32_t)stk16[(LST_ROW0 + 2 * k + 1) * BLK] << 16);
  };
  const DevScene& S = a.scene;
  const V3 bg = ld3(a.bg);
  const uint64_t P = a.n_paths;
  // SHARD (the LDS-node sphere kernels): n dispensers (DISP when the host's small-frame rule cut the batch below these
  // kernels' 1024, else 1), 128 B apart: dispenser d hands out the
  // pass's batches d, d + n, d + 2n, ... (interleaved, so the grid still works through the frame in id order, tile
  // after tile), and a wave takes batches from dispenser (its workgroup + k) mod n, k = 0, 1, ... as each runs dry
  // (workgroups are dealt to the XCDs in turn, so each XCD's waves start on their own word).  One word for the whole
  // grid serialises its atomics: the small batches of small passes -- configs[0], an 8-GPU share's short end-of-pass
  // tail -- queued behind it (r06, share8: jumpy's 1/8 share +5%, configs[0] +11%).  The other kernels keep the one
  // word (their code with the dispenser loop ran 1.2-1.8% slower on full frames: cornell, monument).
  constexpr bool SHARD = NCAP > 0;
  unsigned long long* const dispenser = a.queue;
  const uint32_t batch = a.batch, ndisp = batch < 1024u ? DISP : 1u;
  const uint64_t NB = (P + batch - 1u) / batch;  // batches in the pass
  uint32_t cnt[15] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long nrays = 0;
  // the wave's id pool [next, end) lives in LDS between regenerations: loop-carried 64-bit
  // uniforms otherwise end up as VGPR phis that the 6-wave sphere variant has to spill
  __shared__ uint64_t pool_lds[BLK / 64][SHARD ? 5 : 3];
  // S16 mesh walk: the wave index as a scalar, so the pool address is rebuilt from an SGPR (one v_mov) where it is
  // used instead of kept in a VGPR (the 7-wave walk spilled it to scratch and reloaded it at every regeneration;
  // the sphere and list-mode kernels measured 0.5-1.4% slower with it, profiles/r05/experiments s1)
  uint64_t* const pool = pool_lds[S16 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6];
  if (lane == 0) { pool[0] = 0; pool[1] = 0; }
  if (SHARD && lane == 0) pool[SHARD ? 4 : 0] = 0;
  // the wave's next batch [b, e) of path ids (b = e = P: none left); lane 0 takes it, every lane reads it
  auto refill = [&](uint64_t& b, uint64_t& e) {  // (SHARD)
    if (lane == 0) {
      uint64_t bb = P, ee = P;
      uint32_t k = (uint32_t)pool[4];
      for (; k < ndisp; ++k) {
        const uint32_t d = (blockIdx.x + k) & (ndisp - 1u);
        const uint64_t g = atomicAdd(dispenser + d * DISP_STRIDE, 1ull) * ndisp + d;  // the pass's batch g
        if (g < NB) {
          bb = g * batch;
          ee = bb + batch < P ? bb + batch : P;
          break;
        }
      }
      pool[2] = bb;
      pool[SHARD ? 3 : 0] = ee;
      pool[SHARD ? 4 : 0] = k;
    }
    b = rfl64(pool[2]);
    e = rfl64(pool[SHARD ? 3 : 0]);
  };
  // SRING: the wave's ring of 64 path starts, made by all 64 lanes at once from 64 consecutive ids of its pool and
  // taken by the lanes that regenerate (start_path is a function of the id alone, so which lane makes a path's start
  // changes nothing).  start_path at full lane occupancy instead of the few idle lanes of each regeneration.
  // Per lane slot: o, d, time, rng (2 words), pid (10 words, structure of arrays); rng = 0 marks an off-image id.
  // (the rect list kernel only: its LDS is free and its VGPRs hold the generation; the LDS-node and mesh kernels have
  // no LDS left for 2.5 KB per wave at their occupancy)
  constexpr bool SRING = RTW_SRING && FEAT == (F_BOXES | F_LIST) && !LST;
  __shared__ uint32_t ring_lds[SRING ? (BLK / 64) * 640 : 1];
  __shared__ uint32_t ring_head_lds[SRING ? BLK / 64 : 1];
  uint32_t* const ring = ring_lds + (SRING ? (threadIdx.x >> 6) * 640u : 0u);
  uint32_t* const ring_head = ring_head_lds + (SRING ? threadIdx.x >> 6 : 0u);
  if (SRING && lane == 0) ring_head[0] = 64u;
  bool exhausted = false;                // wave-uniform
  bool has = false;
  TraceState ts;
  ts.on = false;
  PathState st;
  st.pid = 0;
  st.rng = 0;
  st.depth = 0;
  // COUNT: wave-cycles in regeneration / traversal / shading, then the sub-phases: shading's
  // rejection sampling, traversal's node loop and leaf tests, regeneration's start_path
  uint64_t ph[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // [7..10]: RTW_LANE_DIAG builds only
  const uint64_t t_start = COUNT ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t t_mark = t_start;
  auto phase = [&](int k) {
    if (COUNT) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph[k] += t - t_mark;
      t_mark = t;
    }
  };
  for (;;) {
    phase(2);
    // ---- regeneration: compact new path ids into the idle lanes
    const uint64_t need = __ballot(!has);
    if constexpr (SRING) {
      if (need != 0 && !exhausted && ((uint32_t)__popcll(need) >= a.regen_min || need == __ballot(1))) {
        const uint32_t n_need = (uint32_t)__popcll(need);
        const uint32_t rank =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        const uint64_t t_sp = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t head = (uint32_t)__builtin_amdgcn_readfirstlane((int)ring_head[0]);
        const uint32_t have = 64u - head;
        auto take = [&](uint32_t e) {
          const uint32_t lo = ring[7 * 64 + e], hi = ring[8 * 64 + e];
          st.ray.o = mk(__uint_as_float(ring[e]), __uint_as_float(ring[64 + e]), __uint_as_float(ring[2 * 64 + e]));
          st.ray.d = mk(__uint_as_float(ring[3 * 64 + e]), __uint_as_float(ring[4 * 64 + e]),
                        __uint_as_float(ring[5 * 64 + e]));
          st.ray.time = __uint_as_float(ring[6 * 64 + e]);
          st.rng = ((uint64_t)hi << 32) | lo;
          st.pid = ring[9 * 64 + e];
          st.T = mk(1.f, 1.f, 1.f);
          st.depth = SA.max_depth;
          has = (lo | hi) != 0u;
        };
        const bool first = !has && rank < have;
        if (first) take(head + rank);
        if (n_need > have) {  // the ring is spent: 64 more starts from the pool (refilled by one atomic per batch)
          uint64_t pool_next = rfl64(pool[0]), pool_end = rfl64(pool[1]);
          if (pool_next >= pool_end) {
            if constexpr (SHARD) {
              refill(pool_next, pool_end);
            } else {
              if (lane == 0) pool[2] = atomicAdd(dispenser, (unsigned long long)batch);
              const uint64_t b = rfl64(pool[2]);
              pool_next = b < P ? b : P;
              pool_end = b < P ? (b + batch < P ? b + batch : P) : P;
            }
          }
          if (pool_next < pool_end) {  // pools and passes hold whole multiples of 64 ids
            const uint64_t id = pool_next + lane;
            PathState g;
            const bool ok = start_path<SLDS, 0, 0, AB>(SA, id, g);
            ring[lane] = __float_as_uint(g.ray.o.x);
            ring[64 + lane] = __float_as_uint(g.ray.o.y);
            ring[2 * 64 + lane] = __float_as_uint(g.ray.o.z);
            ring[3 * 64 + lane] = __float_as_uint(g.ray.d.x);
            ring[4 * 64 + lane] = __float_as_uint(g.ray.d.y);
            ring[5 * 64 + lane] = __float_as_uint(g.ray.d.z);
            ring[6 * 64 + lane] = __float_as_uint(g.ray.time);
            ring[7 * 64 + lane] = ok ? (uint32_t)g.rng : 0u;
            ring[8 * 64 + lane] = ok ? (uint32_t)(g.rng >> 32) : 0u;
            ring[9 * 64 + lane] = (uint32_t)id;
            pool_next += 64u;
            if (!has && !first) take(rank - have);
            head = n_need - have;
          } else {
            exhausted = true;  // no ids left: the ring stays empty
            head = 64u;
          }
          if (lane == 0) { pool[0] = pool_next; pool[1] = pool_end; }
        } else {
          head += n_need;
        }
        if (lane == 0) ring_head[0] = head;
        if (COUNT) ph[6] += __builtin_amdgcn_s_memtime() - t_sp;  // wave-uniform
      }
    } else if (need != 0 && !exhausted && ((uint32_t)__popcll(need) >= a.regen_min || need == __ballot(1))) {
      const uint32_t n_need = (uint32_t)__popcll(need);
      const uint32_t rank =
          __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      uint64_t pool_next = rfl64(pool[0]), pool_end = rfl64(pool[1]);
      const uint64_t avail = pool_end - pool_next;
      uint64_t nb = P, ne = P;
      if (avail < n_need) {  // refill: one atomic per BATCH paths
        // lane 0 takes BATCH ids and hands them to the wave through LDS (a `b = 0` default
        // for the other lanes would be one more loop-carried VGPR pair)
        if constexpr (SHARD) {
          uint64_t b, e;
          refill(b, e);
          if (b < e) {
            nb = b;
            ne = e;
          } else {
            exhausted = true;
          }
        } else {
          if (lane == 0) pool[2] = atomicAdd(dispenser, (unsigned long long)batch);
          const uint64_t b = rfl64(pool[2]);
          if (b < P) {
            nb = b;
            ne = b + batch < P ? b + batch : P;
          } else {
            exhausted = true;
          }
        }
      }
      const uint64_t t_sp = COUNT ? __builtin_amdgcn_s_memtime() : 0;
      if (!has) {
        const uint64_t id = rank < avail ? pool_next + rank : nb + (rank - avail);
        if ((rank < avail || id < ne) && start_path<SLDS, LST ? BLK : 0, LST_ROW0, AB>(SA, id, st, stk16)) {
          has = true;
        }
      }
      if (COUNT) ph[6] += __builtin_amdgcn_s_memtime() - t_sp;  // wave-uniform
      if (avail >= n_need) {
        pool_next += n_need;
      } else {
        pool_next = nb + (n_need - avail);
        pool_end = ne;
        if (pool_next > pool_end) pool_next = pool_end;
      }
      if (lane == 0) { pool[0] = pool_next; pool[1] = pool_end; }
    }
    if (__ballot(has) == 0) {
      if (exhausted) break;
      continue;  // every id handed out this round was an off-image pixel: draw again
    }
    phase(0);
    // segments starting now, counted per wave with every lane active (so the count is uniform
    // and stays in SGPRs)
    nrays += (unsigned long long)__popcll(__ballot(has && !ts.on));
    if (!has) continue;
    // ---- one segment: closest hit (resumable) + shading (lib.rs:97-117)
    if (!ts.on) {
      trace_begin<COUNT, FEAT, STACK, BLK, (NCAP > 0 || S16), (HN ? 0 : NCAP)>(S, st.ray, ts, cnt, st.rng, stk16, stk,
                                                                              a.err, nodes_lds);
    }
    if (!(FEAT & F_LIST)) {
      const uint32_t act = (uint32_t)__popcll(__ballot(1));
      const uint32_t quota = (act * a.quota16 + 15u) >> 4;
      const uint32_t leaf_thr = (act * a.leaf16 + 15u) >> 4;
      trace_run<COUNT, STACK, SPILL, FEAT, BLK, NCAP, HN, S16>(S, st.ray, ts, stk, spill, a.spill_lanes, cnt, quota,
                                                      leaf_thr, st.rng, a.err, ph + 4, nodes_lds, stk16);
    } else {
      ts.node = -1;  // list mode: trace_begin tested every primitive
      ts.sp = 0;
    }
    phase(1);
    __builtin_amdgcn_s_setprio(0);  // trace_run raised it
    if (ts.node >= 0 || ts.sp > 0) continue;  // traversal suspended: resume next iteration
    ts.on = false;
    if (COUNT) simd_tick(cnt, 12, 13);
    const Best b = ts.b;
#ifdef RTW_DIAG_TRACE_PID  // debugging aid (never in the product build): one path's segments via device printf
    if ((RTW_DIAG_TRACE_PID) < 0 || st.pid == (uint32_t)(RTW_DIAG_TRACE_PID))  // < 0: every path
      printf("rtwtrace pid %u o %a %a %a d %a %a %a t %a prim %d key %u rng %016llx\n", st.pid, st.ray.o.x, st.ray.o.y,
             st.ray.o.z, st.ray.d.x, st.ray.d.y, st.ray.d.z, b.t, b.prim, b.prim >= 0 ? S.prims[b.prim].key : 0u,
             (unsigned long long)st.rng);
#endif
    bool done = false;
    V3 L = mk(0.f, 0.f, 0.f);
    // the throughput; the S16 mesh walk reads it from its LDS rows where it is used, after the hit record and the
    // material, so it is not held across them (the 7-wave walk had spilled T.z to scratch there; s1)
    const V3 T0 = (LST && !S16) ? mk(__uint_as_float(lst_ld(0)), __uint_as_float(lst_ld(1)), __uint_as_float(lst_ld(2)))
                                : st.T;
    auto path_T = [&]() -> V3 {
      return (LST && S16) ? mk(__uint_as_float(lst_ld(0)), __uint_as_float(lst_ld(1)), __uint_as_float(lst_ld(2))) : T0;
    };
    if (b.prim < 0) {  // lib.rs:102-105
      L = mul(path_T(), bg);
      done = true;
      if (__builtin_expect(b.prim == -2, 0)) {
        // trace_run tripped its guard (a corrupt tree; the frame is invalid and reported): close the path queue
        // for every wave and empty this wave's id pool, so the grid drains after about one trip per wave
        // instead of one per 64 paths (a trip is 2^20 node-loop iterations)
        if constexpr (SHARD) {
          for (uint32_t d = 0; d < DISP; ++d) atomicMax(dispenser + d * DISP_STRIDE, (unsigned long long)NB);
        } else {
          atomicMax(dispenser, (unsigned long long)P);
        }
        pool[0] = pool[1];
      }
    } else {
      // the prim's shading record is loaded as soon as the winner is known, beside its geometry
      // (one load instead of the prim -> material -> texture -> checker-child chain)
      // (LST: the second half, the checker's even colour, is read where it is used: held across the hit
      // record it was spilled to scratch)
      DevShade sh;
      if constexpr (LST) {
        const float4 q = *reinterpret_cast<const float4*>(S.shade + b.prim);
        sh.kind = __float_as_uint(q.x); sh.param = q.y; sh.a[0] = q.z; sh.a[1] = q.w;
        sh.a[2] = S.shade[b.prim].a[2];
      } else {
        sh = S.shade[b.prim];
      }
      // a light of one solid colour (light_source.rs:17-24 with SolidColor) needs no hit record: its
      // emission is the colour and it never scatters (the cow's emitting mesh; mesh kernels only: the
      // extra branch measured 0.7% slower on cornell-box)
      const bool solid_light = (FEAT & F_LIGHT) && (FEAT & F_TRI) && (sh.kind & 0xfffu) == (MT_LIGHT | (SM_SOLID << 8));
      Rec h;
      if (!solid_light) h = hit_record<FEAT>(S, st.ray, b, sh.kind);
      else h = Rec{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), 0.0f, 0.0f, true, 0u};
#ifdef RTW_SHADE_DIAG  // COUNT-build diagnostic: shading sub-phases (hit record, unit + texture, scatter) in ph[7..9]
      phase(7);
#endif
      // One body for every material (material.rs:42-165, light_source.rs:17-24): a wave mixing
      // materials runs the rejection loop, unit() and the texture lookup once instead of once per
      // material branch.  Each material's draws and f32 operations are unchanged.
      const uint32_t mt = sh.kind & 0xffu, mode = (sh.kind >> 8) & 0xfu;
      const bool light = (FEAT & F_LIGHT) && mt == MT_LIGHT;
      const bool lam = (FEAT & F_LAMBERT) && mt == MT_LAMBERT;
      const bool met = (FEAT & F_METAL) && mt == MT_METAL;
      const bool iso = (FEAT & F_ISO) && mt == MT_ISOTROPIC;
      V3 rs = mk(0.f, 0.f, 0.f);
      phase(2);
      if (lam || met || iso) rs = rand_in_unit_sphere<AB>(st.rng);  // vec3.rs:101-108
      phase(3);
      const V3 ud = unit(lam ? rs : st.ray.d);                  // Lambertian: unit(rs); else unit(d_in)
      V3 att = mk(1.f, 1.f, 1.f);                                 // Dielectric: attenuation (1,1,1)
      if (met) {
        att = ld3(sh.a);
      } else if (light || lam || iso) {
        if (mode == SM_SOLID) att = ld3(sh.a);  // SolidColor::value
        else if ((FEAT & F_CHECKER) && mode == SM_CHECKER)
          att = checker_odd(sh.param * h.p.x, sh.param * h.p.y, sh.param * h.p.z) ? ld3(sh.a)
                                                                                   : ld3(LST ? S.shade[b.prim].b : sh.b);
        else if ((FEAT & F_IMAGE) && mode == SM_IMAGE)  // (the monument's texture: no record chain)
          att = image_texel(S, __float_as_uint(sh.a[0]), __float_as_uint(sh.a[1]), __float_as_uint(sh.a[2]), h.u, h.v);
        else if (FEAT & F_TEXGEN) att = tex_value<FEAT>(S, S.mats[h.mat].tex, h.u, h.v, h.p);
      }
#ifdef RTW_SHADE_DIAG
      phase(8);
#endif
      V3 Tn = mk(0.f, 0.f, 0.f);  // the throughput after this segment (scattering materials)
      if (light) {  // emit, no scatter
        L = mul(path_T(), att);
        done = true;
      } else {
        V3 dir = rs;  // Isotropic (material.rs:155-165): never absorbs
        if (lam) {    // material.rs:42-56
          dir = add(h.n, ud);
          if (near_zero(dir)) dir = h.n;
        } else if (met) {  // material.rs:78-95
          dir = add(reflect(ud, h.n), scale(rs, sh.param));
          done = !(dot(dir, h.n) > 0.0f);  // absorbed: emitted() is black
        } else if (!iso && (FEAT & F_DIEL)) {  // Dielectric, material.rs:116-142
          // 1 / ir (material.rs:120) and Schlick's r0 (:108-112) for both ratios: the same f32
          // operations, evaluated once by the flattener (DevShade::a)
          const float ratio = h.front ? sh.a[0] : sh.param;
          const float r0 = h.front ? sh.a[1] : sh.a[2];
          const float cos_t = fminf(dot(neg(ud), h.n), 1.0f);
          const float sin_t = sqrtf(1.0f - cos_t * cos_t);
          const bool cannot = (ratio * sin_t) > 1.0f;
          if (cannot || reflectance(cos_t, r0) > gen_f32(st.rng)) dir = reflect(ud, h.n);
          else dir = refract(ud, h.n, ratio);
        }
        const V3 Tp = path_T();
        const V3 T2 = mul(Tp, att);  // x * 1.0f == x: the Dielectric's T is unchanged
        // an absorbed Metal ray returns emitted() = black (material.rs:87, lib.rs:109-110), which the recursion's
        // parents multiply by their attenuations: T * 0, not a constant 0 (NaN / inf throughputs propagate, a
        // negative one gives -0; round 6, a fuzz world whose sphere uv was NaN)
        if (done) L = mul(Tp, mk(0.f, 0.f, 0.f));
        Tn = T2;
        if constexpr (LST) {
          lst_st(0, __float_as_uint(T2.x));
          lst_st(1, __float_as_uint(T2.y));
          lst_st(2, __float_as_uint(T2.z));
        } else {
          st.T = T2;
        }
        st.ray.o = h.p;
        st.ray.d = dir;
      }
#ifdef RTW_SHADE_DIAG
      phase(9);
#endif
      if (!done) {  // lib.rs:98-100: depth 0 returns black, times the attenuations above it (T * 0, as above)
        if constexpr (LST) {
          const uint32_t d = lst_ld(3) - 1u;
          lst_st(3, d);
          done = d == 0u;
        } else {
          done = --st.depth == 0u;
        }
        if (done) L = mul(Tn, mk(0.f, 0.f, 0.f));
      }
    }
    if (done) {
      float* o = a.sbuf + (size_t)(LST ? lst_ld(4) : st.pid) * 3u;  // one path's 12 B share a cache line
#ifdef RTW_DIAG_NO_STORE  // timing diagnostic only: what the sample stores (and the waits behind them) cost
      if (L.x == -1.2345f) o[0] = L.y;  // (keeps L live; never true for a finite non-negative radiance)
#else
#if RTW_NT_SAMPLES
      // streaming stores: the 12.7 GB of samples per frame should not evict the scene tables and the
      // register spill lines from L2 (they are read back once, by reduce_kernel)
      __builtin_nontemporal_store(L.x, o);
      __builtin_nontemporal_store(L.y, o + 1);
      __builtin_nontemporal_store(L.z, o + 2);
#else
      o[0] = L.x;
      o[1] = L.y;
      o[2] = L.z;
#endif
#endif  // RTW_DIAG_NO_STORE
      has = false;
    }
  }
  if (lane == 0 && nrays) atomicAdd(a.counters, nrays);  // nrays counts the whole wave's segments
  if (COUNT) {
    phase(2);
    if (lane == 0) {
      for (int k = 0; k < 3; ++k) atomicAdd(a.counters + 16 + k, (unsigned long long)ph[k]);
      atomicAdd(a.counters + 19, (unsigned long long)(t_mark - t_start));
#if defined(RTW_LANE_DIAG) || defined(RTW_UNI_DIAG) || defined(RTW_SHADE_DIAG)
      for (int k = 7; k < 11; ++k) atomicAdd(a.counters + 13 + k, (unsigned long long)ph[k]);
#else
      for (int k = 3; k < 7; ++k) atomicAdd(a.counters + 17 + k, (unsigned long long)ph[k]);
#endif
    }
    for (int q = 0; q < 15; ++q) {
      unsigned long long c = cnt[q];
      for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
      if (lane == 0 && c) atomicAdd(a.counters + 1 + q, c);
    }
  }
}

#ifndef RTW_MESH_TU  // (rtw_kernel_mesh.hip compiles only the mesh path kernels: see pick_mesh)
// Σ over samples in sample order (lib.rs:83-87), one thread per pixel of the pass.
__global__ __launch_bounds__(256) void reduce_kernel(RenderArgs a, uint32_t n_slots) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_slots * 64u) return;
  const uint32_t slot = g >> 6, l = g & 63u, gslot = a.slot_base + slot;
  const uint32_t tile = a.tile_ids ? a.tile_ids[gslot] : a.tile_first + gslot * a.tile_stride;
  const uint32_t i = (tile % a.tiles_x) * 8u + (l & 7u), row = (tile / a.tiles_x) * 8u + (l >> 3);
  if (i >= a.w || row >= a.h) return;
  float x = 0.f, y = 0.f, z = 0.f;
  const float* q = a.sbuf + ((size_t)slot * a.spp * 64u + l) * 3u;
  for (uint32_t s = 0; s < a.spp; ++s, q += 64u * 3u) {
#if RTW_NT_SAMPLES
    x = x + __builtin_nontemporal_load(q);
    y = y + __builtin_nontemporal_load(q + 1);
    z = z + __builtin_nontemporal_load(q + 2);
#else
    x = x + q[0];
    y = y + q[1];
    z = z + q[2];
#endif
  }
  float* o = a.packed_out ? a.out + ((size_t)gslot * 64u + l) * 3u : a.out + ((size_t)row * a.w + i) * 3u;
  o[0] = x;
  o[1] = y;
  o[2] = z;
}

__global__ void unpack_tiles_kernel(uint32_t w, uint32_t h, uint32_t tiles_x, const uint32_t* tiles,
                                    uint32_t n_tiles, const float* packed, float* img) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_tiles * 64u) return;
  const uint32_t t = g >> 6, lane = g & 63u, tile = tiles[t];
  const uint32_t i = (tile % tiles_x) * 8u + (lane & 7u), row = (tile / tiles_x) * 8u + (lane >> 3);
  if (i >= w || row >= h) return;
  for (int c = 0; c < 3; ++c) img[((size_t)row * w + i) * 3 + c] = packed[(size_t)g * 3 + c];
}

// Diagnostics (rtw_diag_libm): the render path's f32 transcendentals over arrays.
__global__ void libm_kernel(int fn, uint32_t n, const float* a, const float* b, float* out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const float x = a[g];
  if (fn == 4) {  // the camera division: Markstein's correction from the IEEE reciprocal (= RN(1 / b))
    out[g] = div_by_recip(x, b[g], 1.0f / b[g]);
    return;
  }
  if (fn == 5) {  // the sphere test's sqrt
    out[g] = sqrt_rn(x);
    return;
  }
  out[g] = fn == 0 ? dev_log10f(x) : (fn == 1 ? dev_sinf(x) : (fn == 2 ? dev_acosf(x) : dev_atan2f(x, b[g])));
}

// Diagnostics (rtw_diag_sweep): every 32-bit pattern in [lo, hi] as a float b, compared bit for bit
// (NaN == NaN) against the IEEE operation.  fn 0: rcp_rn_fast(b) vs 1.0f / b over the range rcp_rn_ok
// accepts (others are skipped: counted in n[1]).  n[0] = mismatches; the first `cap` are recorded.
__global__ void sweep_kernel(int fn, uint32_t lo, uint32_t hi, unsigned long long* n, uint32_t* bad, uint32_t cap) {
  const uint64_t span = (uint64_t)hi - lo + 1u;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long nbad = 0, nskip = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < span; k += stride) {
    const uint32_t bits = lo + (uint32_t)k;
    const float b = __uint_as_float(bits);
    bool ok = true;
    if (fn == 0) {
      if (!rcp_rn_ok(b)) {
        ++nskip;
        continue;
      }
      const float f = rcp_rn_fast(b), r = 1.0f / b;
      ok = __float_as_uint(f) == __float_as_uint(r) || (f != f && r != r);
    }
    if (!ok) {
      const unsigned long long slot = atomicAdd(n + 2, 1ull);
      if (slot < cap) bad[slot] = bits;
      ++nbad;
    }
  }
  if (nbad) atomicAdd(n, nbad);
  if (nskip) atomicAdd(n + 1, nskip);
}
#endif  // RTW_MESH_TU

}  // namespace dev

// Variants of the path kernel: feature set x the waves per SIMD the register allocator must allow.
// Sphere-only scenes (jumpy-balls) get the specialised kernel; everything else the generic one.
// Trees whose push bound exceeds the LDS stack get the SPILL variant.  Default: 5 waves/SIMD.
// Tuning knobs: RTW_OCC=4 (33-row stack) or RTW_OCC=6 (specialised kernel; spills registers);
// RTW_STACK_LDS=4 selects a generic kernel with a 4-entry LDS stack, so that the HBM spill path
// runs on every scene (tests/test_gpu_parity.py).
typedef void (*path_fn)(RenderArgs);
static int env_int(const char* k, int dflt) {  // a tuning knob (read only with RTW_TUNING=1)
  const char* e = strcmp(k, "RTW_VERBOSE") ? tuning_env(k) : getenv(k);  // RTW_VERBOSE only prints
  return e ? atoi(e) : dflt;
}
struct Variant {
  path_fn fn;
  uint32_t stack;        // LDS stack rows of fn; a deeper push bound spills to HBM (RenderArgs::spill)
  uint32_t block = 256;  // workgroup size fn is compiled for
  bool k16 = false;      // LDS-node kernel (sorted-push walk)
  bool sring = false;    // path starts from the wave's ring (path_kernel SRING)
};
// LDS-node variants: the node table lives in each workgroup's LDS.  512-lane workgroups at 6
// waves/SIMD = 3 per CU: 24 rows of 16-bit stack entries x 512 x 2 B + 224 node4s x 128 B + the pool
// words = 53,440 B per workgroup, 160,320 B per CU (<= 160 KiB): sphere worlds of up to ~850 spheres.
constexpr int LDSN_STACK = 24, LDSN_CAP = 224, LDSN_BLK = 512;
// (The spheres' 32-B test records in LDS too -- 18 stack rows, 512 x 32 B -- and the winner's hit record
// from them measured equal within 0.2%: profiles/r02/experiments n6, h2.)
template <bool C, uint32_t F>
static Variant pick5(uint32_t need, bool half = false, bool codes16 = false) {
  using namespace dev;
  if constexpr (F == F_MESHES) {
    // 16-bit stack entries (the nodes' codes: half the LDS of the 32-bit stack, whose 31 KB per workgroup allow
    // 5 per CU) and the paths' T / depth / id in LDS state rows, at 6 or 7 waves / SIMD (knob RTW_MESH_S16; 0 =
    // the 32-bit stack at 5).  Measured (r04n, r04p): monument-4k +3.0% at 6 waves (80 VGPRs), +2.2% more with
    // the state rows (scratch 40 -> 32 B), 7 waves slower; cow-1080p -4.1% / -0.7% with the rows.  With the
    // start_path operands in LDS (round 5, m1) the SGPR overflow is gone and 7 waves (72 VGPRs) win: monument
    // +2.3%, cow +0.8% over 6 (profiles/r05/experiments, m2), so every tree with half nodes takes the 7-wave walk.
    int s16 = env_int("RTW_MESH_S16", half ? 7 : 0);
    if (s16 != 0 && s16 != 6 && s16 != 7) {  //  no silent fallback for a value no variant has
      fprintf(stderr, "rtw: RTW_MESH_S16=%d ignored (0, 6 or 7)\n", s16);
      s16 = half ? 7 : 0;
    }
    if (codes16 && s16 != 0 && need <= (uint32_t)STACK_DEEP5) {
      const uint32_t st = (uint32_t)STACK_DEEP5;
      if (s16 == 7)
        return half ? Variant{path_kernel<C, STACK_DEEP5, false, 7, F, BLOCK, 0, true, true>, st}
                    : Variant{path_kernel<C, STACK_DEEP5, false, 7, F, BLOCK, 0, false, true>, st};
      return half ? Variant{path_kernel<C, STACK_DEEP5, false, 6, F, BLOCK, 0, true, true>, st}
                  : Variant{path_kernel<C, STACK_DEEP5, false, 6, F, BLOCK, 0, false, true>, st};
    }
  }
  if constexpr (F == F_MESHES) {  // the half-precision node table (DevNode4h) where it was built
    if (half && need <= (uint32_t)STACK_LDS5)
      return {path_kernel<C, STACK_LDS5, false, 5, F, BLOCK, 0, true>, (uint32_t)STACK_LDS5};
    if (half && need <= (uint32_t)STACK_DEEP5)
      return {path_kernel<C, STACK_DEEP5, false, 5, F, BLOCK, 0, true>, (uint32_t)STACK_DEEP5};
  }
  if (need <= (uint32_t)STACK_LDS5) return {path_kernel<C, STACK_LDS5, false, 5, F>, (uint32_t)STACK_LDS5};
  if constexpr (F == F_MESHES || F == F_ALL) {
    if (need <= (uint32_t)STACK_DEEP5) return {path_kernel<C, STACK_DEEP5, false, 5, F>, (uint32_t)STACK_DEEP5};
    return {path_kernel<C, STACK_DEEP5, true, 5, F>, (uint32_t)STACK_DEEP5};
  }
  return {path_kernel<C, STACK_LDS5, true, 5, F>, (uint32_t)STACK_LDS5};
}
// The mesh variants (F_MESHES) are compiled in their own translation unit, rtw_kernel_mesh.hip, with the
// iterative-ILP machine scheduler instead of max-ILP (Makefile KFLAGS_MESH): cow +0.6%, monument +1.2%, where the
// sphere and list-mode kernels lose 0.7-0.8% with it (profiles/r04/experiments k1)
Variant pick_mesh(bool count, uint32_t need, bool half, bool codes16);

#ifndef RTW_MESH_TU

// ---------------------------------------------------------------- host side
static int hip_fail(hipError_t e, const char* what) {
  return fail(RTW_ENODEV, "%s: %s", what, hipGetErrorString(e));
}
#define HIPCHK(x, what)                          \
  do {                                           \
    hipError_t e_ = (x);                         \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

template <class T>
static size_t put(std::vector<uint8_t>& blob, const std::vector<T>& v) {
  size_t off = (blob.size() + 255) & ~(size_t)255;
  blob.resize(off + sizeof(T) * v.size());
  if (!v.empty()) memcpy(blob.data() + off, v.data(), sizeof(T) * v.size());
  return off;
}

int upload(Scene& s, int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(RTW_ENODEV, "no HIP device visible (the render core has no CPU fallback)");
  const int nlog = s.alias_n > 0 ? s.alias_n : ndev;  // logical devices (rtw_diag_alias_devices: all on 0)
  if (device >= nlog) return fail(RTW_EINVAL, "device %d >= device count %d", device, nlog);
  const Flat& f = s.flat;
  std::vector<uint8_t> blob;
  // the far-origin record sits DEVFAR_BACK bytes before the prim table (trace_begin derives it from S.prims)
  DevFar far = f.far;
  const size_t o_nodes = put(blob, f.nodes4), o_far = put(blob, std::vector<DevFar>{far});
  size_t o_prims = put(blob, f.prims), o_always = put(blob, f.always);
  if (o_prims - o_far != DEVFAR_BACK) return fail(RTW_EINVAL, "internal: far record not %u B before the prims", DEVFAR_BACK);
  reinterpret_cast<DevFar*>(blob.data() + o_far)->nodes_back = (uint32_t)(o_prims - o_nodes);
  size_t o_tsh = put(blob, f.tshade), o_inst = put(blob, f.insts), o_mat = put(blob, f.mats);
  size_t o_tex = put(blob, f.texs), o_texel = put(blob, f.texels), o_perlin = put(blob, f.perlins);
  size_t o_shade = put(blob, f.shade), o_hnodes = put(blob, f.nodes4h), o_groups = put(blob, f.lgroups);
  blob.resize((blob.size() + 255) & ~(size_t)255);
  int d0 = device >= 0 ? device : 0, d1 = device >= 0 ? device + 1 : nlog;
  int prev = 0;
  hipGetDevice(&prev);
  for (int d = d0; d < d1; ++d) {
    const int phys = s.alias_n > 0 ? 0 : d;
    HIPCHK(hipSetDevice(phys), "hipSetDevice");
    DeviceCopy c;
    c.device = d;
    c.phys = phys;
    c.bytes = blob.size();
    HIPCHK(hipMalloc(&c.block, c.bytes), "hipMalloc(scene)");
    HIPCHK(hipMemcpy(c.block, blob.data(), c.bytes, hipMemcpyHostToDevice), "hipMemcpy(scene)");
    HIPCHK(hipMalloc((void**)&c.counters, COUNTER_WORDS * sizeof(unsigned long long)), "hipMalloc(counters)");
    // the sticky traversal-error word lives in host memory the kernel writes through (coherent,
    // mapped): the host reads it without a device round trip, also for renders it did not wait for
    HIPCHK(hipHostMalloc((void**)&c.err_host, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc(error word)");
    *(volatile uint32_t*)c.err_host = 0u;
    uint8_t* base = (uint8_t*)c.block;
    c.scene.nodes = (const DevNode4*)(base + o_nodes);
    c.scene.hnodes = f.nodes4h.empty() ? nullptr : (const DevNode4h*)(base + o_hnodes);
    c.scene.prims = (const DevPrim*)(base + o_prims);
    c.scene.always = (const uint32_t*)(base + o_always);
    c.scene.tshade = (const DevTriShade*)(base + o_tsh);
    c.scene.insts = (const DevInst*)(base + o_inst);
    c.scene.mats = (const DevMat*)(base + o_mat);
    c.scene.texs = (const DevTex*)(base + o_tex);
    c.scene.texels = (const uint8_t*)(base + o_texel);
    c.scene.perlins = (const DevPerlin*)(base + o_perlin);
    c.scene.shade = (const DevShade*)(base + o_shade);
    c.scene.lgroups = (const DevGroup*)(base + o_groups);
    c.scene.n_lgroups = (uint32_t)f.lgroups.size();
    c.scene.n_nodes = (uint32_t)f.nodes4.size();
    c.scene.n_prims = (uint32_t)f.prims.size();
    c.scene.n_always = (uint32_t)f.always.size();
    c.scene.n_insts = (uint32_t)f.insts.size();
    c.scene.msphere_unit = f.msphere_unit;
    c.scene.uni_inst = f.uni_inst;
    c.scene.bvh_tri = f.bvh_tri;  // knob RTW_TRI_LEAF (rtw_flatten.cpp)
    c.scene.tri_inst = f.tri_inst;
    c.scene.rect_fast = f.rect_fast;
    memcpy(c.scene.uni_off, f.uni_off, sizeof f.uni_off);
    c.scene.far_check = f.far_check;
    s.dev.push_back(c);
  }
  hipSetDevice(prev);
  return RTW_OK;
}

static void free_buf(DevBuf& b) {
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

void release(Scene& s) {
  for (DeviceCopy& c : s.dev) {
    if (hipSetDevice(c.phys) != hipSuccess) continue;
    if (c.block) hipFree(c.block);
    if (c.counters) hipFree(c.counters);
    if (c.err_host) hipHostFree(c.err_host);
    if (c.sbuf) hipFree(c.sbuf);
    if (c.spill) hipFree(c.spill);
    for (DevBuf* b : {&c.image, &c.tiles, &c.packed, &c.gathered, &c.gather_ids}) free_buf(*b);
    for (void* e : c.ev)
      if (e) hipEventDestroy(static_cast<hipEvent_t>(e));
    for (void* e : c.gev)
      if (e) hipEventDestroy(static_cast<hipEvent_t>(e));
    if (c.stream) hipStreamDestroy(static_cast<hipStream_t>(c.stream));
    for (auto& e : c.kev)
      for (void* x : e)
        if (x) hipEventDestroy(static_cast<hipEvent_t>(x));
  }
  s.dev.clear();
}

DeviceCopy* find_copy(Scene& s, int device) {
  for (DeviceCopy& c : s.dev)
    if (c.device == device || device < 0) return &c;
  return nullptr;
}

int grow(DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return RTW_OK;
  free_buf(b);
  HIPCHK(hipMalloc(&b.p, bytes), "hipMalloc(render buffer)");
  b.cap = bytes;
  return RTW_OK;
}

// the scene copy's event pair (created once)
static int copy_events(DeviceCopy& c, hipEvent_t& e0, hipEvent_t& e1) {
  for (void*& e : c.ev)
    if (!e) {
      hipEvent_t x;
      HIPCHK(hipEventCreate(&x), "hipEventCreate");
      e = x;
    }
  e0 = static_cast<hipEvent_t>(c.ev[0]);
  e1 = static_cast<hipEvent_t>(c.ev[1]);
  return RTW_OK;
}

// Paths per pass (ordered sample buffer = 12 B per path): 2^32 = 51.5 GB of the 288 GB HBM.  A frame
// with more paths (monument 4K x 1024 spp: 8.5 G, 2 passes) runs in several passes, each one persistent
// launch + its in-order reduction.  Tuning knob RTW_PASS_LOG2 (24..33).
static uint64_t max_pass_paths() {
  const char* e = tuning_env("RTW_PASS_LOG2");
  const int l = e ? std::min(32, std::max(24, atoi(e))) : 32;  // PathState::pid is 32-bit
  return 1ull << l;
}

template <bool C>
static Variant pick_kernel(uint32_t feat, uint32_t need, bool list, uint32_t n_nodes, uint32_t need4,
                           bool codes16, bool has_half, bool far) {
  using namespace dev;
  if (env_int("RTW_STACK_LDS", 0) == 4) return {path_kernel<C, 4, true, 4, F_ALL>, 4u};  // spill-path test
  const bool sph = (feat & ~F_SPHERES) == 0;
  // Half-precision nodes (DevNode4h, built when the 16-bit codes fit) trade vector-memory traffic (4 loads /
  // 64 B per visit instead of 7 / 112 B) for VALU issue (v_fma_mix_f32 issues ~1.3x slower than v_fma_f32,
  // scripts/ubench/mix_rate.hip; +5 VALU per visit).  Measured (profiles/r03/experiments, h1): monument-4k
  // +3.3% (its 2,226-node tree), cow-1080p -6.5% (1,591 nodes), jumpy-1080p -4.9% (LDS nodes) at round 3's 5-wave
  // mesh kernel.  With round 4's 6-wave mesh walk (16-bit stack, LDS state rows; pick5) the cow gains too (r04q:
  // +1.8%), so every mesh tree with a half table uses it by default; the LDS-node sphere kernels keep f32 nodes.
  // Knob RTW_HALF_NODES 1 = wherever built (LDS-node kernels too), 0 = never.
  const int half_knob = env_int("RTW_HALF_NODES", -1);
  // (no half-precision table when a bound is beyond f16's range: rtw_flatten.cpp half_node)
  const bool half = has_half && half_knob != 0;
  const bool half_lds = has_half && half_knob > 0;
  if (list) {
    // RTW_GENERIC on a list world: the all-features LIST kernel, whose fold is the reference's (NaN candidates, list
    // order); the BVH kernels' fold treats a NaN candidate as a miss
    if (env_int("RTW_GENERIC", 0)) return {path_kernel<C, 1, false, 5, F_ALL | F_LIST>, 1u};
    // no BVH (list mode): variants without the walk.  The rect/instance one needs 56 VGPRs and
    // runs at 8 waves/SIMD (cornell-box on MI355X: 26.7k Mrays/s at 5-6 waves, 28.9k at 7, 29.5k
    // at 8; knob RTW_LIST_OCC); the all-features one spills below 96 VGPRs, so it stays at 5.
    if ((feat & ~F_BOXES) == 0 && !env_int("RTW_LIST_ALL", 0)) {  // knob: the all-features list kernel instead
      if (env_int("RTW_LIST_OCC", 8) == 6) return {path_kernel<C, 1, false, 6, F_BOXES | F_LIST>, 1u, 256u, false, RTW_SRING != 0};
      return {path_kernel<C, 1, false, 8, F_BOXES | F_LIST>, 1u, 256u, false, RTW_SRING != 0};
    }
    return {path_kernel<C, 1, false, 5, F_ALL | F_LIST>, 1u};
  }
  // sphere worlds default to 6 waves/SIMD (24 B/lane of register spill, +1.6% on jumpy-balls over
  // 5 waves once the kernel-uniform values left the VGPRs); the other variants to 5
  switch (env_int("RTW_OCC", sph ? 6 : 5)) {
    case 4: {
      const bool sp = need > (uint32_t)STACK_LDS;
      const uint32_t st = (uint32_t)STACK_LDS;
      if (sph) return {sp ? path_kernel<C, STACK_LDS, true, 4, F_SPHERES> : path_kernel<C, STACK_LDS, false, 4, F_SPHERES>, st};
      return {sp ? path_kernel<C, STACK_LDS, true, 4, F_ALL> : path_kernel<C, STACK_LDS, false, 4, F_ALL>, st};
    }
    case 6: {
      // 8 waves per SIMD when the tree fits a smaller table: 512-lane workgroups x 4 per CU, 144 node4s and 16
      // stack rows in 36 KB of LDS, 64 VGPRs (the compiler spills 32 B per lane to scratch, outside the node
      // loop).  The latency-bound kernel gains from the extra waves: jumpy-1080p 26.34k -> 27.02k Mrays/s
      // (profiles/r03/experiments, w1); 7 waves (448-lane workgroups, 160 node4s, 18 rows, 72 VGPRs) measured
      // slower (25.18k), as did both with half-precision nodes.  Knob RTW_LDSN_WAVES (6, 7, 8).
      const int ldsn_waves = env_int("RTW_LDSN_WAVES", 8);
      if (sph && codes16 && env_int("RTW_LDS_NODES", 1) && ldsn_waves == 7 && need4 <= 18u && n_nodes <= 160u)
        return half_lds ? Variant{path_kernel<C, 18, false, 7, F_SPHERES, 448, 160, true>, 18u, 448u, true}
                        : Variant{path_kernel<C, 18, false, 7, F_SPHERES, 448, 160>, 18u, 448u, true};
      // 1024-lane workgroups x 2 per CU (knob RTW_LDSN_BLK, 512 = the 4 x 512 form): one node table per 16
      // waves, and the LDS this frees holds the paths' T / depth / id (path_kernel LST) that the 64-VGPR
      // budget otherwise spills to scratch.  LDS per workgroup: 18 KB nodes + 32 KB stack + 20 KB state.
      if (sph && codes16 && env_int("RTW_LDS_NODES", 1) && ldsn_waves == 8 && need4 <= 16u && n_nodes <= 144u &&
          !half_lds && env_int("RTW_LDSN_BLK", 1024) == 1024)
        return Variant{path_kernel<C, 16, false, 8, F_SPHERES, 1024, 144>, 16u, 1024u, true};
      if (sph && codes16 && env_int("RTW_LDS_NODES", 1) && ldsn_waves == 8 && need4 <= 16u && n_nodes <= 144u)
        return half_lds ? Variant{path_kernel<C, 16, false, 8, F_SPHERES, 512, 144, true>, 16u, 512u, true}
                        : Variant{path_kernel<C, 16, false, 8, F_SPHERES, 512, 144>, 16u, 512u, true};
      if (sph && codes16 && need4 <= (uint32_t)LDSN_STACK && n_nodes <= (uint32_t)LDSN_CAP &&
          env_int("RTW_LDS_NODES", 1)) {
        if (half_lds)
          return {path_kernel<C, LDSN_STACK, false, 6, F_SPHERES, LDSN_BLK, LDSN_CAP, true>, (uint32_t)LDSN_STACK,
                  (uint32_t)LDSN_BLK, true};
        return {path_kernel<C, LDSN_STACK, false, 6, F_SPHERES, LDSN_BLK, LDSN_CAP>, (uint32_t)LDSN_STACK,
                (uint32_t)LDSN_BLK, true};
      }
      if (sph && need <= (uint32_t)STACK_LDS5) return {path_kernel<C, STACK_LDS5, false, 6, F_SPHERES>, (uint32_t)STACK_LDS5};
    }
      [[fallthrough]];
    default:
      if (env_int("RTW_GENERIC", 0)) return pick5<C, F_ALL>(need);  // parity of the generic kernel
      if (sph) return pick5<C, F_SPHERES>(need);
      if ((feat & ~F_BOXES) == 0) return pick5<C, F_BOXES>(need);
      if ((feat & ~F_SMOKE) == 0) return pick5<C, F_SMOKE>(need);
      if ((feat & ~F_MESHES) == 0) {
        // a partial LDS node cache (the top 128 / 376 / 760 node4s, the rest from global memory, sorted-push
        // walk) measured slower on cow / monument (profiles/r02/experiments, n7): the full-table kernels
        // are for trees that fit
        if (far) return pick5<C, F_ALL>(need);  // spheres in a mesh world's BVH: the mesh kernels have no far path
        return pick_mesh(C, need, half, codes16);
      }
      return pick5<C, F_ALL>(need);
  }
}
static Variant path_kernel_variant(bool count, const Flat& f) {
  const uint32_t feat = f.features, need = f.stack_need, need4 = f.stack_need4, nn = (uint32_t)f.nodes4.size();
  const bool list = f.nodes4.empty();
  const bool hh = f.codes16 && !f.nodes4h.empty();
  return count ? pick_kernel<true>(feat, need, list, nn, need4, f.codes16, hh, f.far_check != 0)
               : pick_kernel<false>(feat, need, list, nn, need4, f.codes16, hh, f.far_check != 0);
}

static int resident_grid(DeviceCopy& c, path_fn fn, uint32_t block, bool count) {
  int& g = c.grid[count ? 1 : 0];
  void*& gf = c.grid_fn[count ? 1 : 0];
  if (g > 0 && gf == (void*)fn) return g;
  gf = (void*)fn;
  int per_cu = 0, cus = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)block, 0);
  if (e != hipSuccess || per_cu < 1) per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.phys) != hipSuccess || cus < 1) cus = 256;
  g = per_cu * cus;
  if (env_int("RTW_VERBOSE", 0))
    fprintf(stderr, "rtw: path kernel %p: block %u, %d resident blocks per CU x %d CUs\n", (void*)fn, block, per_cu, cus);
  return g;
}

// RN(1 / b) for an integer-valued b in [1, 2^24): the float nearest 1 / b, chosen among the neighbours of
// the double quotient by the exact residual |1 - y b| (y b is exact in double: 24 x 24 bits)
static float recip_rn(float b) {
  float y = (float)(1.0 / (double)b), best = y;
  double e = fabs(1.0 - (double)y * (double)b);
  for (float c : {nextafterf(y, 0.0f), nextafterf(y, 2.0f)}) {
    const double ec = fabs(1.0 - (double)c * (double)b);
    if (ec < e) { e = ec; best = c; }
  }
  return best;
}

int check_guard(DeviceCopy& c) {
  volatile uint32_t* e = c.err_host;
  if (e && *e) {
    *e = 0u;
    return fail(RTW_EINVAL, "a path kernel on device %d tripped its BVH traversal guard (corrupt tree?): the frame "
                "it rendered is invalid", c.device);
  }
  return RTW_OK;
}

int enqueue_render(Scene& sc, DeviceCopy& c, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h,
                   uint32_t spp, uint32_t max_depth, uint64_t seed, const TileSet& ts, float* d_out, void* stream_,
                   uint32_t flags, void* ev0_, void* ev1_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  hipEvent_t ev0 = static_cast<hipEvent_t>(ev0_), ev1 = static_cast<hipEvent_t>(ev1_);
  const uint32_t* d_tiles = ts.ids;
  const uint32_t n_slots = ts.n;
  // an earlier render on this device (one the caller did not wait on) tripped the guard: report it now
  if (int e = check_guard(c)) return e;
  if (w > 65536u || h > 65536u)
    return fail(RTW_EINVAL, "image %ux%u: at most 65536 x 65536 (16-bit pixel coordinates in the path key)", w, h);
  if (cam->time0 < sc.flat.time_lo || cam->time1 > sc.flat.time_hi)
    return fail(RTW_EINVAL, "camera shutter [%g, %g) outside the committed motion range [%g, %g]",
                cam->time0, cam->time1, sc.flat.time_lo, sc.flat.time_hi);
  RenderArgs a;
  memset(&a, 0, sizeof a);
  a.scene = c.scene;
  memcpy(a.cam.origin, cam->origin, sizeof a.cam.origin);
  memcpy(a.cam.llc, cam->lower_left_corner, sizeof a.cam.llc);
  memcpy(a.cam.horizontal, cam->horizontal, sizeof a.cam.horizontal);
  memcpy(a.cam.vertical, cam->vertical, sizeof a.cam.vertical);
  memcpy(a.cam.u, cam->u, sizeof a.cam.u);
  memcpy(a.cam.v, cam->v, sizeof a.cam.v);
  a.cam.lens_radius = cam->lens_radius;
  a.cam.time0 = cam->time0;
  a.cam.time1 = cam->time1;
  memcpy(a.bg, bg, sizeof a.bg);
  a.w = w; a.h = h; a.spp = spp; a.max_depth = max_depth;
  a.tiles_x = (w + 7u) / 8u;
  a.spp_magic = spp > 1u ? UINT64_MAX / spp + 1u : 0u;
  a.fw1 = (float)(w - 1u);
  a.fh1 = (float)(h - 1u);
  a.rw1 = recip_rn(a.fw1);
  a.rh1 = recip_rn(a.fh1);
  {
    volatile float t0 = cam->time0, t1 = cam->time1;  // one IEEE f32 subtraction, as on the device
    a.time_span = t1 - t0;
  }
  a.tiles_x_magic = a.tiles_x > 1u ? UINT64_MAX / a.tiles_x + 1u : 0u;
  a.tile_ids = d_tiles;
  a.tile_first = ts.first;
  a.tile_stride = ts.stride;
  a.packed_out = (d_tiles || ts.packed) ? 1u : 0u;
  a.err = c.err_host;
  a.batch = (uint32_t)std::min(65536, std::max(64, env_int("RTW_BATCH", (int)dev::BATCH)));
  a.quota16 = 12;  // see trace_run (measured best of 4..16 on jumpy-balls); tuning knob RTW_QUOTA16 (1..16)
  if (const char* q = tuning_env("RTW_QUOTA16")) a.quota16 = (uint32_t)std::min(16, std::max(1, atoi(q)));
  // test postponed leaves once leaf16/16 of the wave's lanes hold one and cannot descend (trace_run);
  // knob RTW_LEAF16 (1..16)
  a.leaf16 = (uint32_t)std::min(16, std::max(1, env_int("RTW_LEAF16", 3)));  // LDS-node variants: 5, below
  // the host mirror of dev::splitmix64 (seed pre-hash shared by every pixel)
  uint64_t z = seed + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  a.seed_hash = z ^ (z >> 31);
  a.out = d_out;
  a.counters = c.counters;
  a.queue = c.counters + 32;  // the DISP path-id dispensers (path_kernel), DISP_STRIDE words apart
  HIPCHK(hipMemsetAsync(c.counters, 0, COUNTER_WORDS * sizeof(unsigned long long), stream), "hipMemsetAsync");
  if (ev0) HIPCHK(hipEventRecord(ev0, stream), "hipEventRecord");
  if (n_slots && (spp == 0 || max_depth == 0)) {  // lib.rs:83 loops 0 times / :98 returns black
    size_t n = a.packed_out ? (size_t)n_slots * 64 * 3 : (size_t)w * h * 3;
    HIPCHK(hipMemsetAsync(d_out, 0, n * sizeof(float), stream), "hipMemsetAsync(out)");
  } else if (n_slots) {
    const uint64_t per_slot = 64ull * spp;
    const uint32_t slots_per_pass = (uint32_t)std::max<uint64_t>(1, max_pass_paths() / per_slot);
    const uint64_t need = std::min<uint64_t>(n_slots, slots_per_pass) * per_slot;
    if (need > c.sbuf_paths) {  // grow the ordered sample buffer (first render only)
      if (c.sbuf) HIPCHK(hipFree(c.sbuf), "hipFree(sample buffer)");
      c.sbuf = nullptr;
      c.sbuf_paths = 0;
      HIPCHK(hipMalloc((void**)&c.sbuf, need * 3 * sizeof(float)), "hipMalloc(sample buffer)");
      c.sbuf_paths = need;
    }
    a.sbuf = c.sbuf;
    const bool count = flags & RTW_FLAG_COUNT_TRAVERSAL;
    const Variant var = path_kernel_variant(count, sc.flat);
    const path_fn fn = var.fn;
    // the sorted-push walk of the LDS-node kernels parks fewer leaves early: 5/16 measured best on
    // jumpy-balls (+0.5% over 3; profiles/r02/experiments, n5)
    if (var.k16 && sc.flat.features == (sc.flat.features & F_SPHERES))
      a.leaf16 = (uint32_t)std::min(16, std::max(1, env_int("RTW_LEAF16", 5)));
    // the 1024-lane LDS-node kernel and the BVH-less list kernels: 1024 ids per atomic (a shorter end-of-frame
    // tail; jumpy-1080p +1.2%, cornell-800 +0.5% over 2048, profiles/r03/experiments k3 / k4); the mesh
    // kernels keep 2048 (neutral on cow; their short paths made small batches costly in round 2)
    if ((var.k16 && var.block == 1024u) || sc.flat.nodes4.empty())
      a.batch = (uint32_t)std::min(65536, std::max(64, env_int("RTW_BATCH", 1024)));
    // Regenerate paths only once >= regen_min lanes of a wave are idle (or all are): start_path
    // runs at wave level, so batching it raises its SIMD utilisation.  Measured on MI355X
    // (RTW_REGEN_MIN sweep 1..32): 24 is best for open scenes (jumpy-balls +4.3%, cow +1.6%,
    // monument +1.7% over 1); closed boxes (cornell: 6.6 segments per path, few lanes finish per
    // iteration) lose with deep deferral: 8 (cornell list variant at 8 waves/SIMD: 29.3k at 1, 29.4k at 4, 29.8k at 8, 28.1k at 24).
    // With the start ring (round 6, the rect list kernel) a regeneration costs a few LDS reads, not start_path at
    // the idle lanes' occupancy, so waves refill early: REGEN_RING (cornell-800: 8 -> 2, +1.8%).
    const bool boxed = (sc.flat.features & ~F_SMOKE) == 0;
    a.regen_min = (uint32_t)std::min(64, std::max(1, env_int("RTW_REGEN_MIN", var.sring ? REGEN_RING : (boxed ? 8 : 24))));
    const int grid = resident_grid(c, fn, var.block, count);
    // Small frames: fewer ids per atomic, halving until every resident wave can take >= 32 batches.  configs[0]
    // (jumpy-balls 400x225x50: 4.5 M paths for 8,192 resident waves) handed out 4,395 batches of 1,024, so half the
    // waves got none and the kernel ran 5x slower per ray than at 1080p: 5.43k -> 9.30k Mrays/s at 128.  The same
    // for an 8-GPU share (one eighth of the paths): jumpy +5% at 256, cornell +4.4% at 256, cow +22% at 512
    // (profiles/r05/experiments, r05l).  Floors: the mesh / generic kernels' short paths queue on the one atomic
    // word below 512 (cow 256: -16%), the others' below 128.  Full frames keep the defaults (>= 32 batches per
    // wave already); knob RTW_BATCH sets the size outright.
    const uint32_t batch0 = a.batch, batch_floor = batch0 >= 2048u ? 512u : 128u;
    const bool batch_auto = tuning_env("RTW_BATCH") == nullptr;
    const uint64_t waves = (uint64_t)grid * var.block / 64u;
    // the LDS-node variants walk 16-bit codes within their own stack rows (pick_kernel checked
    // stack_need4 against them) and have no HBM spill path
    const uint32_t lds = var.stack;
    a.spill_depth = (!var.k16 && sc.flat.stack_need > lds) ? sc.flat.stack_need - lds : 0;
    a.spill_lanes = (uint32_t)grid * var.block;
    const size_t spill_bytes = (size_t)a.spill_depth * a.spill_lanes * sizeof(int32_t);
    if (spill_bytes > c.spill_bytes) {  // first render of a deep tree only
      if (c.spill) HIPCHK(hipFree(c.spill), "hipFree(stack spill)");
      c.spill = nullptr;
      c.spill_bytes = 0;
      HIPCHK(hipMalloc((void**)&c.spill, spill_bytes), "hipMalloc(stack spill)");
      c.spill_bytes = spill_bytes;
    }
    a.spill = c.spill;
    for (uint32_t base = 0; base < n_slots; base += slots_per_pass) {
      const uint32_t ns = std::min(slots_per_pass, n_slots - base);
      a.slot_base = base;
      a.n_paths = (uint64_t)ns * per_slot;
      a.batch = batch0;
      if (batch_auto)
        while (a.batch / 2u >= batch_floor && a.n_paths < (uint64_t)a.batch * waves * 32u) a.batch /= 2u;
      // (a pass the rule above gave smaller batches spreads its atomics over DISP words in the LDS-node kernels:
      // path_kernel SHARD; r06 share8: an 8-GPU share of jumpy-1080p +5%, configs[0] +11%)
      if (base) HIPCHK(hipMemsetAsync(a.queue, 0, DISP * DISP_STRIDE * sizeof(unsigned long long), stream),
                       "hipMemsetAsync(queue)");
      hipEvent_t* ke = reinterpret_cast<hipEvent_t*>(c.kev[c.kev_head]);
      if (!ke[0]) HIPCHK(hipEventCreate(&ke[0]), "hipEventCreate");
      if (!ke[1]) HIPCHK(hipEventCreate(&ke[1]), "hipEventCreate");
      HIPCHK(hipEventRecord(ke[0], stream), "hipEventRecord");
      hipLaunchKernelGGL(fn, dim3(grid), dim3(var.block), 0, stream, a);
      HIPCHK(hipGetLastError(), "path_kernel launch");
      HIPCHK(hipEventRecord(ke[1], stream), "hipEventRecord");
      c.kev_head = (c.kev_head + 1) % 64u;
      c.kev_count = std::min(c.kev_count + 1u, 64u);
      hipLaunchKernelGGL(dev::reduce_kernel, dim3((ns * 64u + 255u) / 256u), dim3(256), 0, stream, a, ns);
      HIPCHK(hipGetLastError(), "reduce_kernel launch");
    }
  }
  if (ev1) HIPCHK(hipEventRecord(ev1, stream), "hipEventRecord");
  return RTW_OK;
}

int collect_stats(DeviceCopy& c, void* stream_, void* ev0_, void* ev1_, uint64_t paths, rtw_stats* st) {
  hipEvent_t ev0 = static_cast<hipEvent_t>(ev0_), ev1 = static_cast<hipEvent_t>(ev1_);
  HIPCHK(hipStreamSynchronize(static_cast<hipStream_t>(stream_)), "render_kernel");
  unsigned long long cnt[32];
  HIPCHK(hipMemcpy(cnt, c.counters, sizeof cnt, hipMemcpyDeviceToHost), "hipMemcpy(counters)");
  float ms = 0.f;
  if (ev0 && ev1) HIPCHK(hipEventElapsedTime(&ms, ev0, ev1), "hipEventElapsedTime");
  if (int e = check_guard(c)) return e;
  st->rays = cnt[0];
  st->paths = paths;
  st->kernel_ms = ms;
  st->node_visits = cnt[1];
  st->prim_tests = cnt[2];
  for (int k = 0; k < 6; ++k) st->prim_tests_by_type[k] = cnt[3 + k];
  for (int k = 0; k < 6; ++k) st->simd[k] = cnt[9 + k];
  for (int k = 0; k < 4; ++k) st->phase_cycles[k] = cnt[16 + k];
  st->boxes_tested = cnt[15];
  for (int k = 0; k < 4; ++k) st->sub_cycles[k] = cnt[20 + k];
  return RTW_OK;
}

int enqueue_unpack(uint32_t w, uint32_t h, const uint32_t* d_tiles, uint32_t n_tiles, const float* d_packed,
                   float* d_image, void* stream) {
  const uint32_t n = n_tiles * 64u;
  if (!n) return RTW_OK;
  hipLaunchKernelGGL(dev::unpack_tiles_kernel, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     w, h, (w + 7u) / 8u, d_tiles, n_tiles, d_packed, d_image);
  HIPCHK(hipGetLastError(), "unpack_tiles_kernel");
  return RTW_OK;
}

#endif  // RTW_MESH_TU
}  // namespace rtw

#ifndef RTW_MESH_TU
using namespace rtw;

extern "C" {

int rtw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// restores the caller's current device on every return path
struct DeviceGuard {
  int prev = 0;
  DeviceGuard() { hipGetDevice(&prev); }
  ~DeviceGuard() { hipSetDevice(prev); }
};

int rtw_render(rtw_scene* s, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h,
               uint32_t spp, uint32_t max_depth, uint64_t seed, float* out, rtw_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!s || !cam || !bg || !out) return fail(RTW_EINVAL, "NULL argument");
  if (!s->s.committed) return fail(RTW_ESTATE, "scene not committed");
  if (w < 2 || h < 2) return fail(RTW_EINVAL, "image must be at least 2x2 (lib.rs:84-85 divides by w-1, h-1)");
  DeviceCopy* c = find_copy(s->s, -1);
  if (!c) return fail(RTW_ENODEV, "scene has no device copy");
  DeviceGuard g;
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  const size_t bytes = (size_t)w * h * 3 * sizeof(float);
  hipEvent_t e0, e1;
  if (int e = copy_events(*c, e0, e1)) return e;
  if (int e = grow(c->image, bytes)) return e;  // kept for the next frame (no per-call hipMalloc)
  float* d_out = static_cast<float*>(c->image.p);
  const uint32_t n_tiles = ((w + 7u) / 8u) * ((h + 7u) / 8u);
  rtw_stats st;
  memset(&st, 0, sizeof st);
  TileSet all;
  all.n = n_tiles;
  int rc = enqueue_render(s->s, *c, cam, bg, w, h, spp, max_depth, seed, all, d_out, nullptr, 0, e0, e1);
  if (rc == RTW_OK) rc = collect_stats(*c, nullptr, e0, e1, (uint64_t)w * h * spp, &st);
  if (rc == RTW_OK && hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(RTW_ENODEV, "hipMemcpy(image)");
  st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = st;
  return rc;
}

static int render_device(rtw_scene* s, int device, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h,
                         uint32_t spp, uint32_t max_depth, uint64_t seed, TileSet ts, float* d_out, void* stream,
                         uint32_t flags, rtw_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!s || !cam || !bg || !d_out) return fail(RTW_EINVAL, "NULL argument");
  if (!s->s.committed) return fail(RTW_ESTATE, "scene not committed");
  if (w < 2 || h < 2) return fail(RTW_EINVAL, "image must be at least 2x2");
  DeviceCopy* c = find_copy(s->s, device);
  if (!c) return fail(RTW_ENODEV, "scene was not committed to device %d", device);
  DeviceGuard g;
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (stats)
    if (int e = copy_events(*c, e0, e1)) return e;
  int rc = enqueue_render(s->s, *c, cam, bg, w, h, spp, max_depth, seed, ts, d_out, stream, flags, e0, e1);
  if (rc == RTW_OK && stats) {
    rtw_stats st;
    memset(&st, 0, sizeof st);
    rc = collect_stats(*c, stream, e0, e1, (uint64_t)ts.n * 64u * spp, &st);
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *stats = st;
  }
  return rc;
}

int rtw_render_device(rtw_scene* s, int device, const rtw_camera* cam, const float bg[3], uint32_t w,
                      uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, const uint32_t* d_tiles,
                      uint32_t n_tiles, float* d_out, void* stream, uint32_t flags, rtw_stats* stats) {
  TileSet ts;
  ts.ids = d_tiles;
  ts.n = d_tiles ? n_tiles : ((w + 7u) / 8u) * ((h + 7u) / 8u);
  return render_device(s, device, cam, bg, w, h, spp, max_depth, seed, ts, d_out, stream, flags, stats);
}

int rtw_render_device_strided(rtw_scene* s, int device, const rtw_camera* cam, const float bg[3], uint32_t w,
                              uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, uint32_t first_tile,
                              uint32_t tile_stride, uint32_t n_tiles, float* d_out, void* stream, uint32_t flags,
                              rtw_stats* stats) {
  const uint64_t nt = (uint64_t)((w + 7u) / 8u) * ((h + 7u) / 8u);
  if (tile_stride == 0 || (n_tiles && first_tile + (uint64_t)(n_tiles - 1) * tile_stride >= nt))
    return fail(RTW_EINVAL, "tiles %u + k * %u (k < %u) leave the frame's %llu tiles", first_tile, tile_stride, n_tiles,
                (unsigned long long)nt);
  TileSet ts;
  ts.first = first_tile;
  ts.stride = tile_stride;
  ts.n = n_tiles;
  ts.packed = true;
  return render_device(s, device, cam, bg, w, h, spp, max_depth, seed, ts, d_out, stream, flags, stats);
}

int rtw_render_status(rtw_scene* s, int device) {
  if (!s) return fail(RTW_EINVAL, "NULL argument");
  DeviceCopy* c = find_copy(s->s, device);
  if (!c) return fail(RTW_ENODEV, "scene was not committed to device %d", device);
  DeviceGuard g;
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  HIPCHK(hipDeviceSynchronize(), "render (hipDeviceSynchronize)");
  return check_guard(*c);
}

// Test hook: overwrite the first two node4s of the device copy with a cycle (node 0 -> node 1 -> node 1
// ..., every box infinite, in both the 32-bit child words and the 16-bit codes), so that every ray's
// walk trips the traversal guard.  The host tables are untouched; renders of this copy are invalid.
int rtw_diag_corrupt_bvh(rtw_scene* s, int device) {
  if (!s) return fail(RTW_EINVAL, "NULL argument");
  if (!s->s.committed) return fail(RTW_ESTATE, "scene not committed");
  DeviceCopy* c = find_copy(s->s, device);
  if (!c) return fail(RTW_ENODEV, "scene was not committed to device %d", device);
  if (c->scene.n_nodes < 2) return fail(RTW_EINVAL, "the scene's BVH has %u node4s (needs 2)", c->scene.n_nodes);
  DevNode4 nd[2];
  memset(nd, 0, sizeof nd);
  for (DevNode4& n : nd) {
    for (int k = 0; k < 4; ++k) {
      const float lo = k ? INFINITY : -1e30f, hi = k ? -INFINITY : 1e30f;  // slots 1-3 empty
      n.lo_x[k] = n.lo_y[k] = n.lo_z[k] = lo;
      n.hi_x[k] = n.hi_y[k] = n.hi_z[k] = hi;
    }
    n.child[0] = 1;
    n.code[0] = 1u;
  }
  DeviceGuard g;
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  HIPCHK(hipMemcpy(const_cast<DevNode4*>(c->scene.nodes), nd, sizeof nd, hipMemcpyHostToDevice), "hipMemcpy(nodes)");
  if (c->scene.hnodes) {  // the half-precision table too: slot 0 = [-65504, +inf) on every axis, slots 1-3 empty
    DevNode4h hn[2];
    memset(hn, 0, sizeof hn);
    for (DevNode4h& n : hn) {
      for (uint16_t* ax : {&n.x[0][0], &n.y[0][0], &n.z[0][0]})
        for (int k = 0; k < 4; ++k) {
          const uint16_t lo = k ? 0x7C00 : 0x0000, hi = k ? 0xFC00 : 0x7C00;
          ax[k] = lo; ax[4 + k] = hi; ax[8 + k] = hi; ax[12 + k] = lo;
        }
      n.origin[0] = n.origin[1] = n.origin[2] = 0xFBFF;  // -65504
      n.code[0] = 1;
    }
    HIPCHK(hipMemcpy(const_cast<DevNode4h*>(c->scene.hnodes), hn, sizeof hn, hipMemcpyHostToDevice), "hipMemcpy(hnodes)");
  }
  return RTW_OK;
}

int rtw_render_stream(rtw_scene* s, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h, uint32_t spp,
                      uint32_t max_depth, uint64_t seed, uint32_t band_rows, rtw_pixel_sink sink, void* user,
                      rtw_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!s || !cam || !bg || !sink) return fail(RTW_EINVAL, "NULL argument");
  if (!s->s.committed) return fail(RTW_ESTATE, "scene not committed");
  if (w < 2 || h < 2) return fail(RTW_EINVAL, "image must be at least 2x2 (lib.rs:84-85 divides by w-1, h-1)");
  DeviceCopy* c = find_copy(s->s, -1);
  if (!c) return fail(RTW_ENODEV, "scene has no device copy");
  const uint32_t tiles_x = (w + 7u) / 8u, tiles_y = (h + 7u) / 8u;
  const uint32_t band_ty = std::max(1u, ((band_rows ? band_rows : 64u) + 7u) / 8u);  // tile rows per band
  DeviceGuard g;
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  const size_t band_tiles = (size_t)band_ty * tiles_x;
  if (int e = grow(c->packed, band_tiles * 64 * 3 * sizeof(float))) return e;
  float* d_packed = static_cast<float*>(c->packed.p);
  hipEvent_t e0, e1;
  if (int e = copy_events(*c, e0, e1)) return e;
  int rc = RTW_OK;
  std::vector<float> packed(band_tiles * 64 * 3);
  std::vector<rtw_pixel> px;
  rtw_stats tot;
  memset(&tot, 0, sizeof tot);
  for (uint32_t ty0 = 0; rc == RTW_OK && ty0 < tiles_y; ty0 += band_ty) {
    const uint32_t nty = std::min(band_ty, tiles_y - ty0), nt = nty * tiles_x;
    TileSet band;  // tile row ty = output rows [8 ty, 8 ty + 8): the band's tiles are consecutive
    band.first = ty0 * tiles_x;
    band.n = nt;
    band.packed = true;
    rc = enqueue_render(s->s, *c, cam, bg, w, h, spp, max_depth, seed, band, d_packed, nullptr, 0, e0, e1);
    rtw_stats st;
    memset(&st, 0, sizeof st);
    if (rc == RTW_OK) rc = collect_stats(*c, nullptr, e0, e1, 0, &st);
    if (rc == RTW_OK && hipMemcpy(packed.data(), d_packed, (size_t)nt * 64 * 3 * sizeof(float),
                                  hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(RTW_ENODEV, "hipMemcpy(band)");
    if (rc != RTW_OK) break;
    tot.rays += st.rays;
    tot.kernel_ms += st.kernel_ms;
    // emit rows of this band in reference order: output row r <-> j = h-1-r, columns 0..w-1
    const uint32_t r0 = ty0 * 8u, r1 = std::min(h, (ty0 + nty) * 8u);
    px.clear();
    for (uint32_t r = r0; r < r1; ++r)
      for (uint32_t i = 0; i < w; ++i) {
        const size_t slot = (size_t)(r / 8u - ty0) * tiles_x + i / 8u, lane = (r % 8u) * 8u + (i % 8u);
        const float* v = &packed[(slot * 64 + lane) * 3];
        px.push_back(rtw_pixel{h - 1u - r, i, {v[0], v[1], v[2]}});
      }
    if (int e = sink(px.data(), (uint32_t)px.size(), user)) rc = e;
  }
  tot.paths = (uint64_t)w * h * spp;
  tot.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = tot;
  return rc;
}

int rtw_path_kernel_times(rtw_scene* s, int device, float* ms, uint32_t max_n) {
  if (!s || (!ms && max_n)) return fail(RTW_EINVAL, "NULL argument");
  DeviceCopy* c = find_copy(s->s, device);
  if (!c) return fail(RTW_ENODEV, "scene was not committed to device %d", device);
  int prev = 0;
  hipGetDevice(&prev);
  HIPCHK(hipSetDevice(c->phys), "hipSetDevice");
  const uint32_t n = std::min(c->kev_count, max_n);
  int rc = (int)n;
  for (uint32_t q = 0; q < n; ++q) {  // the n most recent, oldest first
    hipEvent_t* e = reinterpret_cast<hipEvent_t*>(c->kev[(c->kev_head + 64u - n + q) % 64u]);
    hipError_t err = hipEventSynchronize(e[1]);
    if (err == hipSuccess) err = hipEventElapsedTime(&ms[q], e[0], e[1]);
    if (err != hipSuccess) {
      rc = hip_fail(err, "path-kernel events");
      break;
    }
  }
  c->kev_count = 0;
  if (rc >= 0 && n)  // the launches waited for: report a tripped traversal guard (its frame is invalid)
    if (int e = check_guard(*c)) rc = e;
  hipSetDevice(prev);
  return rc;
}

int rtw_diag_recip(uint32_t n, const float* b, float* out) {
  if (n && (!b || !out)) return fail(RTW_EINVAL, "NULL argument");
  for (uint32_t k = 0; k < n; ++k) out[k] = recip_rn(b[k]);
  return RTW_OK;
}

int rtw_diag_libm(int fn, uint32_t n, const float* a, const float* b, float* out) {
  if (fn < 0 || fn > 5 || (n && (!a || !out || ((fn == 3 || fn == 4) && !b)))) return fail(RTW_EINVAL, "bad arguments");
  if (!n) return RTW_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RTW_ENODEV, "no HIP device visible");
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  const size_t bytes = (size_t)n * sizeof(float);
  int rc = RTW_OK;
  if (hipMalloc((void**)&da, bytes) != hipSuccess || hipMalloc((void**)&dout, bytes) != hipSuccess ||
      ((fn == 3 || fn == 4) && hipMalloc((void**)&db, bytes) != hipSuccess)) {
    rc = fail(RTW_ENOMEM, "hipMalloc(diag)");
  } else if (hipMemcpy(da, a, bytes, hipMemcpyHostToDevice) != hipSuccess ||
             (db && hipMemcpy(db, b, bytes, hipMemcpyHostToDevice) != hipSuccess)) {
    rc = fail(RTW_ENODEV, "hipMemcpy(diag)");
  } else {
    hipLaunchKernelGGL(dev::libm_kernel, dim3((n + 255) / 256), dim3(256), 0, nullptr, fn, n, da, db, dout);
    if (hipGetLastError() != hipSuccess || hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(RTW_ENODEV, "libm_kernel");
  }
  if (da) hipFree(da);
  if (db) hipFree(db);
  if (dout) hipFree(dout);
  return rc;
}

int rtw_diag_sweep(int fn, uint32_t lo, uint32_t hi, uint64_t* counts, uint32_t* bad, uint32_t cap) {
  if (fn != 0 || lo > hi || !counts || (cap && !bad)) return fail(RTW_EINVAL, "bad arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RTW_ENODEV, "no HIP device visible");
  unsigned long long* dn = nullptr;
  uint32_t* dbad = nullptr;
  int rc = RTW_OK;
  if (hipMalloc((void**)&dn, 3 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc((void**)&dbad, (cap ? cap : 1) * sizeof(uint32_t)) != hipSuccess) {
    rc = fail(RTW_ENOMEM, "hipMalloc(sweep)");
  } else if (hipMemset(dn, 0, 3 * sizeof(unsigned long long)) != hipSuccess) {
    rc = fail(RTW_ENODEV, "hipMemset(sweep)");
  } else {
    hipLaunchKernelGGL(dev::sweep_kernel, dim3(16384), dim3(256), 0, nullptr, fn, lo, hi, dn, dbad, cap);
    unsigned long long h[3];
    if (hipGetLastError() != hipSuccess || hipMemcpy(h, dn, sizeof h, hipMemcpyDeviceToHost) != hipSuccess ||
        (cap && hipMemcpy(bad, dbad, cap * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)) {
      rc = fail(RTW_ENODEV, "sweep_kernel");
    } else {
      counts[0] = h[0];
      counts[1] = h[1];
    }
  }
  if (dn) hipFree(dn);
  if (dbad) hipFree(dbad);
  return rc;
}

int rtw_unpack_tiles_device(int device, uint32_t w, uint32_t h, const uint32_t* d_tiles, uint32_t n_tiles,
                            const float* d_packed, float* d_image, void* stream) {
  if (!d_tiles || !d_packed || !d_image) return fail(RTW_EINVAL, "NULL argument");
  DeviceGuard g;
  if (device >= 0) HIPCHK(hipSetDevice(device), "hipSetDevice");
  return enqueue_unpack(w, h, d_tiles, n_tiles, d_packed, d_image, stream);
}

}  // extern "C"
#endif  // RTW_MESH_TU
