/*
 * rtw_oracle.c — plain-C restatement of raytracer_weekend_lib's render hot path
 * (Raytracer::render → sample_pixel → sample_ray → Hittable::hit / Material::scatter).
 *
 * TEST INFRASTRUCTURE ONLY — the parity checker and the timed CPU baseline.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference root, raytracer_weekend_lib/src/ unless stated).  Compile with
 * -ffp-contract=off: Rust never contracts a*b+c into an FMA, so neither may we.
 *
 * Parity status: "parity unpinned" at image level — the reference cannot be run
 * here (no Rust toolchain) and draws from an unseeded ThreadRng (lib.rs:34-35,64).
 * Function-level parity is pinned by spherical.rs:66-68 (in-code KAT table), the
 * analytic KATs in tests/test_oracle_kat.py, and the independent numpy restatement's
 * golden vectors (tests/golden/).  See DESIGN.md §Parity.
 *
 * RNG: the reference's rand 0.9.0-alpha.1 (Cargo.lock:2662-2670, not vendored) is
 * restated only for its float conversions (Standard f32/f64, UniformFloat
 * sample_single).  The bit source of a path is this build's xoroshiro64* (Blackman &
 * Vigna 2018) seeded with splitmix64(splitmix64(seed) ^ (j << 48 | i << 32 | sample)) —
 * the reference's ThreadRng is OS-seeded, so no bit stream of it can be matched anyway.
 * Scene placement and the reference-BvhNode axis draws use a PCG32 (XSH-RR 64/32) stream.
 */
#include "rtw_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ errors */
static __thread char g_err[256];
static void set_err(const char* m) { snprintf(g_err, sizeof g_err, "%s", m); }
const char* oracle_last_error(void) { return g_err; }

/* ------------------------------------------------------------------ vec3.rs */
typedef struct { float x, y, z; } vec3;
static inline vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static inline float vget(vec3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
/* vec3.rs:205-215 Add, :194-203 Sub, :247-253 Mul<U>, :266-276 Mul, :288-292 Div<T>, :323-329 Neg */
static inline vec3 vadd(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 vsub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 vmul(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 vscale(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline vec3 vdivs(vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline vec3 vneg(vec3 a) { return v3(-a.x, -a.y, -a.z); }
/* vec3.rs:41-44 length_squared, :46-48 dot, :50-56 cross (left-to-right sums) */
static inline float vlen2(vec3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float vdot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline vec3 vcross(vec3 a, vec3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* vec3.rs:81-87 length / unit_vector: component-wise division by the length */
static inline vec3 vunit(vec3 a) { return vdivs(a, sqrtf(vlen2(a))); }
/* vec3.rs:133-138 */
static inline int vnear_zero(vec3 a) {
  const float S = 1e-8f;
  return fabsf(a.x) < S && fabsf(a.y) < S && fabsf(a.z) < S;
}
/* vec3.rs:140-142: self - (2*dot)*n */
static inline vec3 vreflect(vec3 v, vec3 n) { return vsub(v, vscale(n, 2.0f * vdot(v, n))); }
/* vec3.rs:144-151 */
static inline vec3 vrefract(vec3 uv, vec3 n, float eta) {
  float cos_theta = fminf(vdot(vneg(uv), n), 1.0f);
  vec3 r_perp = vscale(vadd(uv, vscale(n, cos_theta)), eta);
  float k = -sqrtf(fabsf(1.0f - vlen2(r_perp)));
  vec3 r_par = vscale(n, k);
  return vadd(r_perp, r_par);
}

/* ------------------------------------------------------------------ RNG */
uint64_t oracle_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
/* PCG32 (XSH-RR 64/32): the scene-placement / reference-BVH stream (host side only) */
typedef struct { uint64_t s; } pcg32;
static inline uint32_t pcg_next(pcg32* r) {
  uint64_t old = r->s;
  r->s = old * 6364136223846793005ull + 1442695040888963407ull;
  uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
  uint32_t rot = (uint32_t)(old >> 59);
  return (xs >> rot) | (xs << ((32u - rot) & 31u));
}
uint32_t oracle_pcg32_stream(uint64_t state, uint32_t n, uint32_t* out, uint64_t* state_out) {
  pcg32 r = {state};
  for (uint32_t k = 0; k < n; ++k) out[k] = pcg_next(&r);
  if (state_out) *state_out = r.s;
  return n;
}
/* xoroshiro64* (Blackman & Vigna 2018): the per-path stream.  State = s0 | s1 << 32, never 0.
 * One 32-bit multiply per draw (the GPU's PCG32 needed a 64-bit one); the multiply's high bits,
 * which every float conversion below uses, pass BigCrush. */
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
static inline uint32_t xoro_next(uint64_t* st) {
  uint32_t s0 = (uint32_t)*st, s1 = (uint32_t)(*st >> 32);
  const uint32_t result = s0 * 0x9E3779BBu;
  s1 ^= s0;
  s0 = rotl32(s0, 26) ^ s1 ^ (s1 << 9);
  s1 = rotl32(s1, 13);
  *st = ((uint64_t)s1 << 32) | s0;
  return result;
}
/* seeds a stream from a 64-bit hash (the all-zero state is xoroshiro's fixed point) */
static inline uint64_t xoro_seed(uint64_t h) { return h ? h : 0x9E3779B97F4A7C15ull; }
uint32_t oracle_rng_stream(uint64_t state, uint32_t n, uint32_t* out, uint64_t* state_out) {
  uint64_t st = state;
  for (uint32_t k = 0; k < n; ++k) out[k] = xoro_next(&st);
  if (state_out) *state_out = st;
  return n;
}
/* Per-path stream state: (seed, pixel row j, column i, sample s); j, i < 2^16. */
uint64_t oracle_path_state(uint64_t seed, uint32_t j, uint32_t i, uint32_t s) {
  const uint64_t key = ((uint64_t)j << 48) | ((uint64_t)i << 32) | (uint64_t)s;
  return xoro_seed(oracle_splitmix64(oracle_splitmix64(seed) ^ key));
}
static inline float bits_to_f(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static inline uint32_t f_to_bits(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }
/* rand Standard for f32: (u >> 8) * 2^-24 */
float oracle_u32_to_f32(uint32_t u) { return (float)(u >> 8) * (1.0f / 16777216.0f); }
/* rand Standard for f64 from next_u64 = lo | hi << 32: (u >> 11) * 2^-53 */
double oracle_u64_to_f64(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }
/* rand UniformFloat<f32>::sample_single, one attempt: value1_2 from 23 mantissa bits,
 * res = value0_1 * scale + low (multiply, then add: no FMA) */
static inline float range_attempt(uint32_t u, float scale, float lo) {
  float v12 = bits_to_f((u >> 9) | 0x3F800000u);
  float v01 = v12 - 1.0f;
  return v01 * scale + lo;
}
float oracle_u32_to_range(uint32_t u, float lo, float hi) { return range_attempt(u, hi - lo, lo); }

/* A draw source: either a live path stream (xoroshiro64* state) or an explicit array (unit tests). */
typedef struct {
  struct { uint64_t s; } rng;
  const uint32_t* arr;
  uint32_t n, used;
} draws;
static inline uint32_t next_u32(draws* d) {
  if (d->arr) { uint32_t v = d->used < d->n ? d->arr[d->used] : 0x80000000u; d->used++; return v; }  /* exhausted -> 0.0 in [-1,1) */
  d->used++;
  return xoro_next(&d->rng.s);
}
static inline float gen_f32(draws* d) { return oracle_u32_to_f32(next_u32(d)); }
static inline float gen_range(draws* d, float lo, float hi) {
  float scale = hi - lo;
  for (;;) {
    float res = range_attempt(next_u32(d), scale, lo);
    if (res < hi) return res;
    scale = bits_to_f(f_to_bits(scale) - 1u); /* rand: shrink scale by one ulp and retry */
  }
}
/* vec3.rs:97-108 random_min_max(-1..1) + rejection, draw order x, y, z */
static inline vec3 rand_in_unit_sphere(draws* d) {
  for (;;) {
    float x = gen_range(d, -1.0f, 1.0f);
    float y = gen_range(d, -1.0f, 1.0f);
    float z = gen_range(d, -1.0f, 1.0f);
    vec3 p = v3(x, y, z);
    if (vlen2(p) < 1.0f) return p;
  }
}
/* vec3.rs:110-112 */
static inline vec3 rand_unit_vector(draws* d) { return vunit(rand_in_unit_sphere(d)); }
/* vec3.rs:124-131 */
static inline vec3 rand_in_unit_disk(draws* d) {
  for (;;) {
    float x = gen_range(d, -1.0f, 1.0f);
    float y = gen_range(d, -1.0f, 1.0f);
    vec3 p = v3(x, y, 0.0f);
    if (vlen2(p) < 1.0f) return p;
  }
}


/* ------------------------------------------------------------------ libm (f32 transcendentals)
 * Rust's f32::sin / acos / atan2 / log10 call the platform libm.  glibc 2.35's float versions
 * (this image) are faithfully but not correctly rounded (<= 1 ulp; e.g. log10f differs from the
 * correctly rounded value for 23% of the rand Standard<f32> inputs), and other platforms' libms
 * differ again, so the reference's exact bits are platform-defined.  This build defines them as
 * the CORRECTLY ROUNDED values: each function is evaluated in double precision with a
 * polynomial of error < 2^-60 and rounded once to f32.  Only IEEE double +,-,*,/,sqrt and floor
 * are used (no FMA contraction), so the GPU kernel (rtw_kernel.hip, same algorithm) produces
 * the same bits.  tests/test_libm.py pins these against (float)glibc-double exhaustively
 * over the ranges the render path reaches; tests/test_gpu_parity.py pins GPU == oracle. */
static inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
/* ln(m), m in [sqrt(1/2), sqrt(2)]: 2 atanh(s), s = (m-1)/(m+1), |s| <= 0.1716 */
static double ol_ln_core(double m) {
  double s = (m - 1.0) / (m + 1.0), z = s * s;
  double p = 1.0 / 23.0;
  p = p * z + 1.0 / 21.0; p = p * z + 1.0 / 19.0; p = p * z + 1.0 / 17.0; p = p * z + 1.0 / 15.0;
  p = p * z + 1.0 / 13.0; p = p * z + 1.0 / 11.0; p = p * z + 1.0 / 9.0; p = p * z + 1.0 / 7.0;
  p = p * z + 1.0 / 5.0; p = p * z + 1.0 / 3.0; p = p * z + 1.0;
  return 2.0 * s * p;
}
float oracle_log10f(float x) {
  if (x != x) return x;
  if (x == 0.0f) return -INFINITY;
  if (x < 0.0f) return NAN;
  if (isinf(x)) return x;
  uint64_t u = d2u((double)x);
  int e = (int)((u >> 52) & 0x7ff) - 1023; /* x normal or subnormal as f32 is normal as f64 */
  double m = u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
  if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
  const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  const double INV_LN10 = 0.43429448190325182765;
  double lnx = ((double)e * LN2_HI + ol_ln_core(m)) + (double)e * LN2_LO;
  return (float)(lnx * INV_LN10);
}
static double ol_sin_core(double r) { /* |r| <= pi/4 */
  double z = r * r, p = -1.0 / 1307674368000.0;
  p = p * z + 1.0 / 6227020800.0; p = p * z - 1.0 / 39916800.0; p = p * z + 1.0 / 362880.0;
  p = p * z - 1.0 / 5040.0; p = p * z + 1.0 / 120.0; p = p * z - 1.0 / 6.0;
  return r + r * z * p;
}
static double ol_cos_core(double r) {
  double z = r * r, p = 1.0 / 20922789888000.0;
  p = p * z - 1.0 / 87178291200.0; p = p * z + 1.0 / 479001600.0; p = p * z - 1.0 / 3628800.0;
  p = p * z + 1.0 / 40320.0; p = p * z - 1.0 / 720.0; p = p * z + 1.0 / 24.0; p = p * z - 0.5;
  return 1.0 + z * p;
}
float oracle_sinf(float x) {
  if (x != x || x == 0.0f) return x; /* keeps the sign of zero */
  if (isinf(x)) return NAN;
  double d = x;
  /* Cody-Waite reduction by pi/2 (three 33-bit parts: exact products for |k| < 2^20) */
  const double TWO_OVER_PI = 6.36619772367581382433e-01;
  const double P1 = 1.57079632673412561417e+00, P2 = 6.07710050650619224932e-11,
               P3 = 2.02226624879595063154e-21;
  double k = floor(d * TWO_OVER_PI + 0.5);
  double r = ((d - k * P1) - k * P2) - k * P3;
  double q = k - 4.0 * floor(k * 0.25);
  double v = q == 0.0 ? ol_sin_core(r) : (q == 1.0 ? ol_cos_core(r) : (q == 2.0 ? -ol_sin_core(r) : -ol_cos_core(r)));
  return (float)v;
}
static double ol_atan_core(double t) { /* |t| <= tan(pi/16) */
  double z = t * t, p = -1.0 / 29.0;
  p = p * z + 1.0 / 27.0; p = p * z - 1.0 / 25.0; p = p * z + 1.0 / 23.0; p = p * z - 1.0 / 21.0;
  p = p * z + 1.0 / 19.0; p = p * z - 1.0 / 17.0; p = p * z + 1.0 / 15.0; p = p * z - 1.0 / 13.0;
  p = p * z + 1.0 / 11.0; p = p * z - 1.0 / 9.0; p = p * z + 1.0 / 7.0; p = p * z - 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  return t - t * z * p;
}
static double ol_atan01(double a) { /* 0 <= a <= 1: atan(a) = j pi/8 + atan((a - c_j) / (1 + a c_j)) */
  const double T1 = 0.19891236737965800691, T3 = 0.66817863791929891999; /* tan(pi/16), tan(3pi/16) */
  const double C1 = 0.41421356237309504880;                               /* tan(pi/8) */
  const double PI_8 = 0.39269908169872415481, PI_4 = 0.78539816339744830962;
  if (a <= T1) return ol_atan_core(a);
  if (a <= T3) return PI_8 + ol_atan_core((a - C1) / (1.0 + a * C1));
  return PI_4 + ol_atan_core((a - 1.0) / (1.0 + a));
}
static double ol_atan2_pos(double y, double x) { /* y > 0 finite, x finite non-zero */
  const double PI = 3.14159265358979323846, PI_2 = 1.57079632679489661923;
  double ax = fabs(x), r;
  r = y <= ax ? ol_atan01(y / ax) : PI_2 - ol_atan01(ax / y);
  return x < 0.0 ? PI - r : r;
}
float oracle_atan2f(float y, float x) { /* C99 Annex F special cases, as glibc */
  const double PI = 3.14159265358979323846, PI_2 = 1.57079632679489661923, PI_4 = 0.78539816339744830962;
  if (x != x || y != y) return x + y;
  const int sx = signbit(x) != 0, sy = signbit(y) != 0;
  double r;
  if (y == 0.0f) r = sx ? PI : 0.0;
  else if (isinf(x)) r = isinf(y) ? (sx ? 3.0 * PI_4 : PI_4) : (sx ? PI : 0.0);
  else if (x == 0.0f || isinf(y)) r = PI_2;
  else r = ol_atan2_pos(fabs((double)y), (double)x);
  return (float)(sy ? -r : r);
}
float oracle_acosf(float x) { /* acos x = atan2(sqrt((1-x)(1+x)), x); (1-x)(1+x) is exact in f64 */
  if (x != x) return x;
  if (!(fabsf(x) <= 1.0f)) return NAN;
  double d = x, s = sqrt((1.0 - d) * (1.0 + d));
  if (s == 0.0) return d > 0.0 ? 0.0f : (float)3.14159265358979323846;
  return (float)ol_atan2_pos(s, d);
}
int oracle_libm(int fn, uint32_t n, const float* a, const float* b, float* out) {
  for (uint32_t k = 0; k < n; ++k) {
    switch (fn) {
      case 0: out[k] = oracle_log10f(a[k]); break;
      case 1: out[k] = oracle_sinf(a[k]); break;
      case 2: out[k] = oracle_acosf(a[k]); break;
      case 3: out[k] = oracle_atan2f(a[k], b[k]); break;
      default: return -22;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------ ray.rs */
typedef struct { vec3 o, d; float time; } ray;
static inline vec3 ray_at(const ray* r, float t) { return vadd(r->o, vscale(r->d, t)); } /* ray.rs:25-27 */

/* ------------------------------------------------------------------ camera.rs */
static inline float to_radians(float deg) { return deg * (3.14159265358979323846f / 180.0f); }
void oracle_camera_new(const float lf[3], const float la[3], const float up[3], float vfov,
                       float aspect, float aperture, float focus, float t0, float t1,
                       oracle_camera* c) {
  /* camera.rs:25-64 */
  float theta = to_radians(vfov);
  float h = tanf(theta / 2.0f);
  float vh = 2.0f * h;
  float vw = aspect * vh;
  vec3 from = v3(lf[0], lf[1], lf[2]), at = v3(la[0], la[1], la[2]), vup = v3(up[0], up[1], up[2]);
  vec3 w = vunit(vsub(from, at));
  vec3 u = vunit(vcross(vup, w));
  vec3 v = vcross(w, u);
  vec3 hor = vscale(u, focus * vw);
  vec3 ver = vscale(v, focus * vh);
  vec3 llc = vsub(vsub(vsub(from, vdivs(hor, 2.0f)), vdivs(ver, 2.0f)), vscale(w, focus));
  float* dst[7] = {c->origin, c->lower_left_corner, c->horizontal, c->vertical, c->u, c->v, c->w};
  vec3 src[7] = {from, llc, hor, ver, u, v, w};
  for (int k = 0; k < 7; ++k) { dst[k][0] = src[k].x; dst[k][1] = src[k].y; dst[k][2] = src[k].z; }
  c->lens_radius = aperture / 2.0f;
  c->time0 = t0;
  c->time1 = t1;
}
static inline vec3 cv(const float* a) { return v3(a[0], a[1], a[2]); }
/* camera.rs:66-74 — the disk is drawn even for aperture 0 */
static ray camera_get_ray(const oracle_camera* c, float s, float t, draws* d) {
  vec3 rd = vscale(rand_in_unit_disk(d), c->lens_radius);
  vec3 offset = vadd(vscale(cv(c->u), rd.x), vscale(cv(c->v), rd.y));
  ray r;
  r.o = vadd(cv(c->origin), offset);
  r.d = vsub(vsub(vadd(vadd(cv(c->lower_left_corner), vscale(cv(c->horizontal), s)),
                       vscale(cv(c->vertical), t)),
                  cv(c->origin)),
             offset);
  r.time = gen_range(d, c->time0, c->time1);
  return r;
}

/* ------------------------------------------------------------------ scene model */
enum { T_SOLID, T_CHECKER, T_IMAGE, T_UVDEBUG, T_NOISE };
/* perlin.rs:8-12: 256 gradients, three permutations */
typedef struct { vec3 g[256]; int perm[3][256]; } operlin;
typedef struct { int kind; float c[3]; int odd, even; float freq; int w, h; const uint8_t* img; operlin* perlin; } otex;
enum { M_LAMBERT, M_METAL, M_DIELECTRIC, M_LIGHT, M_ISOTROPIC };
typedef struct { int kind; int tex; float albedo[3]; float fuzz; float ir; } omat;

enum { K_LIST, K_BVH, K_TRANSLATE, K_ROTY, K_SPHERE, K_MSPHERE, K_RECT, K_CUBOID, K_TRI, K_BVHNODE, K_MEDIUM };
typedef struct { vec3 mn, mx; int ok; } aabb;
typedef struct onode {
  int kind, mat, axis;
  uint32_t key;        /* DFS leaf index (world leaves; a ConstantMedium is one leaf) */
  int n, cap;
  struct onode** ch;
  float f[16];         /* primitive / wrapper parameters */
  vec3 tv[3], tn[3];   /* triangle vertices, normals (after defaults) */
  float tuv[3][2];     /* triangle uvs (after defaults) */
  float sin_t, cos_t;  /* YRotation */
  aabb rot_box;        /* YRotation bounding box (transformations.rs:65-67) */
  struct onode *left, *right; /* K_BVHNODE (reference build) */
  aabb box;
  struct onode* ref_tree;     /* K_BVH: reference BvhNode tree (bvh_mode 1) */
} onode;

struct oracle_scene {
  otex* tex; int ntex;
  omat* mat; int nmat;
  onode* root;
  int nleaf;
};

typedef struct { vec3 p, n; int mat; float t, u, v; int front; } hitrec;

/* hittable/mod.rs:32-48 */
static inline void set_face_normal(hitrec* h, const ray* r, vec3 outward) {
  h->front = vdot(r->d, outward) < 0.0f;
  h->n = h->front ? outward : vneg(outward);
}

/* ------------------------------------------------------------------ aabb.rs */
static int aabb_hit(const aabb* b, const ray* r, float tmin, float tmax) {
  /* aabb.rs:23-48; Rust f32::max/min return the non-NaN operand = fmaxf/fminf */
  for (int a = 0; a < 3; ++a) {
    float inv = 1.0f / vget(r->d, a);
    float t0 = (vget(b->mn, a) - vget(r->o, a)) * inv;
    float t1 = (vget(b->mx, a) - vget(r->o, a)) * inv;
    if (inv < 0.0f) { float tt = t0; t0 = t1; t1 = tt; }
    tmin = fmaxf(t0, tmin);
    tmax = fminf(t1, tmax);
    if (tmax <= tmin) return 0;
  }
  return 1;
}
static aabb surrounding(aabb a, aabb b) { /* aabb.rs:74-88 */
  aabb r;
  r.mn = v3(fminf(a.mn.x, b.mn.x), fminf(a.mn.y, b.mn.y), fminf(a.mn.z, b.mn.z));
  r.mx = v3(fmaxf(a.mx.x, b.mx.x), fmaxf(a.mx.y, b.mx.y), fmaxf(a.mx.z, b.mx.z));
  r.ok = 1;
  return r;
}

/* ------------------------------------------------------------------ primitives */
void oracle_sphere_uv(const float p[3], float uv[2]) {
  /* spherical.rs:62-77 */
  const float PI = 3.14159265358979323846f;
  float theta = oracle_acosf(-p[1]);         /* f32::acos / atan2: correctly rounded, see libm */
  float phi = oracle_atan2f(-p[2], p[0]) + PI;
  uv[0] = phi / (2.0f * PI);
  uv[1] = theta / PI;
}
/* spherical.rs:18-60 */
static int hit_sphere(const ray* r, float tmin, float tmax, vec3 center, float radius, int mat,
                      hitrec* h) {
  vec3 oc = vsub(r->o, center);
  float a = vlen2(r->d);
  float half_b = vdot(oc, r->d);
  float c = vlen2(oc) - radius * radius;
  float disc = half_b * half_b - a * c;
  if (disc < 0.0f) return 0;
  float sqrtd = sqrtf(disc);
  float root = (-half_b - sqrtd) / a;
  if (root < tmin || tmax < root) {
    root = (-half_b + sqrtd) / a;
    if (root < tmin || tmax < root) return 0;
  }
  h->t = root;
  h->p = ray_at(r, root);
  vec3 outward = vdivs(vsub(h->p, center), radius);
  float pp[3] = {outward.x, outward.y, outward.z}, uv[2];
  oracle_sphere_uv(pp, uv);
  h->u = uv[0];
  h->v = uv[1];
  h->mat = mat;
  set_face_normal(h, r, outward);
  return 1;
}
/* spherical.rs:117-123 */
static inline vec3 center_at_time(const onode* s, float time) {
  vec3 c0 = v3(s->f[0], s->f[1], s->f[2]), c1 = v3(s->f[4], s->f[5], s->f[6]);
  float t0 = s->f[3], t1 = s->f[7];
  return vadd(c0, vscale(vsub(c1, c0), (time - t0) / (t1 - t0)));
}
/* rectangular.rs:27-57 (XY), :78-108 (XZ), :129-159 (YZ).  axis: 0 XY(k on z) 1 XZ(k on y) 2 YZ(k on x) */
static int hit_rect(const ray* r, float tmin, float tmax, int axis, const float* f, int mat,
                    hitrec* h) {
  float a0 = f[0], a1 = f[1], b0 = f[2], b1 = f[3], k = f[4];
  int kax = axis == 0 ? 2 : (axis == 1 ? 1 : 0);
  int aax = axis == 2 ? 1 : 0;
  int bax = axis == 0 ? 1 : 2;
  float t = (k - vget(r->o, kax)) / vget(r->d, kax);
  if (t < tmin || t > tmax) return 0;
  float x = vget(r->o, aax) + t * vget(r->d, aax);
  float y = vget(r->o, bax) + t * vget(r->d, bax);
  if (x < a0 || x > a1 || y < b0 || y > b1) return 0;
  h->u = (x - a0) / (a1 - a0);
  h->v = (y - b0) / (b1 - b0);
  h->t = t;
  vec3 outward = axis == 0 ? v3(0, 0, 1) : (axis == 1 ? v3(0, 1, 0) : v3(1, 0, 0));
  h->p = ray_at(r, t);
  h->mat = mat;
  set_face_normal(h, r, outward);
  return 1;
}
/* triangular.rs:97-138; interpolate_barycentric :315-323 */
static int hit_tri(const onode* tr, const ray* r, float tmin, float tmax, hitrec* h) {
  vec3 a = tr->tv[0], b = tr->tv[1], c = tr->tv[2];
  vec3 ab = vsub(b, a), ac = vsub(c, a);
  vec3 n = vcross(ab, ac);
  float det = -vdot(r->d, n);
  float inv = 1.0f / det;
  vec3 ao = vsub(r->o, a);
  vec3 aoxd = vcross(ao, r->d);
  float u = vdot(ac, aoxd) * inv;
  float v = -vdot(ab, aoxd) * inv;
  float t = vdot(ao, n) * inv;
  if (t < tmin || t > tmax) return 0;
  if (!(t >= 0.0f && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f)) return 0;
  h->t = t;
  h->p = ray_at(r, t);
  float w = 1.0f - u - v;
  vec3 hn = vadd(vadd(vscale(tr->tn[0], w), vscale(tr->tn[1], u)), vscale(tr->tn[2], v));
  h->u = (w * tr->tuv[0][0] + u * tr->tuv[1][0]) + v * tr->tuv[2][0];
  h->v = (w * tr->tuv[0][1] + u * tr->tuv[1][1]) + v * tr->tuv[2][1];
  h->mat = tr->mat;
  set_face_normal(h, r, hn);
  return 1;
}

static int node_hit(const onode* nd, const ray* r, float tmin, float tmax, int bvh_mode, hitrec* h);
/* The path's RNG state at the start of the current segment (set by world_hit): keys the
 * ConstantMedium draw, see K_MEDIUM below. */
static __thread uint64_t g_seg;

/* hittable/mod.rs:57-69 — linear closest hit, later object wins exact ties */
static int list_hit(onode* const* ch, int n, const ray* r, float tmin, float tmax, int bvh_mode,
                    hitrec* h) {
  float closest = tmax;
  int any = 0;
  hitrec tmp;
  for (int k = 0; k < n; ++k) {
    if (node_hit(ch[k], r, tmin, closest, bvh_mode, &tmp)) {
      closest = tmp.t;
      *h = tmp;
      any = 1;
    }
  }
  return any;
}

static int node_hit(const onode* nd, const ray* r, float tmin, float tmax, int bvh_mode, hitrec* h) {
  switch (nd->kind) {
    case K_LIST:
    case K_CUBOID: /* rectangular.rs:238-240 */
      return list_hit(nd->ch, nd->n, r, tmin, tmax, bvh_mode, h);
    case K_BVH:
      if (bvh_mode == ORACLE_BVH_REFERENCE && nd->ref_tree)
        return node_hit(nd->ref_tree, r, tmin, tmax, bvh_mode, h);
      return list_hit(nd->ch, nd->n, r, tmin, tmax, bvh_mode, h);
    case K_BVHNODE: { /* bvh.rs:100-120 — right child wins ties */
      if (!aabb_hit(&nd->box, r, tmin, tmax)) return 0;
      hitrec hl, hr;
      int l = node_hit(nd->left, r, tmin, tmax, bvh_mode, &hl);
      float tm = l ? hl.t : tmax;
      int rr = nd->right ? node_hit(nd->right, r, tmin, tm, bvh_mode, &hr) : 0;
      if (rr) { *h = hr; return 1; }
      if (l) { *h = hl; return 1; }
      return 0;
    }
    case K_TRANSLATE: { /* transformations.rs:23-38 */
      vec3 off = v3(nd->f[0], nd->f[1], nd->f[2]);
      ray tr = {vsub(r->o, off), r->d, r->time};
      hitrec in;
      if (!list_hit(nd->ch, nd->n, &tr, tmin, tmax, bvh_mode, &in)) return 0;
      *h = in;
      h->p = vadd(in.p, off);
      set_face_normal(h, &tr, in.n);
      return 1;
    }
    case K_ROTY: { /* transformations.rs:115-148 */
      float s = nd->sin_t, c = nd->cos_t;
      ray rr;
      rr.o = v3(c * r->o.x - s * r->o.z, r->o.y, s * r->o.x + c * r->o.z);
      rr.d = v3(c * r->d.x - s * r->d.z, r->d.y, s * r->d.x + c * r->d.z);
      rr.time = r->time;
      hitrec in;
      if (!list_hit(nd->ch, nd->n, &rr, tmin, tmax, bvh_mode, &in)) return 0;
      *h = in;
      h->p = v3(c * in.p.x + s * in.p.z, in.p.y, -s * in.p.x + c * in.p.z);
      vec3 nn = v3(c * in.n.x + s * in.n.z, in.n.y, -s * in.n.x + c * in.n.z);
      set_face_normal(h, &rr, nn);
      return 1;
    }
    case K_SPHERE: /* spherical.rs:86-96 */
      return hit_sphere(r, tmin, tmax, v3(nd->f[0], nd->f[1], nd->f[2]), nd->f[3], nd->mat, h);
    case K_MSPHERE: /* spherical.rs:127-138 */
      return hit_sphere(r, tmin, tmax, center_at_time(nd, r->time), nd->f[8], nd->mat, h);
    case K_RECT:
      return hit_rect(r, tmin, tmax, nd->axis, nd->f, nd->mat, h);
    case K_TRI:
      return hit_tri(nd, r, tmin, tmax, h);
    case K_MEDIUM: { /* volumes.rs:37-78 */
      hitrec r1, r2;
      if (nd->n != 1) return 0;
      if (!node_hit(nd->ch[0], r, -INFINITY, INFINITY, bvh_mode, &r1)) return 0;
      if (!node_hit(nd->ch[0], r, r1.t + 0.0001f, INFINITY, bvh_mode, &r2)) return 0;
      float t1 = fmaxf(r1.t, tmin); /* f32::max ignores NaN = fmaxf */
      /* Deviation: the reference clips rec2 to t_max (the closest hit so far)
       * and draws from the path's shared stream only when the clipped interval is non-empty, so
       * its draws depend on the order objects are tested in.  Here the distance test uses the
       * unclipped rec2 and the draw comes from a sub-stream keyed by (segment state, leaf key);
       * the candidate t is then compared with t_max like any primitive's, which makes the
       * answer independent of traversal order (the GPU's BVH order reproduces it). */
      float t2 = r2.t;
      if (t1 >= t2) return 0;
      t1 = fmaxf(t1, 0.0f);
      float len = sqrtf(vlen2(r->d)); /* vec3.rs:81-83 */
      float dist = (t2 - t1) * len;
      uint64_t g = xoro_seed(oracle_splitmix64(g_seg ^ oracle_splitmix64((uint64_t)nd->key)));
      float hd = nd->f[1] * oracle_log10f(oracle_u32_to_f32(xoro_next(&g)));
      if (hd > dist) return 0;
      float t = t1 + hd / len;
      if (t > tmax) return 0;
      h->t = t;
      h->p = ray_at(r, t);
      h->n = v3(1.0f, 0.0f, 0.0f); /* arbitrary (volumes.rs:65-66) */
      h->front = 1;
      h->u = 0.0f;
      h->v = 0.0f;
      h->mat = nd->mat;
      return 1;
    }
  }
  return 0;
}

/* ---- bounding boxes (reference semantics, used by bvh_mode 1 only) */
static aabb node_box(const onode* nd, float t0, float t1) {
  aabb b = {{0, 0, 0}, {0, 0, 0}, 0};
  switch (nd->kind) {
    case K_SPHERE: { /* spherical.rs:98-103 (inverted for r<0, as in the reference) */
      vec3 c = v3(nd->f[0], nd->f[1], nd->f[2]);
      float rr = nd->f[3];
      vec3 rv = v3(rr, rr, rr);
      b.mn = vsub(c, rv); b.mx = vadd(c, rv); b.ok = 1;
      return b;
    }
    case K_MSPHERE: { /* spherical.rs:140-150 */
      float rr = nd->f[8];
      vec3 rv = v3(rr, rr, rr);
      vec3 c0 = center_at_time(nd, t0), c1 = center_at_time(nd, t1);
      aabb a0 = {vsub(c0, rv), vadd(c0, rv), 1}, a1 = {vsub(c1, rv), vadd(c1, rv), 1};
      return surrounding(a0, a1);
    }
    case K_RECT: { /* rectangular.rs:59-64, :110-115, :161-166 */
      float a0 = nd->f[0], a1 = nd->f[1], b0 = nd->f[2], b1 = nd->f[3], k = nd->f[4];
      if (nd->axis == 0) { b.mn = v3(a0, b0, k - 0.0001f); b.mx = v3(a1, b1, k + 0.0001f); }
      else if (nd->axis == 1) { b.mn = v3(a0, k - 0.0001f, b0); b.mx = v3(a1, k + 0.0001f, b1); }
      else { b.mn = v3(k - 0.0001f, a0, b0); b.mx = v3(k + 0.0001f, a1, b1); }
      b.ok = 1;
      return b;
    }
    case K_CUBOID: /* rectangular.rs:242-244 */
      b.mn = v3(nd->f[0], nd->f[1], nd->f[2]); b.mx = v3(nd->f[3], nd->f[4], nd->f[5]); b.ok = 1;
      return b;
    case K_TRI: { /* triangular.rs:79-93, :140-149 */
      float mn[3], mx[3];
      for (int a = 0; a < 3; ++a) {
        float lo = vget(nd->tv[0], a), hi = lo;
        for (int k = 1; k < 3; ++k) {
          float x = vget(nd->tv[k], a);
          if (x < lo) lo = x;
          if (x > hi) hi = x;
        }
        if (fabsf(lo - hi) < 0.0002f) { lo = lo - 0.0001f; hi = hi + 0.0001f; }
        mn[a] = lo; mx[a] = hi;
      }
      b.mn = v3(mn[0], mn[1], mn[2]); b.mx = v3(mx[0], mx[1], mx[2]); b.ok = 1;
      return b;
    }
    case K_TRANSLATE: { /* transformations.rs:40-47 */
      aabb in = {{0, 0, 0}, {0, 0, 0}, 0};
      for (int k = 0; k < nd->n; ++k) {
        aabb c = node_box(nd->ch[k], t0, t1);
        if (!c.ok) return b;
        in = in.ok ? surrounding(in, c) : c;
      }
      if (!in.ok) return b;
      vec3 off = v3(nd->f[0], nd->f[1], nd->f[2]);
      b.mn = vadd(in.mn, off); b.mx = vadd(in.mx, off); b.ok = 1;
      return b;
    }
    case K_ROTY:
      return nd->rot_box;
    case K_MEDIUM: /* volumes.rs:80-82 */
      return nd->n == 1 ? node_box(nd->ch[0], t0, t1) : b;
    case K_BVHNODE:
      return nd->box;
    case K_LIST:
    case K_BVH: { /* hittable/mod.rs:71-87 */
      for (int k = 0; k < nd->n; ++k) {
        aabb c = node_box(nd->ch[k], t0, t1);
        if (!c.ok) { b.ok = 0; return b; }
        b = b.ok ? surrounding(b, c) : c;
      }
      return b;
    }
  }
  return b;
}
/* transformations.rs:77-111 */
static aabb rotate_box(aabb bb, float s, float c) {
  aabb r;
  r.mn = v3(INFINITY, INFINITY, INFINITY);
  r.mx = v3(-INFINITY, -INFINITY, -INFINITY);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        float fi = (float)i, fj = (float)j, fk = (float)k;
        float x = fi * bb.mx.x + (1.0f - fi) * bb.mn.x;
        float y = fj * bb.mx.y + (1.0f - fj) * bb.mn.y;
        float z = fk * bb.mx.z + (1.0f - fk) * bb.mn.z;
        float nx = c * x + s * z;
        float nz = -s * x + c * z;
        r.mn = v3(fminf(r.mn.x, nx), fminf(r.mn.y, y), fminf(r.mn.z, nz));
        r.mx = v3(fmaxf(r.mx.x, nx), fmaxf(r.mx.y, y), fmaxf(r.mx.z, nz));
      }
  r.ok = 1;
  return r;
}

/* ---- reference BvhNode build (bvh.rs:19-74) with a seeded axis stream */
typedef struct { onode** items; float* key; } sortctx;
static void merge_sort(onode** a, float* key, onode** tmpa, float* tmpk, int n) {
  if (n < 2) return;
  int m = n / 2;
  merge_sort(a, key, tmpa, tmpk, m);
  merge_sort(a + m, key + m, tmpa, tmpk, n - m);
  int i = 0, j = m, o = 0;
  while (i < m && j < n) {
    if (key[j] < key[i]) { tmpa[o] = a[j]; tmpk[o++] = key[j++]; }
    else { tmpa[o] = a[i]; tmpk[o++] = key[i++]; }
  }
  while (i < m) { tmpa[o] = a[i]; tmpk[o++] = key[i++]; }
  while (j < n) { tmpa[o] = a[j]; tmpk[o++] = key[j++]; }
  memcpy(a, tmpa, sizeof(onode*) * n);
  memcpy(key, tmpk, sizeof(float) * n);
}
static onode* build_ref_bvh(onode** objs, int n, float t0, float t1, pcg32* rng) {
  onode* nd = (onode*)calloc(1, sizeof(onode));
  nd->kind = K_BVHNODE;
  /* bvh.rs:25 gen_range(0..=2): widening multiply (rand's UniformInt, not pinned) */
  int axis = (int)(((uint64_t)pcg_next(rng) * 3u) >> 32);
  if (n == 1) {
    nd->left = objs[0];
    nd->right = NULL;
  } else if (n == 2) { /* left = pop() (last), right = pop() (first) */
    nd->left = objs[1];
    nd->right = objs[0];
  } else {
    float* key = (float*)malloc(sizeof(float) * n);
    float* tk = (float*)malloc(sizeof(float) * n);
    onode** ta = (onode**)malloc(sizeof(onode*) * n);
    for (int k = 0; k < n; ++k) key[k] = vget(node_box(objs[k], 0.0f, 0.0f).mn, axis); /* :88-97 */
    merge_sort(objs, key, ta, tk, n); /* Rust sort_by is stable */
    free(key); free(tk); free(ta);
    int mid = n / 2;
    nd->left = build_ref_bvh(objs, mid, t0, t1, rng);
    nd->right = build_ref_bvh(objs + mid, n - mid, t0, t1, rng);
  }
  aabb bl = node_box(nd->left, t0, t1);
  nd->box = nd->right ? surrounding(bl, node_box(nd->right, t0, t1)) : bl;
  return nd;
}

/* ------------------------------------------------------------------ textures / materials */
/* perlin.rs:50-76 noise: lattice corners hashed by permutation xor, trilinear blend (perlin_interp
 * :93-117 — the Hermite-filtered point is used for both the blend and the weight vector, as the
 * reference's shadowing `let point_within_lattice_cell = filter_hermit(..)` makes it) */
static int64_t f32_as_i64(float x) { /* Rust `as i64`: saturating, NaN -> 0 */
  if (x != x) return 0;
  if (x >= 9223372036854775807.0f) return INT64_MAX;
  if (x <= -9223372036854775808.0f) return INT64_MIN;
  return (int64_t)x;
}
static float perlin_noise(const operlin* P, vec3 p) {
  vec3 fl = v3(floorf(p.x), floorf(p.y), floorf(p.z));
  uint64_t base[3] = {(uint64_t)f32_as_i64(fl.x), (uint64_t)f32_as_i64(fl.y), (uint64_t)f32_as_i64(fl.z)};
  vec3 w = vsub(p, fl);
  vec3 g[2][2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        int hash = P->perm[0][(base[0] + (uint64_t)i) & 255] ^ P->perm[1][(base[1] + (uint64_t)j) & 255] ^
                   P->perm[2][(base[2] + (uint64_t)k) & 255];
        g[i][j][k] = P->g[hash];
      }
  vec3 f = vmul(vmul(w, w), vsub(v3(3.0f, 3.0f, 3.0f), vscale(w, 2.0f))); /* filter_hermit :119-122 */
  const vec3 one = v3(1.0f, 1.0f, 1.0f);
  float accum = 0.0f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int k = 0; k < 2; ++k) {
        vec3 c = v3((float)i, (float)j, (float)k);
        vec3 wv = vsub(f, c);
        vec3 bl = vadd(vmul(c, f), vmul(vsub(one, c), vsub(one, f)));
        float bf = bl.x * bl.y * bl.z; /* vec3.rs:58-62 internal_product */
        accum += bf * vdot(g[i][j][k], wv);
      }
  return accum;
}
static float perlin_turbulence(const operlin* P, vec3 p, int depth) { /* perlin.rs:78-91 */
  float accum = 0.0f, weight = 1.0f;
  vec3 tp = p;
  for (int d = 0; d < depth; ++d) {
    accum += weight * perlin_noise(P, tp);
    weight *= 0.5f;
    tp = vscale(tp, 2.0f);
  }
  return fabsf(accum);
}
float oracle_noise(const float* grad, const int32_t* perm, const float p[3], int depth) {
  operlin P;
  for (int k = 0; k < 256; ++k) {
    P.g[k] = v3(grad[3 * k], grad[3 * k + 1], grad[3 * k + 2]);
    for (int a = 0; a < 3; ++a) P.perm[a][k] = perm[256 * a + k];
  }
  return depth <= 0 ? perlin_noise(&P, v3(p[0], p[1], p[2])) : perlin_turbulence(&P, v3(p[0], p[1], p[2]), depth);
}

/* texture.rs:56-60 SolidColor, :69-81 Checker, image_texture.rs:34-52 ImageTexture, texture.rs:97-104 UVDebug */
static vec3 tex_value(const oracle_scene* s, int id, float u, float v, vec3 p) {
  for (;;) {
    const otex* t = &s->tex[id];
    switch (t->kind) {
      case T_SOLID: return v3(t->c[0], t->c[1], t->c[2]);
      case T_CHECKER: {
        float sines = sinf(t->freq * p.x) * sinf(t->freq * p.y) * sinf(t->freq * p.z);
        id = sines < 0.0f ? t->odd : t->even;
        continue;
      }
      case T_IMAGE: {
        float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u); /* f32::clamp keeps NaN */
        float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
        float vv = 1.0f - vc;
        float fi = uu * (float)t->w, fj = vv * (float)t->h;
        uint32_t i = (fi != fi || fi <= 0.0f) ? 0u : (fi >= 4294967295.0f ? 0xFFFFFFFFu : (uint32_t)fi);
        uint32_t j = (fj != fj || fj <= 0.0f) ? 0u : (fj >= 4294967295.0f ? 0xFFFFFFFFu : (uint32_t)fj);
        if (i > (uint32_t)t->w - 1) i = (uint32_t)t->w - 1;
        if (j > (uint32_t)t->h - 1) j = (uint32_t)t->h - 1;
        const uint8_t* px = t->img + ((size_t)j * t->w + i) * 3;
        const float scale = 1.0f / 255.0f;
        return v3((float)px[0] * scale, (float)px[1] * scale, (float)px[2] * scale);
      }
      case T_UVDEBUG: return v3(u, v, 0.0f);
      case T_NOISE: { /* texture.rs:89-95: Color(1,1,1) * 0.5 * (1 + sin(scale z + 10 turb(p, 7))) */
        float tb = perlin_turbulence(t->perlin, p, 7);
        float sv = 0.5f * (1.0f + oracle_sinf(t->freq * p.z + 10.0f * tb));
        return v3(sv, sv, sv);
      }
    }
    return v3(0, 0, 0);
  }
}

/* material.rs:18-21 Scatter */
typedef struct { vec3 att; ray out; } scatter_t;
/* material.rs:108-112 — powi(5) lowers to x * ((x*x)*(x*x)) (LLVM ExpandPowI) */
static inline float reflectance(float cosine, float ref_idx) {
  float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  r0 = r0 * r0;
  float x = 1.0f - cosine;
  float x2 = x * x;
  float x5 = x * (x2 * x2);
  return r0 + (1.0f - r0) * x5;
}
static int mat_scatter(const oracle_scene* s, const omat* m, const ray* rin, const hitrec* h,
                       draws* d, scatter_t* out) {
  switch (m->kind) {
    case M_LAMBERT: { /* material.rs:42-56 */
      vec3 dir = vadd(h->n, rand_unit_vector(d));
      if (vnear_zero(dir)) dir = h->n;
      out->out.o = h->p; out->out.d = dir; out->out.time = rin->time;
      out->att = tex_value(s, m->tex, h->u, h->v, h->p);
      return 1;
    }
    case M_METAL: { /* material.rs:78-95 */
      vec3 refl = vreflect(vunit(rin->d), h->n);
      vec3 dir = vadd(refl, vscale(rand_in_unit_sphere(d), m->fuzz));
      out->out.o = h->p; out->out.d = dir; out->out.time = rin->time;
      out->att = v3(m->albedo[0], m->albedo[1], m->albedo[2]);
      return vdot(dir, h->n) > 0.0f;
    }
    case M_DIELECTRIC: { /* material.rs:116-142 */
      float ir = m->ir;
      float ratio = h->front ? 1.0f / ir : ir;
      vec3 ud = vunit(rin->d);
      float cos_t = fminf(vdot(vneg(ud), h->n), 1.0f);
      float sin_t = sqrtf(1.0f - cos_t * cos_t);
      int cannot = (ratio * sin_t) > 1.0f;
      vec3 dir;
      if (cannot || reflectance(cos_t, ratio) > gen_f32(d)) dir = vreflect(ud, h->n);
      else dir = vrefract(ud, h->n, ratio);
      out->out.o = h->p; out->out.d = dir; out->out.time = rin->time;
      out->att = v3(1.0f, 1.0f, 1.0f);
      return 1;
    }
    case M_LIGHT: /* light_source.rs:18-20 */
      return 0;
    case M_ISOTROPIC: /* material.rs:155-165: random_in_unit_sphere direction, never absorbs */
      out->att = tex_value(s, m->tex, h->u, h->v, h->p);
      out->out.o = h->p; out->out.d = rand_in_unit_sphere(d); out->out.time = rin->time;
      return 1;
  }
  return 0;
}
static vec3 mat_emitted(const oracle_scene* s, const omat* m, const hitrec* h) {
  if (m->kind == M_LIGHT) return tex_value(s, m->tex, h->u, h->v, h->p); /* light_source.rs:22-24 */
  return v3(0, 0, 0); /* material.rs:58-60, 97-99, 144-146 */
}

/* ------------------------------------------------------------------ integrators (lib.rs) */
typedef struct {
  const oracle_scene* s;
  vec3 bg;
  int bvh_mode;
  uint64_t rays;
} ctx_t;

static int world_hit(ctx_t* c, const ray* r, const draws* d, hitrec* h) {
  c->rays++;
  g_seg = d->rng.s;
  return list_hit(c->s->root->ch, c->s->root->n, r, 0.001f, INFINITY, c->bvh_mode, h); /* lib.rs:102 */
}
/* lib.rs:97-117, literal recursion: emitted + attenuation * sample_ray(next) */
static vec3 sample_ray_rec(ctx_t* c, const ray* r, draws* d, uint32_t depth) {
  if (depth == 0) return v3(0, 0, 0);
  hitrec h;
  if (!world_hit(c, r, d, &h)) return c->bg;
  const omat* m = &c->s->mat[h.mat];
  vec3 e = mat_emitted(c->s, m, &h);
  scatter_t sc;
  if (!mat_scatter(c->s, m, r, &h, d, &sc)) return e;
  return vadd(e, vmul(sc.att, sample_ray_rec(c, &sc.out, d, depth - 1)));
}
/* The same estimator, evaluated front-to-back as the GPU does: L = T * terminal with
 * T = ((a0*a1)*a2)...  Identical paths and draws; the product differs from the literal
 * right-to-left recursion only by rounding (tolerance stated in tests). */
/* Debug aid (test infrastructure): ORACLE_TRACE="j,i,s" prints that path's segments to stderr. */
static __thread int g_trace;
static vec3 sample_ray_iter(ctx_t* c, ray r, draws* d, uint32_t depth) {
  vec3 T = v3(1.0f, 1.0f, 1.0f);
  for (; depth > 0; --depth) {
    hitrec h;
    const int hit = world_hit(c, &r, d, &h);
    if (g_trace) {
      fprintf(stderr, "depth %u o (%a %a %a) d (%a %a %a) time %a rng %016llx", depth, r.o.x, r.o.y, r.o.z, r.d.x,
              r.d.y, r.d.z, r.time, (unsigned long long)d->rng.s);
      if (hit)
        fprintf(stderr, " -> t %a p (%a %a %a) n (%a %a %a) mat %d front %d\n", h.t, h.p.x, h.p.y, h.p.z, h.n.x,
                h.n.y, h.n.z, h.mat, h.front);
      else
        fprintf(stderr, " -> miss\n");
    }
    if (!hit) return vmul(T, c->bg);
    const omat* m = &c->s->mat[h.mat];
    scatter_t sc;
    if (!mat_scatter(c->s, m, &r, &h, d, &sc)) return vmul(T, mat_emitted(c->s, m, &h));
    T = vmul(T, sc.att);
    r = sc.out;
  }
  /* depth exhausted: sample_ray(.., 0) returns black (lib.rs:98-100), which every level above multiplies by its
   * attenuation (lib.rs:109-116): T * 0, not a constant 0 -- a NaN or infinite throughput gives NaN, a negative
   * one -0, as the recursion does (RECURSIVE above) */
  return vmul(T, v3(0, 0, 0));
}

typedef struct {
  oracle_scene* s;
  const oracle_camera* cam;
  vec3 bg;
  uint32_t w, h, spp, depth;
  uint64_t seed;
  int integrator, bvh_mode;
  const uint32_t* rows;
  uint32_t n_rows;
  const uint32_t* px; /* oracle_render_pixels: (j, i) pairs, one work item each; the sums go to out[k * 3] */
  uint32_t n_px;
  float* out;
  uint32_t* pixel_rays;
  atomic_uint next;
  atomic_ullong rays;
} job_t;

/* one pixel's sum over its samples in sample order (lib.rs:78-95) */
static vec3 render_pixel(job_t* jb, ctx_t* c, uint32_t j, uint32_t i, long tj, long ti, long ts) {
  vec3 sum = v3(0, 0, 0);
  for (uint32_t sidx = 0; sidx < jb->spp; ++sidx) {
    draws d;
    memset(&d, 0, sizeof d);
    d.rng.s = oracle_path_state(jb->seed, j, i, sidx);
    g_trace = (long)j == tj && (long)i == ti && (long)sidx == ts;
    float u = ((float)i + gen_f32(&d)) / (float)(jb->w - 1u);
    float v = ((float)j + gen_f32(&d)) / (float)(jb->h - 1u);
    ray r = camera_get_ray(jb->cam, u, v, &d);
    vec3 col = jb->integrator == ORACLE_RECURSIVE ? sample_ray_rec(c, &r, &d, jb->depth)
                                                  : sample_ray_iter(c, r, &d, jb->depth);
    sum = vadd(sum, col);
  }
  return sum;
}

static void* worker(void* arg) {
  job_t* jb = (job_t*)arg;
  ctx_t c = {jb->s, jb->bg, jb->bvh_mode, 0};
  long tj = -1, ti = -1, ts = -1;
  const char* tr = getenv("ORACLE_TRACE");
  if (tr) sscanf(tr, "%ld,%ld,%ld", &tj, &ti, &ts);
  for (;;) {
    uint32_t k = atomic_fetch_add(&jb->next, 1u);
    if (jb->px) {
      if (k >= jb->n_px) break;
      const vec3 sum = render_pixel(jb, &c, jb->px[2 * k], jb->px[2 * k + 1], tj, ti, ts);
      float* o = jb->out + (size_t)k * 3;
      o[0] = sum.x; o[1] = sum.y; o[2] = sum.z;
      continue;
    }
    if (k >= jb->n_rows) break;
    uint32_t j = jb->rows ? jb->rows[k] : (jb->h - 1u - k);
    for (uint32_t i = 0; i < jb->w; ++i) {
      const uint64_t rays0 = c.rays;
      const vec3 sum = render_pixel(jb, &c, j, i, tj, ti, ts);
      float* o = jb->out + ((size_t)(jb->h - 1u - j) * jb->w + i) * 3;
      o[0] = sum.x; o[1] = sum.y; o[2] = sum.z;
      if (jb->pixel_rays) jb->pixel_rays[(size_t)(jb->h - 1u - j) * jb->w + i] = (uint32_t)(c.rays - rays0);
    }
  }
  atomic_fetch_add(&jb->rays, c.rays);
  return NULL;
}

int oracle_render(oracle_scene* s, const oracle_camera* cam, const float background[3], uint32_t w,
                  uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, int integrator,
                  int bvh_mode, int n_threads, const uint32_t* rows, uint32_t n_rows, float* out,
                  uint64_t* rays) {
  return oracle_render_counts(s, cam, background, w, h, spp, max_depth, seed, integrator, bvh_mode, n_threads, rows,
                              n_rows, out, rays, NULL);
}
int oracle_render_counts(oracle_scene* s, const oracle_camera* cam, const float background[3], uint32_t w,
                         uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, int integrator,
                         int bvh_mode, int n_threads, const uint32_t* rows, uint32_t n_rows, float* out,
                         uint64_t* rays, uint32_t* pixel_rays) {
  if (!s || !cam || !out || w < 2 || h < 2) { set_err("bad arguments"); return -22; }
  if (w > 65536 || h > 65536) { set_err("w, h <= 65536 (16-bit pixel coordinates in the path key)"); return -22; }
  job_t jb;
  memset(&jb, 0, sizeof jb);
  jb.s = s; jb.cam = cam; jb.bg = v3(background[0], background[1], background[2]);
  jb.w = w; jb.h = h; jb.spp = spp; jb.depth = max_depth; jb.seed = seed;
  jb.integrator = integrator; jb.bvh_mode = bvh_mode;
  jb.rows = rows; jb.n_rows = rows ? n_rows : h;
  jb.out = out;
  jb.pixel_rays = pixel_rays;
  atomic_init(&jb.next, 0u);
  atomic_init(&jb.rays, 0ull);
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, worker, &jb);
  worker(&jb);
  for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
  if (rays) *rays = atomic_load(&jb.rays);
  return 0;
}

/* Selected pixels only: px = n_px (j, i) pairs (j bottom-based, as rows above); out[k * 3 ..] = pixel k's sums.
 * (A full-spp frame's differing pixels re-rendered through another traversal mode, scripts/fullspp_parity.py.) */
int oracle_render_pixels(oracle_scene* s, const oracle_camera* cam, const float background[3], uint32_t w,
                         uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, int integrator, int bvh_mode,
                         int n_threads, const uint32_t* px, uint32_t n_px, float* out, uint64_t* rays) {
  if (!s || !cam || !out || !px || w < 2 || h < 2) { set_err("bad arguments"); return -22; }
  if (w > 65536 || h > 65536) { set_err("w, h <= 65536 (16-bit pixel coordinates in the path key)"); return -22; }
  for (uint32_t k = 0; k < n_px; ++k)
    if (px[2 * k] >= h || px[2 * k + 1] >= w) { set_err("pixel out of the frame"); return -22; }
  job_t jb;
  memset(&jb, 0, sizeof jb);
  jb.s = s; jb.cam = cam; jb.bg = v3(background[0], background[1], background[2]);
  jb.w = w; jb.h = h; jb.spp = spp; jb.depth = max_depth; jb.seed = seed;
  jb.integrator = integrator; jb.bvh_mode = bvh_mode;
  jb.px = px; jb.n_px = n_px;
  jb.out = out;
  atomic_init(&jb.next, 0u);
  atomic_init(&jb.rays, 0ull);
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pthread_t th[256];
  for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, worker, &jb);
  worker(&jb);
  for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
  if (rays) *rays = atomic_load(&jb.rays);
  return 0;
}

/* ------------------------------------------------------------------ scene text parser */
static onode* new_node(int kind) {
  onode* n = (onode*)calloc(1, sizeof(onode));
  n->kind = kind;
  return n;
}
static void add_child(onode* p, onode* c) {
  if (p->n == p->cap) {
    p->cap = p->cap ? p->cap * 2 : 4;
    p->ch = (onode**)realloc(p->ch, sizeof(onode*) * p->cap);
  }
  p->ch[p->n++] = c;
}
static void free_ref(onode* n) {
  if (!n || n->kind != K_BVHNODE) return;
  free_ref(n->left);
  free_ref(n->right);
  free(n);
}
static void free_node(onode* n) {
  if (!n) return;
  for (int k = 0; k < n->n; ++k) free_node(n->ch[k]);
  free(n->ch);
  free_ref(n->ref_tree);
  free(n);
}
void oracle_scene_free(oracle_scene* s) {
  if (!s) return;
  free_node(s->root);
  for (int k = 0; k < s->ntex; ++k) free(s->tex[k].perlin);
  free(s->tex);
  free(s->mat);
  free(s);
}
int oracle_scene_count(const oracle_scene* s, int what) {
  return what == 0 ? s->nleaf : (what == 1 ? s->nmat : s->ntex);
}

typedef struct { const char* p; } lexer;
static int next_tok(lexer* L, char* buf, int cap) {
  while (*L->p == ' ' || *L->p == '\t' || *L->p == '\r') L->p++;
  if (*L->p == '\n' || *L->p == 0) return 0;
  int n = 0;
  while (*L->p && *L->p != ' ' && *L->p != '\t' && *L->p != '\n' && *L->p != '\r') {
    if (n < cap - 1) buf[n++] = *L->p;
    L->p++;
  }
  buf[n] = 0;
  return 1;
}
static int tok_f(lexer* L, float* v) {
  char b[64];
  if (!next_tok(L, b, sizeof b)) return 0;
  char* e;
  double d = strtod(b, &e); /* f64 parse then cast, exact for the %a text the dumper writes */
  if (e == b) return 0;
  *v = (float)d;
  return 1;
}
static int tok_i(lexer* L, long* v) {
  char b[64];
  if (!next_tok(L, b, sizeof b)) return 0;
  char* e;
  *v = strtol(b, &e, 10);
  return e != b;
}
static int tok_fn(lexer* L, float* v, int n) {
  for (int k = 0; k < n; ++k) if (!tok_f(L, &v[k])) return 0;
  return 1;
}

static void prepare(onode* n, oracle_scene* s, pcg32* rng) {
  for (int k = 0; k < n->n; ++k) prepare(n->ch[k], s, rng);
  if (n->kind == K_ROTY) {
    /* transformations.rs:59-75: box of the inner at (0,1), rotated */
    aabb in = {{0, 0, 0}, {0, 0, 0}, 0};
    int ok = 1;
    for (int k = 0; k < n->n; ++k) {
      aabb c = node_box(n->ch[k], 0.0f, 1.0f);
      if (!c.ok) { ok = 0; break; }
      in = in.ok ? surrounding(in, c) : c;
    }
    if (ok && in.ok) n->rot_box = rotate_box(in, n->sin_t, n->cos_t);
  }
  if (n->kind == K_BVH && n->n > 0) {
    onode** objs = (onode**)malloc(sizeof(onode*) * n->n);
    memcpy(objs, n->ch, sizeof(onode*) * n->n);
    n->ref_tree = build_ref_bvh(objs, n->n, n->f[0], n->f[1], rng);
    free(objs);
  }
}

/* a primitive of the world gets the next DFS leaf key; inside a ConstantMedium it is boundary
 * geometry, not a world leaf */
static void add_leaf(oracle_scene* s, onode* parent, onode* n, int medium_depth) {
  if (medium_depth == 0) n->key = (uint32_t)s->nleaf++;
  add_child(parent, n);
}

oracle_scene* oracle_scene_parse(const char* text, const uint8_t* const* images, int n_images) {
  oracle_scene* s = (oracle_scene*)calloc(1, sizeof(oracle_scene));
  s->root = new_node(K_LIST);
  onode* stack[64];
  int sp = 0;
  stack[sp] = s->root;
  lexer L = {text};
  char tok[64];
  int line = 0, ok = 1, medium_depth = 0;
  uint64_t bvh_seed = 0;
  while (*L.p && ok) {
    line++;
    if (next_tok(&L, tok, sizeof tok)) {
      long a = 0, b = 0, c = 0, d = 0;
      float f[32];
      if (!strcmp(tok, "rtwscene") || tok[0] == '#') {
        /* header / comment */
      } else if (!strcmp(tok, "bvhseed")) {
        char bb[64];
        ok = next_tok(&L, bb, sizeof bb);
        if (ok) bvh_seed = strtoull(bb, NULL, 0);
      } else if (!strcmp(tok, "tex")) {
        char kind[32];
        ok = tok_i(&L, &a) && next_tok(&L, kind, sizeof kind) && a == s->ntex;
        if (ok) {
          s->tex = (otex*)realloc(s->tex, sizeof(otex) * (s->ntex + 1));
          otex* t = &s->tex[s->ntex];
          memset(t, 0, sizeof *t);
          if (!strcmp(kind, "solid")) { t->kind = T_SOLID; ok = tok_fn(&L, t->c, 3); }
          else if (!strcmp(kind, "checker")) {
            t->kind = T_CHECKER;
            ok = tok_i(&L, &b) && tok_i(&L, &c) && tok_f(&L, &t->freq);
            t->odd = (int)b; t->even = (int)c;
            ok = ok && b < s->ntex && c < s->ntex;
          } else if (!strcmp(kind, "image")) {
            t->kind = T_IMAGE;
            ok = tok_i(&L, &b) && tok_i(&L, &c) && tok_i(&L, &d) && d >= 0 && d < n_images && b > 0 && c > 0;
            if (ok) { t->w = (int)b; t->h = (int)c; t->img = images[d]; }
          } else if (!strcmp(kind, "uvdebug")) { t->kind = T_UVDEBUG; }
          else if (!strcmp(kind, "noise")) { /* texture.rs:83-87 Noise{noise: Perlin, scale} */
            t->kind = T_NOISE;
            t->perlin = (operlin*)calloc(1, sizeof(operlin));
            ok = tok_f(&L, &t->freq);
            for (int k = 0; ok && k < 256; ++k) {
              float g3[3];
              ok = tok_fn(&L, g3, 3);
              t->perlin->g[k] = v3(g3[0], g3[1], g3[2]);
            }
            for (int k = 0; ok && k < 768; ++k) {
              ok = tok_i(&L, &b) && b >= 0 && b < 256;
              t->perlin->perm[k / 256][k % 256] = (int)b;
            }
          } else ok = 0;
          s->ntex++;
        }
      } else if (!strcmp(tok, "mat")) {
        char kind[32];
        ok = tok_i(&L, &a) && next_tok(&L, kind, sizeof kind) && a == s->nmat;
        if (ok) {
          s->mat = (omat*)realloc(s->mat, sizeof(omat) * (s->nmat + 1));
          omat* m = &s->mat[s->nmat];
          memset(m, 0, sizeof *m);
          if (!strcmp(kind, "lambertian")) { m->kind = M_LAMBERT; ok = tok_i(&L, &b); m->tex = (int)b; ok = ok && b < s->ntex; }
          else if (!strcmp(kind, "metal")) { m->kind = M_METAL; ok = tok_fn(&L, m->albedo, 3) && tok_f(&L, &m->fuzz); }
          else if (!strcmp(kind, "dielectric")) { m->kind = M_DIELECTRIC; ok = tok_f(&L, &m->ir); }
          else if (!strcmp(kind, "light")) { m->kind = M_LIGHT; ok = tok_i(&L, &b); m->tex = (int)b; ok = ok && b < s->ntex; }
          else if (!strcmp(kind, "isotropic")) { m->kind = M_ISOTROPIC; ok = tok_i(&L, &b); m->tex = (int)b; ok = ok && b < s->ntex; }
          else ok = 0;
          s->nmat++;
        }
      } else if (!strcmp(tok, "begin")) {
        char kind[32];
        ok = next_tok(&L, kind, sizeof kind) && sp < 62;
        onode* n = NULL;
        if (ok) {
          if (!strcmp(kind, "list")) n = new_node(K_LIST);
          else if (!strcmp(kind, "bvh")) { n = new_node(K_BVH); ok = tok_fn(&L, f, 2); n->f[0] = f[0]; n->f[1] = f[1]; }
          else if (!strcmp(kind, "translate")) { n = new_node(K_TRANSLATE); ok = tok_fn(&L, n->f, 3); }
          else if (!strcmp(kind, "rotate_y")) {
            n = new_node(K_ROTY);
            ok = tok_f(&L, &n->f[0]);
            float rad = to_radians(n->f[0]); /* transformations.rs:60-63 */
            n->sin_t = sinf(rad);
            n->cos_t = cosf(rad);
          } else if (!strcmp(kind, "medium")) { /* volumes.rs:24-35 ConstantMedium::new */
            n = new_node(K_MEDIUM);
            ok = tok_f(&L, &n->f[0]) && tok_i(&L, &a) && a < s->nmat;
            n->f[1] = -1.0f / n->f[0]; /* neg_inv_density */
            n->mat = (int)a;
            if (ok && medium_depth == 0) n->key = (uint32_t)s->nleaf++;
          } else ok = 0;
        }
        if (ok) { add_child(stack[sp], n); stack[++sp] = n; if (n->kind == K_MEDIUM) medium_depth++; }
      } else if (!strcmp(tok, "end")) {
        ok = sp > 0;
        if (ok && stack[sp]->kind == K_MEDIUM) { medium_depth--; ok = stack[sp]->n == 1; }
        sp--;
      } else if (!strcmp(tok, "sphere")) {
        onode* n = new_node(K_SPHERE);
        ok = tok_fn(&L, n->f, 4) && tok_i(&L, &a) && a < s->nmat;
        n->mat = (int)a;
        add_leaf(s, stack[sp], n, medium_depth);
      } else if (!strcmp(tok, "msphere")) {
        onode* n = new_node(K_MSPHERE);
        ok = tok_fn(&L, n->f, 9) && tok_i(&L, &a) && a < s->nmat;
        n->mat = (int)a;
        add_leaf(s, stack[sp], n, medium_depth);
      } else if (!strcmp(tok, "rect")) {
        char ax[8];
        onode* n = new_node(K_RECT);
        ok = next_tok(&L, ax, sizeof ax) && tok_fn(&L, n->f, 5) && tok_i(&L, &a) && a < s->nmat;
        n->axis = !strcmp(ax, "xy") ? 0 : (!strcmp(ax, "xz") ? 1 : (!strcmp(ax, "yz") ? 2 : -1));
        ok = ok && n->axis >= 0;
        n->mat = (int)a;
        add_leaf(s, stack[sp], n, medium_depth);
      } else if (!strcmp(tok, "cuboid")) {
        /* rectangular.rs:177-234: six sides in this order */
        onode* n = new_node(K_CUBOID);
        ok = tok_fn(&L, n->f, 6) && tok_i(&L, &a) && a < s->nmat;
        n->mat = (int)a;
        float* p0 = n->f;
        float* p1 = n->f + 3;
        float sides[6][6] = {
            {0, p0[0], p1[0], p0[1], p1[1], p1[2]}, {0, p0[0], p1[0], p0[1], p1[1], p0[2]},
            {1, p0[0], p1[0], p0[2], p1[2], p1[1]}, {1, p0[0], p1[0], p0[2], p1[2], p0[1]},
            {2, p0[1], p1[1], p0[2], p1[2], p1[0]}, {2, p0[1], p1[1], p0[2], p1[2], p0[0]}};
        for (int k = 0; k < 6; ++k) {
          onode* r = new_node(K_RECT);
          r->axis = (int)sides[k][0];
          for (int q = 0; q < 5; ++q) r->f[q] = sides[k][q + 1];
          r->mat = (int)a;
          add_leaf(s, n, r, medium_depth);
        }
        add_child(stack[sp], n);
      } else if (!strcmp(tok, "tri")) {
        /* triangular.rs:42-73: missing normals -> geometric normal, missing uv -> defaults */
        onode* n = new_node(K_TRI);
        float vv[9], nn[9], uv[6];
        long nmask = 0, uvmask = 0;
        ok = tok_fn(&L, vv, 9) && tok_i(&L, &nmask) && tok_fn(&L, nn, 9) && tok_i(&L, &uvmask) &&
             tok_fn(&L, uv, 6) && tok_i(&L, &a) && a < s->nmat;
        for (int k = 0; k < 3; ++k) n->tv[k] = v3(vv[3 * k], vv[3 * k + 1], vv[3 * k + 2]);
        vec3 geo = vcross(vsub(n->tv[1], n->tv[0]), vsub(n->tv[2], n->tv[0]));
        const float defuv[3][2] = {{0, 0}, {1, 0}, {0, 1}};
        for (int k = 0; k < 3; ++k) {
          n->tn[k] = (nmask >> k) & 1 ? v3(nn[3 * k], nn[3 * k + 1], nn[3 * k + 2]) : geo;
          n->tuv[k][0] = (uvmask >> k) & 1 ? uv[2 * k] : defuv[k][0];
          n->tuv[k][1] = (uvmask >> k) & 1 ? uv[2 * k + 1] : defuv[k][1];
        }
        n->mat = (int)a;
        add_leaf(s, stack[sp], n, medium_depth);
      } else {
        ok = 0;
      }
    }
    while (*L.p && *L.p != '\n') L.p++;
    if (*L.p == '\n') L.p++;
  }
  if (!ok || sp != 0) {
    char m[96];
    snprintf(m, sizeof m, "scene parse error at line %d", line);
    set_err(m);
    oracle_scene_free(s);
    return NULL;
  }
  pcg32 rng = {oracle_splitmix64(bvh_seed ^ 0x62766873656564ull)};
  prepare(s->root, s, &rng);
  return s;
}

/* ------------------------------------------------------------------ unit-level entry points */
static ray ray_from(const float r[7]) {
  ray o = {v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]), r[6]};
  return o;
}
int oracle_hit_primitive(int kind, const float* p, const float rr[7], float tmin, float tmax,
                         float* out) {
  ray r = ray_from(rr);
  hitrec h;
  int hit = 0;
  onode n;
  memset(&n, 0, sizeof n);
  if (kind == 0) hit = hit_sphere(&r, tmin, tmax, v3(p[0], p[1], p[2]), p[3], 0, &h);
  else if (kind == 1) {
    n.kind = K_MSPHERE;
    memcpy(n.f, p, sizeof(float) * 9);
    hit = hit_sphere(&r, tmin, tmax, center_at_time(&n, r.time), p[8], 0, &h);
  } else if (kind == 2) hit = hit_rect(&r, tmin, tmax, (int)p[0], p + 1, 0, &h);
  else if (kind == 3) {
    for (int k = 0; k < 3; ++k) n.tv[k] = v3(p[3 * k], p[3 * k + 1], p[3 * k + 2]);
    vec3 geo = vcross(vsub(n.tv[1], n.tv[0]), vsub(n.tv[2], n.tv[0]));
    const float defuv[3][2] = {{0, 0}, {1, 0}, {0, 1}};
    for (int k = 0; k < 3; ++k) { n.tn[k] = geo; n.tuv[k][0] = defuv[k][0]; n.tuv[k][1] = defuv[k][1]; }
    hit = hit_tri(&n, &r, tmin, tmax, &h);
  }
  if (!hit) return 0;
  out[0] = h.t; out[1] = h.p.x; out[2] = h.p.y; out[3] = h.p.z;
  out[4] = h.n.x; out[5] = h.n.y; out[6] = h.n.z; out[7] = h.u; out[8] = h.v; out[9] = (float)h.front;
  return 1;
}
int oracle_aabb_hit(const float mn[3], const float mx[3], const float rr[7], float tmin, float tmax) {
  aabb b = {v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]), 1};
  ray r = ray_from(rr);
  return aabb_hit(&b, &r, tmin, tmax);
}
int oracle_scatter(int kind, const float* params, const float rr[7], const float* rec,
                   const uint32_t* arr, uint32_t n_draws, float* out, uint32_t* used) {
  oracle_scene s;
  memset(&s, 0, sizeof s);
  otex t = {T_SOLID, {params[0], params[1], params[2]}, 0, 0, 0, 0, 0, NULL, NULL};
  s.tex = &t; s.ntex = 1;
  omat m;
  memset(&m, 0, sizeof m);
  m.kind = kind == 0 ? M_LAMBERT : (kind == 1 ? M_METAL : M_DIELECTRIC);
  m.albedo[0] = params[0]; m.albedo[1] = params[1]; m.albedo[2] = params[2];
  m.fuzz = params[3]; m.ir = params[3];
  hitrec h;
  h.p = v3(rec[0], rec[1], rec[2]);
  h.n = v3(rec[3], rec[4], rec[5]);
  h.front = rec[6] != 0.0f;
  h.u = h.v = 0; h.t = 0; h.mat = 0;
  draws d;
  memset(&d, 0, sizeof d);
  d.arr = arr; d.n = n_draws;
  ray r = ray_from(rr);
  scatter_t sc;
  int ok = mat_scatter(&s, &m, &r, &h, &d, &sc);
  out[0] = sc.out.d.x; out[1] = sc.out.d.y; out[2] = sc.out.d.z;
  out[3] = sc.att.x; out[4] = sc.att.y; out[5] = sc.att.z;
  *used = d.used;
  return ok;
}
void oracle_get_ray(const oracle_camera* cam, float s, float t, const uint32_t* arr, uint32_t n,
                    float out[7], uint32_t* used) {
  draws d;
  memset(&d, 0, sizeof d);
  d.arr = arr; d.n = n;
  ray r = camera_get_ray(cam, s, t, &d);
  out[0] = r.o.x; out[1] = r.o.y; out[2] = r.o.z;
  out[3] = r.d.x; out[4] = r.d.y; out[5] = r.d.z; out[6] = r.time;
  *used = d.used;
}
/* console_app/src/main.rs:78-88 */
uint8_t oracle_tonemap(float sum, uint32_t spp) {
  float scale = 1.0f / (float)spp;
  float c = sqrtf(scale * sum);
  float cl = c < 0.0f ? 0.0f : (c > 0.999f ? 0.999f : c);
  float x = 255.999f * cl;
  if (x != x || x <= 0.0f) return 0; /* `as u8` saturates, NaN -> 0 */
  if (x >= 255.0f) return 255;
  return (uint8_t)x;
}

/* ConstantMedium::hit (volumes.rs:37-78, order-independent form) around a Sphere (kind 0,
 * params cx cy cz r) or a Cuboid (kind 1, p0[3] p1[3]) with the segment state `seg` and leaf
 * key `key`; returns 1 and *t_out on a hit */
int oracle_medium_hit(int kind, const float* params, float density, const float rr[7], float tmin, float tmax,
                      uint64_t seg, uint32_t key, float* t_out) {
  onode b, sides[6], med;
  onode* side_ptr[6];
  onode* bptr = &b;
  memset(&b, 0, sizeof b);
  memset(&med, 0, sizeof med);
  if (kind == 0) {
    b.kind = K_SPHERE;
    memcpy(b.f, params, 4 * sizeof(float));
  } else {
    const float* p0 = params;
    const float* p1 = params + 3;
    const float sd[6][6] = {{0, p0[0], p1[0], p0[1], p1[1], p1[2]}, {0, p0[0], p1[0], p0[1], p1[1], p0[2]},
                            {1, p0[0], p1[0], p0[2], p1[2], p1[1]}, {1, p0[0], p1[0], p0[2], p1[2], p0[1]},
                            {2, p0[1], p1[1], p0[2], p1[2], p1[0]}, {2, p0[1], p1[1], p0[2], p1[2], p0[0]}};
    b.kind = K_CUBOID;
    for (int k = 0; k < 6; ++k) {
      memset(&sides[k], 0, sizeof sides[k]);
      sides[k].kind = K_RECT;
      sides[k].axis = (int)sd[k][0];
      for (int q = 0; q < 5; ++q) sides[k].f[q] = sd[k][q + 1];
      side_ptr[k] = &sides[k];
    }
    b.ch = side_ptr;
    b.n = 6;
  }
  med.kind = K_MEDIUM;
  med.ch = &bptr;
  med.n = 1;
  med.f[0] = density;
  med.f[1] = -1.0f / density;
  med.key = key;
  g_seg = seg;
  ray r = ray_from(rr);
  hitrec h;
  if (!node_hit(&med, &r, tmin, tmax, ORACLE_BVH_AS_LIST, &h)) return 0;
  *t_out = h.t;
  return 1;
}
