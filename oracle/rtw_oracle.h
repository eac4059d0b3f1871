/*
 * rtw_oracle.h — CPU restatement of raytracer_weekend_lib's render hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline.  The product (raytracer-weekend_amd/, include/rtw.h) never links it.
 *
 * Parity status: the reference (Rust, nightly, rand 0.9.0-alpha.1, unseeded
 * ThreadRng) cannot be built or run in this image, and its test suite holds no
 * golden vectors for this path.  This oracle is pinned by
 *   (a) the reference's in-code KAT table, hittable/spherical.rs:66-68,
 *   (b) analytic KATs derived from cited reference lines, and
 *   (c) golden vectors from an independent numpy float32 restatement
 *       (tests/golden/make_golden.py).
 * Image-level agreement with the reference binary itself is therefore
 * "parity unpinned" (see DESIGN.md §Parity).
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

/* Camera as built by camera.rs:25-64 (Camera::new). */
typedef struct {
  float origin[3], lower_left_corner[3], horizontal[3], vertical[3];
  float u[3], v[3], w[3];
  float lens_radius, time0, time1;
} oracle_camera;

/* Parse the scene text emitted by rtw_scene_dump() (format: DESIGN.md §Scene text).
 * images[k] is the RGB8 buffer of the k-th 'tex image' record. */
oracle_scene* oracle_scene_parse(const char* text, const uint8_t* const* images, int n_images);
void oracle_scene_free(oracle_scene* s);
const char* oracle_last_error(void);
int oracle_scene_count(const oracle_scene* s, int what); /* 0=leaf prims, 1=materials, 2=textures */

void oracle_camera_new(const float look_from[3], const float look_at[3], const float vup[3],
                       float vfov_deg, float aspect, float aperture, float focus_dist,
                       float time0, float time1, oracle_camera* out);

/* Render options. */
enum { ORACLE_ITERATIVE = 0, ORACLE_RECURSIVE = 1 };
enum { ORACLE_BVH_AS_LIST = 0, ORACLE_BVH_REFERENCE = 1 };

/* Render the pixels (j, i) for rows listed in rows[] (all rows when rows == NULL),
 * writing un-normalised Σ over spp (lib.rs:78-95) in the reference emission order
 * (lib.rs:58: j = H-1 .. 0, i = 0 .. W-1) into out[((H-1-j)*W + i)*3 + c].
 * Returns the number of world.hit queries (rays) in *rays. */
int oracle_render(oracle_scene* s, const oracle_camera* cam, const float background[3],
                  uint32_t w, uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed,
                  int integrator, int bvh_mode, int n_threads,
                  const uint32_t* rows, uint32_t n_rows, float* out, uint64_t* rays);
/* The same, also writing each pixel's ray count (all spp samples) into pixel_rays[(H-1-j)*W + i] when non-NULL
 * (a debugging aid: locates paths whose segment counts differ from the GPU's). */
int oracle_render_counts(oracle_scene* s, const oracle_camera* cam, const float background[3],
                         uint32_t w, uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed,
                         int integrator, int bvh_mode, int n_threads,
                         const uint32_t* rows, uint32_t n_rows, float* out, uint64_t* rays, uint32_t* pixel_rays);
/* Selected pixels: px holds n_px (j, i) pairs (j bottom-based); out[k * 3 ..] receives pixel k's sums. */
int oracle_render_pixels(oracle_scene* s, const oracle_camera* cam, const float background[3],
                         uint32_t w, uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed,
                         int integrator, int bvh_mode, int n_threads,
                         const uint32_t* px, uint32_t n_px, float* out, uint64_t* rays);

/* ---- unit-level entry points used by the KAT / golden-vector tests ---- */
uint32_t oracle_pcg32_stream(uint64_t state, uint32_t n, uint32_t* out, uint64_t* state_out);
uint32_t oracle_rng_stream(uint64_t state, uint32_t n, uint32_t* out, uint64_t* state_out);
uint64_t oracle_splitmix64(uint64_t z);
uint64_t oracle_path_state(uint64_t seed, uint32_t j, uint32_t i, uint32_t s);
float oracle_u32_to_f32(uint32_t u);                       /* rand Standard f32 */
float oracle_u32_to_range(uint32_t u, float lo, float hi); /* rand UniformFloat, 1 draw */
double oracle_u64_to_f64(uint64_t u);                      /* rand Standard f64 */
void oracle_sphere_uv(const float p[3], float uv[2]);
/* hit one primitive: kind 0 sphere(cx,cy,cz,r) 1 moving(c0,t0,c1,t1,r) 2 rect(axis,a0,a1,b0,b1,k)
 * 3 triangle(9 verts) ; out: t,p[3],n[3],u,v,front -> 10 floats; returns 1 on hit */
int oracle_hit_primitive(int kind, const float* params, const float ray[7], float tmin, float tmax,
                         float* out);
int oracle_aabb_hit(const float mn[3], const float mx[3], const float ray[7], float tmin, float tmax);
/* scatter with an explicit u32 draw stream: mat kind 0 lambert 1 metal 2 dielectric; params:
 * albedo[3], fuzz/ir.  rec: p[3] n[3] front.  out: dir[3], att[3]; returns 1 if scattered,
 * draws consumed in *used */
int oracle_scatter(int kind, const float* params, const float ray[7], const float* rec,
                   const uint32_t* draws, uint32_t n_draws, float* out, uint32_t* used);
void oracle_get_ray(const oracle_camera* cam, float s, float t, const uint32_t* draws,
                    uint32_t n_draws, float ray_out[7], uint32_t* used);
uint8_t oracle_tonemap(float sum, uint32_t spp);
/* f32 transcendentals as this build defines them (correctly rounded; rtw_oracle.c §libm):
 * fn 0 log10f(a), 1 sinf(a), 2 acosf(a), 3 atan2f(a, b) over n values */
int oracle_libm(int fn, uint32_t n, const float* a, const float* b, float* out);
float oracle_log10f(float x);
float oracle_sinf(float x);
float oracle_acosf(float x);
float oracle_atan2f(float y, float x);
/* ConstantMedium around a Sphere (kind 0: c[3], r) or Cuboid (kind 1: p0[3], p1[3]); seg = path
 * RNG state at the segment start, key = the medium's DFS leaf key; 1 + *t_out on a hit */
int oracle_medium_hit(int kind, const float* params, float density, const float ray[7], float tmin,
                      float tmax, uint64_t seg, uint32_t key, float* t_out);
/* perlin.rs noise (depth <= 0) or turbulence(p, depth); grad: 256x3, perm: 3x256 */
float oracle_noise(const float* grad, const int32_t* perm, const float p[3], int depth);

#ifdef __cplusplus
}
#endif
#endif
