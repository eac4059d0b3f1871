// rtw_presets.cpp — console_app/src/scenes.rs restated on the builder C-ABI, so the
// CLI, bench.py and the tests can build the reference's scenes without Rust.
//
// thread_rng() (scenes.rs:42, console_app/src/main.rs:40) is replaced by a seeded PCG32
// stream: state0 = splitmix64(splitmix64(seed) ^ 0x5343454E45) ("SCENE").  The draws use
// rand 0.9's conversions (Standard f32/f64, UniformFloat sample_single) in the reference's
// call order, so the layout is a pure function of the seed (tests/test_presets.py checks it
// against an independent Python restatement).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_scene.hpp"

namespace rtw {
namespace {

uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct SceneRng {
  uint64_t s;
  explicit SceneRng(uint64_t seed) : s(splitmix64(splitmix64(seed) ^ 0x5343454E45ull)) {}
  uint32_t next_u32() {
    uint64_t old = s;
    s = old * 6364136223846793005ull + 1442695040888963407ull;
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
  }
  uint64_t next_u64() {  // rand_core next_u64_via_u32: low word first
    uint64_t x = next_u32();
    uint64_t y = next_u32();
    return (y << 32) | x;
  }
  float gen_f32() { return (float)(next_u32() >> 8) * (1.0f / 16777216.0f); }
  double gen_f64() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
  // rand UniformInt<usize>::sample_single(0..n) as a widening multiply (rand's rejection zone is
  // not restated: this stream replaces ThreadRng and is pinned only by tests/test_presets.py)
  uint32_t gen_below(uint32_t n) { return (uint32_t)(((uint64_t)next_u32() * n) >> 32); }
  float gen_range(float lo, float hi) {
    float sc = hi - lo;
    for (;;) {
      uint32_t b = (next_u32() >> 9) | 0x3F800000u;
      float v12;
      memcpy(&v12, &b, 4);
      float r = (v12 - 1.0f) * sc + lo;
      if (r < hi) return r;
      uint32_t sb;
      memcpy(&sb, &sc, 4);
      sb -= 1;
      memcpy(&sc, &sb, 4);
    }
  }
};

#define TRY(x)                 \
  do {                         \
    int e_ = (x);              \
    if (e_) return e_;         \
  } while (0)

int solid(rtw_scene* s, float r, float g, float b, uint32_t* id) { return rtw_texture_solid(s, r, g, b, id); }

// perlin.rs:14-48 Perlin::new(rng): 256 gradients random_min_max(-1..1).unit_vector(), then the x, y, z
// permutations, each a Fisher-Yates shuffle `for i in (1..256).rev() { swap(i, gen_range(0..i)) }`
void perlin_new(SceneRng& rng, float* grad, uint32_t* perm) {
  for (int k = 0; k < 256; ++k) {
    float v[3];
    for (float& c : v) c = rng.gen_range(-1.0f, 1.0f);
    const float len = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);  // vec3.rs:81-87
    for (int a = 0; a < 3; ++a) grad[3 * k + a] = v[a] / len;
  }
  for (int a = 0; a < 3; ++a) {
    uint32_t* p = perm + 256 * a;
    for (uint32_t i = 0; i < 256; ++i) p[i] = i;
    for (uint32_t i = 255; i >= 1; --i) {
      const uint32_t t = rng.gen_below(i);
      const uint32_t x = p[i];
      p[i] = p[t];
      p[t] = x;
    }
  }
}
int noise_tex(rtw_scene* s, SceneRng& rng, float scale, uint32_t* id) {  // texture.rs:83-95 Noise::new
  float grad[768];
  uint32_t perm[768];
  perlin_new(rng, grad, perm);
  return rtw_texture_noise(s, grad, perm, scale, id);
}
int lambert_rgb(rtw_scene* s, float r, float g, float b, uint32_t* id) {
  uint32_t t;
  TRY(solid(s, r, g, b, &t));
  return rtw_material_lambertian(s, t, id);
}
int light_rgb(rtw_scene* s, float r, float g, float b, uint32_t* id) {
  uint32_t t;
  TRY(solid(s, r, g, b, &t));
  return rtw_material_diffuse_light(s, t, id);
}
int ground_checker(rtw_scene* s, uint32_t* mat) {  // scenes.rs:64-69
  uint32_t odd, even, ck;
  TRY(solid(s, 0.2f, 0.3f, 0.1f, &odd));
  TRY(solid(s, 0.9f, 0.9f, 0.9f, &even));
  TRY(rtw_texture_checker(s, odd, even, 10.0f, &ck));
  return rtw_material_lambertian(s, ck, mat);
}
int sphere(rtw_scene* s, float x, float y, float z, float r, uint32_t m) {
  return rtw_add_spheres(s, 1, &x, &y, &z, &r, &m);
}
int rect(rtw_scene* s, uint32_t axis, float a0, float a1, float b0, float b1, float k, uint32_t m) {
  return rtw_add_rects(s, 1, &axis, &a0, &a1, &b0, &b1, &k, &m);
}
void set3(float* d, float a, float b, float c) { d[0] = a; d[1] = b; d[2] = c; }

int camera(rtw_camera* cam, float fx, float fy, float fz, float ax, float ay, float az, float ux, float uy,
           float uz, float vfov, float aspect, float aperture, float focus) {
  float f[3] = {fx, fy, fz}, a[3] = {ax, ay, az}, u[3] = {ux, uy, uz};
  return rtw_camera_new(f, a, u, vfov, aspect, aperture, focus, 0.0f, 1.0f, cam);
}

// models/<stem>.ppm (binary P6, RGB8, top row first; decoded from the reference's JPEG by
// models/make_images.py) -> ImageTexture (image_texture.rs:23-30)
int image_tex(rtw_scene* s, const char* dir, const char* stem, uint32_t* id) {
  std::string path = std::string(dir && *dir ? dir : "models") + "/" + stem + ".ppm";
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return fail(RTW_EIO, "cannot open image '%s' (run models/make_images.py)", path.c_str());
  char magic[3] = {0, 0, 0};
  unsigned w = 0, h = 0, mx = 0;
  const int got = fscanf(f, "%2s %u %u %u", magic, &w, &h, &mx);
  fgetc(f);  // the single whitespace byte after maxval
  std::vector<uint8_t> px((size_t)w * h * 3);
  const bool ok = got == 4 && !strcmp(magic, "P6") && mx == 255 && w && h && w < 65536 && h < 65536 &&
                  fread(px.data(), 1, px.size(), f) == px.size();
  fclose(f);
  if (!ok) return fail(RTW_EIO, "'%s' is not an 8-bit binary PPM", path.c_str());
  return rtw_texture_image(s, px.data(), w, h, id);
}

std::string model(const char* dir, const char* stem) {
  std::string d = dir && *dir ? dir : "models";
  for (const char* ext : {".rtwm", ".obj"}) {
    std::string p = d + "/" + stem + ext;
    FILE* f = fopen(p.c_str(), "rb");
    if (f) { fclose(f); return p; }
  }
  return d + "/" + stem + ".obj";
}

// scenes.rs:63-162
int jumpy_balls(rtw_scene* s, float aspect, uint64_t seed, rtw_camera* cam, float* bg) {
  SceneRng rng(seed);
  uint32_t ground, lam, glass, metal;
  TRY(ground_checker(s, &ground));
  TRY(lambert_rgb(s, 0.4f, 0.2f, 0.1f, &lam));
  TRY(rtw_material_dielectric(s, 1.5f, &glass));
  TRY(rtw_material_metal(s, 0.7f, 0.6f, 0.5f, 0.0f, &metal));
  TRY(sphere(s, 0.0f, -1000.0f, 0.0f, 1000.0f, ground));
  TRY(sphere(s, -4.0f, 0.2f, 0.1f, 1.0f, lam));
  TRY(sphere(s, 0.0f, 1.0f, 0.0f, 1.0f, glass));
  TRY(sphere(s, 0.0f, 1.0f, 0.0f, -0.95f, glass));
  TRY(sphere(s, 4.0f, 1.0f, 0.0f, 1.0f, metal));
  for (int ai = -11; ai < 11; ++ai) {
    for (int bi = -11; bi < 11; ++bi) {
      float a = (float)ai, b = (float)bi;
      float cx = a + 0.9f * rng.gen_f32();
      float cy = 0.2f;
      float cz = b + 0.9f * rng.gen_f32();
      float dx = cx - 4.0f, dy = cy - 0.2f, dz = cz - 0.0f;
      if (sqrtf(dx * dx + dy * dy + dz * dz) <= 0.9f) continue;  // :109-111
      uint32_t m;
      double choose = rng.gen_f64();
      if (choose < 0.8) {  // :116-118 Color::random(rng) * Color::random(rng)
        float r1[3], r2[3];
        for (float& c : r1) c = rng.gen_range(0.0f, 1.0f);
        for (float& c : r2) c = rng.gen_range(0.0f, 1.0f);
        TRY(lambert_rgb(s, r1[0] * r2[0], r1[1] * r2[1], r1[2] * r2[2], &m));
      } else if (choose < 0.95) {  // :119-122
        float al[3];
        for (float& c : al) c = rng.gen_range(0.5f, 1.0f);
        float fuzz = rng.gen_range(0.0f, 0.5f);
        TRY(rtw_material_metal(s, al[0], al[1], al[2], fuzz, &m));
      } else {
        TRY(rtw_material_dielectric(s, 1.5f, &m));
      }
      float c2y = cy + rng.gen_range(0.0f, 0.5f);  // :127
      float t0 = 0.0f, t1 = 1.0f, r = 0.2f;
      TRY(rtw_add_moving_spheres(s, 1, &cx, &cy, &cz, &t0, &cx, &c2y, &cz, &t1, &r, &m));
    }
  }
  TRY(camera(cam, 13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0f, aspect, 0.1f, 10.0f));
  set3(bg, 0.7f, 0.8f, 1.0f);  // DEFAULT_BACKGROUND scenes.rs:862
  return RTW_OK;
}

// scenes.rs:163-206
int two_spheres(rtw_scene* s, float aspect, rtw_camera* cam, float* bg) {
  uint32_t g;
  TRY(ground_checker(s, &g));
  TRY(sphere(s, 0, -10, 0, 10, g));
  TRY(sphere(s, 0, 10, 0, 10, g));
  TRY(camera(cam, 13, 2, 3, 0, 0, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.7f, 0.8f, 1.0f);
  return RTW_OK;
}

// scenes.rs:350-414
int cornell_box(rtw_scene* s, float aspect, rtw_camera* cam, float* bg) {
  uint32_t red, white, green, light;
  TRY(lambert_rgb(s, 0.65f, 0.05f, 0.05f, &red));
  TRY(lambert_rgb(s, 0.73f, 0.73f, 0.73f, &white));
  TRY(lambert_rgb(s, 0.12f, 0.45f, 0.15f, &green));
  TRY(light_rgb(s, 15.0f, 15.0f, 15.0f, &light));
  TRY(rect(s, 2, 0, 555, 0, 555, 555, green));
  TRY(rect(s, 2, 0, 555, 0, 555, 0, red));
  TRY(rect(s, 1, 213, 343, 227, 332, 554, light));
  TRY(rect(s, 1, 0, 555, 0, 555, 0, white));
  TRY(rect(s, 1, 0, 555, 0, 555, 555, white));
  TRY(rect(s, 0, 0, 555, 0, 555, 555, white));
  const float z3[3] = {0, 0, 0};
  const float b1[3] = {165, 330, 165}, b2[3] = {165, 165, 165};
  TRY(rtw_begin_translate(s, 265, 0, 295));  // :357-363
  TRY(rtw_begin_rotate_y(s, 15.0f));
  TRY(rtw_add_cuboid(s, z3, b1, white));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(rtw_begin_translate(s, 130, 0, 65));  // :365-371
  TRY(rtw_begin_rotate_y(s, -18.0f));
  TRY(rtw_add_cuboid(s, z3, b2, white));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(camera(cam, 278, 278, -800, 278, 278, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.0f, 0.0f, 0.0f);
  return RTW_OK;
}

// scenes.rs:672-717
int simple_triangle(rtw_scene* s, float aspect, rtw_camera* cam, float* bg) {
  uint32_t g, dbg, m;
  TRY(ground_checker(s, &g));
  TRY(sphere(s, 0, -10, 0, 10, g));
  TRY(rtw_texture_uvdebug(s, &dbg));
  TRY(rtw_material_lambertian(s, dbg, &m));
  const float v[9] = {-5, 0, 5, 0, 7, 0, 5, 0, -5};
  TRY(rtw_add_triangles(s, 1, v, nullptr, nullptr, nullptr, nullptr, m));
  TRY(camera(cam, 13, 2, 3, 0, 2.5f, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.7f, 0.8f, 1.0f);
  return RTW_OK;
}

// scenes.rs:719-771
int wavefront_cow(rtw_scene* s, float aspect, const char* dir, rtw_camera* cam, float* bg) {
  uint32_t g, lt;
  TRY(ground_checker(s, &g));
  TRY(sphere(s, 0, -10.6f, 0, 10, g));
  TRY(light_rgb(s, 1.4f, 1.3f, 1.3f, &lt));
  TRY(rect(s, 0, 1, 5, 1, 7, 5, lt));
  TRY(rtw_begin_translate(s, 0, 2.5f, 0));
  TRY(rtw_load_wavefront_obj(s, model(dir, "cow-nonormals").c_str(), nullptr, UINT32_MAX, nullptr));
  TRY(rtw_end(s));
  TRY(camera(cam, 13, 2, 3, 0, 2.5f, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.085f, 0.1f, 0.125f);
  return RTW_OK;
}


// scenes.rs:211-252
int two_perlin_spheres(rtw_scene* s, float aspect, uint64_t seed, rtw_camera* cam, float* bg) {
  SceneRng rng(seed);
  uint32_t nt, m;
  TRY(noise_tex(s, rng, 4.0f, &nt));
  TRY(rtw_material_lambertian(s, nt, &m));
  TRY(sphere(s, 0, -1000, 0, 1000, m));
  TRY(sphere(s, 0, 2, 0, 2, m));
  TRY(camera(cam, 13, 2, 3, 0, 0, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.7f, 0.8f, 1.0f);
  return RTW_OK;
}

// scenes.rs:254-288
int earth(rtw_scene* s, float aspect, const char* dir, rtw_camera* cam, float* bg) {
  uint32_t et, m;
  TRY(image_tex(s, dir, "earthmap", &et));
  TRY(rtw_material_lambertian(s, et, &m));
  TRY(sphere(s, 0, 0, 0, 2, m));
  TRY(camera(cam, 13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.7f, 0.8f, 1.0f);
  return RTW_OK;
}

// scenes.rs:290-348
int simple_light(rtw_scene* s, float aspect, uint64_t seed, const char* dir, rtw_camera* cam, float* bg) {
  SceneRng rng(seed);
  uint32_t et, lt, nt, m;
  TRY(image_tex(s, dir, "earthmap", &et));
  TRY(rtw_material_diffuse_light(s, et, &lt));
  TRY(noise_tex(s, rng, 4.0f, &nt));
  TRY(rtw_material_lambertian(s, nt, &m));
  TRY(sphere(s, 0, -1000, 0, 1000, m));
  TRY(sphere(s, 0, 2, 0, 2, m));
  TRY(rect(s, 0, 3, 5, 1, 3, -2, lt));
  TRY(sphere(s, 0, 6, 0, 2, lt));
  TRY(camera(cam, 26, 3, 6, 0, 2, 0, 0, 1, 0, 20.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.0f, 0.0f, 0.0f);
  return RTW_OK;
}

// scenes.rs:416-483: the two boxes of cornell-box as ConstantMedium(density 0.005)
int smokey_cornell_box(rtw_scene* s, float aspect, rtw_camera* cam, float* bg) {
  uint32_t red, white, green, light, black, bright;
  TRY(lambert_rgb(s, 0.65f, 0.05f, 0.05f, &red));
  TRY(lambert_rgb(s, 0.73f, 0.73f, 0.73f, &white));
  TRY(lambert_rgb(s, 0.12f, 0.45f, 0.15f, &green));
  TRY(light_rgb(s, 7.0f, 7.0f, 7.0f, &light));
  TRY(solid(s, 0.0f, 0.0f, 0.0f, &black));
  TRY(solid(s, 1.0f, 1.0f, 1.0f, &bright));
  TRY(rect(s, 2, 0, 555, 0, 555, 555, green));
  TRY(rect(s, 2, 0, 555, 0, 555, 0, red));
  TRY(rect(s, 1, 113, 443, 127, 432, 554, light));
  TRY(rect(s, 1, 0, 555, 0, 555, 0, white));
  TRY(rect(s, 1, 0, 555, 0, 555, 555, white));
  TRY(rect(s, 0, 0, 555, 0, 555, 555, white));
  const float z3[3] = {0, 0, 0};
  const float b1[3] = {165, 330, 165}, b2[3] = {165, 165, 165};
  TRY(rtw_begin_constant_medium(s, 0.005f, black, nullptr));  // :439
  TRY(rtw_begin_translate(s, 265, 0, 295));
  TRY(rtw_begin_rotate_y(s, 15.0f));
  TRY(rtw_add_cuboid(s, z3, b1, white));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(rtw_begin_constant_medium(s, 0.005f, bright, nullptr));  // :440
  TRY(rtw_begin_translate(s, 130, 0, 65));
  TRY(rtw_begin_rotate_y(s, -18.0f));
  TRY(rtw_add_cuboid(s, z3, b2, white));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(camera(cam, 278, 278, -800, 278, 278, 0, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.0f, 0.0f, 0.0f);
  return RTW_OK;
}

// scenes.rs:485-620 (the world only; the camera is set by the callers)
int book2_world(rtw_scene* s, SceneRng& rng, const char* dir) {
  uint32_t ground;
  TRY(lambert_rgb(s, 0.48f, 0.83f, 0.53f, &ground));
  TRY(rtw_begin_bvh(s, 0.0f, 1.0f));  // :513 BvhNode::new(boxes1, 0, 1, rng)
  for (int i = 0; i < 20; ++i)
    for (int j = 0; j < 20; ++j) {
      const float w = 100.0f;
      const float x0 = -1000.0f + (float)i * w, z0 = -1000.0f + (float)j * w, y0 = 0.0f;
      const float x1 = x0 + w, y1 = rng.gen_range(1.0f, 101.0f), z1 = z0 + w;
      const float p0[3] = {x0, y0, z0}, p1[3] = {x1, y1, z1};
      TRY(rtw_add_cuboid(s, p0, p1, ground));
    }
  TRY(rtw_end(s));
  uint32_t light, msm, glass, metal, fog_glass, air_glass, emat, et, nt, pm, white;
  TRY(light_rgb(s, 7.0f, 7.0f, 7.0f, &light));
  TRY(rect(s, 1, 123, 423, 147, 412, 554, light));
  TRY(lambert_rgb(s, 0.7f, 0.3f, 0.1f, &msm));
  {
    const float c0x = 400, c0y = 400, c0z = 200, t0 = 0, c1x = 400 + 30.0f, c1y = 400, c1z = 200, t1 = 1, r = 50;
    TRY(rtw_add_moving_spheres(s, 1, &c0x, &c0y, &c0z, &t0, &c1x, &c1y, &c1z, &t1, &r, &msm));
  }
  TRY(rtw_material_dielectric(s, 1.5f, &glass));
  TRY(sphere(s, 260, 150, 45, 50, glass));
  TRY(rtw_material_metal(s, 0.8f, 0.8f, 0.9f, 1.0f, &metal));
  TRY(sphere(s, 0, 150, 145, 50, metal));
  TRY(rtw_material_dielectric(s, 1.5f, &fog_glass));
  TRY(sphere(s, 360, 150, 145, 70, fog_glass));  // :544-548 the boundary itself, then the medium in it
  uint32_t blue, white_t;
  TRY(solid(s, 0.2f, 0.4f, 0.9f, &blue));
  TRY(rtw_begin_constant_medium(s, 0.2f, blue, nullptr));
  TRY(sphere(s, 360, 150, 145, 70, fog_glass));
  TRY(rtw_end(s));
  TRY(rtw_material_dielectric(s, 1.5f, &air_glass));
  TRY(solid(s, 1.0f, 1.0f, 1.0f, &white_t));
  TRY(rtw_begin_constant_medium(s, 0.0001f, white_t, nullptr));  // :555-563 global mist
  TRY(sphere(s, 0, 0, 0, 5000, air_glass));
  TRY(rtw_end(s));
  TRY(image_tex(s, dir, "earthmap", &et));
  TRY(rtw_material_lambertian(s, et, &emat));
  TRY(sphere(s, 400, 200, 400, 100, emat));
  TRY(noise_tex(s, rng, 0.1f, &nt));
  TRY(rtw_material_lambertian(s, nt, &pm));
  TRY(sphere(s, 220, 280, 300, 80, pm));
  TRY(lambert_rgb(s, 0.73f, 0.73f, 0.73f, &white));
  TRY(rtw_begin_translate(s, -100, 270, 395));  // :589-592
  TRY(rtw_begin_rotate_y(s, 15.0f));
  TRY(rtw_begin_bvh(s, 0.0f, 1.0f));
  for (int k = 0; k < 1000; ++k) {
    float c[3];
    for (float& x : c) x = rng.gen_range(0.0f, 165.0f);  // Point3::random_min_max(rng, 0..165)
    TRY(sphere(s, c[0], c[1], c[2], 10.0f, white));
  }
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  TRY(rtw_end(s));
  return RTW_OK;
}
float dist(const float a[3], const float b[3]) {  // (look_at - look_from).length()
  const float d[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  return sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
}
int book2_final(rtw_scene* s, float aspect, uint64_t seed, const char* dir, rtw_camera* cam, float* bg) {
  SceneRng rng(seed);
  TRY(book2_world(s, rng, dir));
  const float from[3] = {478, 278, -600}, at[3] = {278, 278, 0};
  TRY(camera(cam, 478, 278, -600, 278, 278, 0, 0, 1, 0, 40.0f, aspect, 0.0f, dist(at, from)));
  set3(bg, 0.0f, 0.0f, 0.0f);
  return RTW_OK;
}
// scenes.rs:622-667: the same world under one BvhNode, 30 cameras (3 s at 10 fps) sweeping x
int animated_camera(float aspect, uint32_t frame, rtw_camera* cam) {
  const float frames = 10.0f * 3.0f;
  const float from_x = 478.0f - (float)frame * (2.0f * 478.0f) / frames;
  const float from[3] = {from_x, 278.0f, -600.0f}, at[3] = {278, 278, 278};
  return camera(cam, from[0], from[1], from[2], at[0], at[1], at[2], 0, 1, 0, 40.0f, aspect, 1.0f, dist(at, from));
}
int animated_book2(rtw_scene* s, float aspect, uint64_t seed, const char* dir, rtw_camera* cam, float* bg) {
  SceneRng rng(seed);
  TRY(rtw_begin_bvh(s, 0.0f, 1.0f));
  TRY(book2_world(s, rng, dir));
  TRY(rtw_end(s));
  TRY(animated_camera(aspect, 0, cam));
  set3(bg, 0.0f, 0.0f, 0.0f);
  return RTW_OK;
}
}  // namespace

// Synthetic stand-in for the monument's missing diffuse PNG (.MISSING_LARGE_BLOBS:1):
// 2048x2048 RGB8, 64-px checker of two greys plus a UV gradient.
std::vector<uint8_t> synthetic_monument_texture(uint32_t n) {
  std::vector<uint8_t> px((size_t)n * n * 3);
  for (uint32_t y = 0; y < n; ++y)
    for (uint32_t x = 0; x < n; ++x) {
      int c = (((x >> 6) + (y >> 6)) & 1) ? 176 : 96;
      int r = c + (int)(x * 64u / n) - 32, b = c + (int)(y * 64u / n) - 32;
      uint8_t* p = &px[((size_t)y * n + x) * 3];
      p[0] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
      p[1] = (uint8_t)c;
      p[2] = (uint8_t)(b < 0 ? 0 : (b > 255 ? 255 : b));
    }
  return px;
}

namespace {
// scenes.rs:773-814.  Normals_Try3.obj uses `usemtl` without `mtllib`, so the reference panics in
// load_wavefront_obj (triangular.rs:176 unwrap); this restatement returns that error (RTW_EIO).
int wavefront_suspension(rtw_scene* s, float aspect, const char* dir, rtw_camera* cam, float* bg) {
  uint32_t lt;
  TRY(light_rgb(s, 1.2f, 1.0f, 1.0f, &lt));
  TRY(rect(s, 0, -5, 5, -7, 7, 1, lt));
  TRY(rtw_begin_translate(s, 0, 2.5f, 0));
  TRY(rtw_load_wavefront_obj(s, model(dir, "Normals_Try3").c_str(), nullptr, UINT32_MAX, nullptr));
  TRY(rtw_end(s));
  TRY(camera(cam, 0.5f, 2.5f, 0.8f, -0.1f, 2.3f, 0.15f, 0, 1, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.085f, 0.1f, 0.125f);
  return RTW_OK;
}

// scenes.rs:816-858
int textured_monument(rtw_scene* s, float aspect, const char* dir, rtw_camera* cam, float* bg) {
  uint32_t lt, tex, mat;
  TRY(light_rgb(s, 1.2f, 1.0f, 1.0f, &lt));
  TRY(rect(s, 0, -15, 15, -17, 17, 33, lt));
  std::vector<uint8_t> img = synthetic_monument_texture(2048);
  TRY(rtw_texture_image(s, img.data(), 2048, 2048, &tex));
  TRY(rtw_material_lambertian(s, tex, &mat));
  TRY(rtw_begin_translate(s, 0, 0, -19.0f));
  TRY(rtw_load_wavefront_obj(s, model(dir, "monument_downscaled_polygon_reduced").c_str(), nullptr, mat, nullptr));
  TRY(rtw_end(s));
  TRY(camera(cam, -5, -30, 25, 0, 0, 5, 1, 0, 0, 40.0f, aspect, 0.0f, 10.0f));
  set3(bg, 0.085f, 0.1f, 0.125f);
  return RTW_OK;
}
}  // namespace
}  // namespace rtw

using namespace rtw;

extern "C" int rtw_scene_preset(rtw_scene* s, const char* name, float aspect, uint64_t seed,
                                const char* models_dir, rtw_camera* cam, float bg[3]) {
  if (!s || !name || !cam || !bg) return fail(RTW_EINVAL, "NULL argument");
  if (!strcmp(name, "jumpy-balls")) return jumpy_balls(s, aspect, seed, cam, bg);
  if (!strcmp(name, "two-spheres")) return two_spheres(s, aspect, cam, bg);
  if (!strcmp(name, "cornell-box")) return cornell_box(s, aspect, cam, bg);
  if (!strcmp(name, "simple-triangle")) return simple_triangle(s, aspect, cam, bg);
  if (!strcmp(name, "wavefront-cow-obj")) return wavefront_cow(s, aspect, models_dir, cam, bg);
  if (!strcmp(name, "textured-monument")) return textured_monument(s, aspect, models_dir, cam, bg);
  if (!strcmp(name, "two-perlin-spheres")) return two_perlin_spheres(s, aspect, seed, cam, bg);
  if (!strcmp(name, "earth")) return earth(s, aspect, models_dir, cam, bg);
  if (!strcmp(name, "simple-light")) return simple_light(s, aspect, seed, models_dir, cam, bg);
  if (!strcmp(name, "smokey-cornell-box")) return smokey_cornell_box(s, aspect, cam, bg);
  if (!strcmp(name, "book2-final-scene")) return book2_final(s, aspect, seed, models_dir, cam, bg);
  if (!strcmp(name, "animated-book2-final-scene")) return animated_book2(s, aspect, seed, models_dir, cam, bg);
  if (!strcmp(name, "wavefront-suspension-obj")) return wavefront_suspension(s, aspect, models_dir, cam, bg);
  return fail(RTW_EINVAL,
              "unknown or out-of-scope scene '%s' (available: jumpy-balls, two-spheres, two-perlin-spheres, "
              "earth, simple-light, cornell-box, smokey-cornell-box, book2-final-scene, "
              "animated-book2-final-scene, simple-triangle, wavefront-cow-obj, wavefront-suspension-obj, "
              "textured-monument)",
              name);
}

extern "C" int rtw_preset_cameras(const char* name, float aspect, const char* models_dir, rtw_camera* cams,
                                  uint32_t cap, uint32_t* n) {
  if (!name || !n || (cap && !cams)) return fail(RTW_EINVAL, "NULL argument");
  if (!strcmp(name, "animated-book2-final-scene")) {  // scenes.rs:636-660
    *n = 30;
    for (uint32_t f = 0; f < 30 && f < cap; ++f) TRY(animated_camera(aspect, f, &cams[f]));
    return RTW_OK;
  }
  // every other scene has one camera (vec![cam]); build it on a scratch scene
  rtw_scene* tmp = nullptr;
  TRY(rtw_scene_create(&tmp));
  rtw_camera c;
  float bg[3];
  const int rc = rtw_scene_preset(tmp, name, aspect, 0, models_dir, &c, bg);
  rtw_scene_destroy(tmp);
  if (rc) return rc;
  *n = 1;
  if (cap) cams[0] = c;
  return RTW_OK;
}

extern "C" int rtw_perlin_generate(uint64_t seed, float* gradients, uint32_t* permutations) {
  if (!gradients || !permutations) return fail(RTW_EINVAL, "NULL argument");
  SceneRng rng(seed);
  perlin_new(rng, gradients, permutations);
  return RTW_OK;
}
