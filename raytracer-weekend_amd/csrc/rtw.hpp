// rtw.hpp — C++ mirror of raytracer_weekend_lib's public API on top of the C-ABI.
//
// Same names and argument meaning as the Rust crate, so host code reads like
// console_app: build a world, then Raytracer(world, cam, background, w, h, spp).render().
//   Rust                                          C++ (this header)
//   Camera::new(from, at, up, vfov, a, ap, f, t0, t1)   Camera::new_(...)       camera.rs:25-64
//   SolidColor::new_rgb / Checker::new / UVDebug::new   world.solid_rgb / checker / uv_debug
//   Lambertian::new / Metal::new / Dielectric::new /    world.lambertian / metal / dielectric /
//   DiffuseLight::new                                   diffuse_light                material.rs, light_source.rs
//   Sphere::new / MovingSphere::new / XYRectangle::new  world.sphere / moving_sphere / xy_rect ...
//   Cuboid::new(...).rotate_y(a).translate(v)           world.translate(v, [&]{ world.rotate_y(a, [&]{ world.cuboid(...); }); })
//   BvhNode::new(objs, t0, t1, rng)                     world.bvh(t0, t1, [&]{ ... })
//   load_wavefront_obj(path, rng)                       world.load_wavefront_obj(path)
//   Raytracer::new(..).render() -> Pixel stream         Raytracer(..).render() -> std::vector<Pixel>
// Errors (the reference panics) throw rtw::Error with rtw_last_error()'s message.
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtw.h"

namespace rtw {

struct Error : std::runtime_error {
  int code;
  Error(int c, const char* m) : std::runtime_error(m), code(c) {}
};
inline void check(int rc) {
  if (rc != RTW_OK) throw Error(rc, rtw_last_error());
}

struct Vec3 {
  float x, y, z;
};
using Point3 = Vec3;
using Color = Vec3;

// lib.rs:120-126: row counts from the bottom (j), colour is the un-normalised sum.
struct Pixel {
  uint32_t row, column;
  Color color;
};

struct Camera {
  rtw_camera c{};
  static Camera new_(Point3 from, Point3 at, Vec3 up, float vfov, float aspect, float aperture, float focus,
                     float t0, float t1) {
    Camera k;
    const float f[3] = {from.x, from.y, from.z}, a[3] = {at.x, at.y, at.z}, u[3] = {up.x, up.y, up.z};
    check(rtw_camera_new(f, a, u, vfov, aspect, aperture, focus, t0, t1, &k.c));
    return k;
  }
};

using TextureId = uint32_t;
using MaterialId = uint32_t;

class World {
 public:
  World() { check(rtw_scene_create(&s_)); }
  ~World() { rtw_scene_destroy(s_); }
  World(const World&) = delete;
  World& operator=(const World&) = delete;
  rtw_scene* raw() const { return s_; }

  TextureId solid_rgb(float r, float g, float b) { TextureId t; check(rtw_texture_solid(s_, r, g, b, &t)); return t; }
  TextureId checker(TextureId odd, TextureId even, float freq) { TextureId t; check(rtw_texture_checker(s_, odd, even, freq, &t)); return t; }
  TextureId image(const uint8_t* rgb, uint32_t w, uint32_t h) { TextureId t; check(rtw_texture_image(s_, rgb, w, h, &t)); return t; }
  TextureId uv_debug() { TextureId t; check(rtw_texture_uvdebug(s_, &t)); return t; }
  // Noise::new(Perlin::new(rng), scale): Perlin tables from the build's seeded stream
  TextureId noise(float scale, uint64_t perlin_seed) {
    float g[768];
    uint32_t p[768];
    check(rtw_perlin_generate(perlin_seed, g, p));
    TextureId t;
    check(rtw_texture_noise(s_, g, p, scale, &t));
    return t;
  }

  MaterialId lambertian(TextureId t) { MaterialId m; check(rtw_material_lambertian(s_, t, &m)); return m; }
  MaterialId lambertian_solid(Color c) { return lambertian(solid_rgb(c.x, c.y, c.z)); }
  MaterialId metal(Color albedo, float fuzz) { MaterialId m; check(rtw_material_metal(s_, albedo.x, albedo.y, albedo.z, fuzz, &m)); return m; }
  MaterialId dielectric(float ir) { MaterialId m; check(rtw_material_dielectric(s_, ir, &m)); return m; }
  MaterialId diffuse_light(TextureId t) { MaterialId m; check(rtw_material_diffuse_light(s_, t, &m)); return m; }
  MaterialId isotropic(TextureId t) { MaterialId m; check(rtw_material_isotropic(s_, t, &m)); return m; }

  void sphere(Point3 c, float r, MaterialId m) { check(rtw_add_spheres(s_, 1, &c.x, &c.y, &c.z, &r, &m)); }
  void moving_sphere(Point3 c0, float t0, Point3 c1, float t1, float r, MaterialId m) {
    check(rtw_add_moving_spheres(s_, 1, &c0.x, &c0.y, &c0.z, &t0, &c1.x, &c1.y, &c1.z, &t1, &r, &m));
  }
  void rect(uint32_t axis, float a0, float a1, float b0, float b1, float k, MaterialId m) {
    check(rtw_add_rects(s_, 1, &axis, &a0, &a1, &b0, &b1, &k, &m));
  }
  void xy_rect(float x0, float x1, float y0, float y1, float k, MaterialId m) { rect(0, x0, x1, y0, y1, k, m); }
  void xz_rect(float x0, float x1, float z0, float z1, float k, MaterialId m) { rect(1, x0, x1, z0, z1, k, m); }
  void yz_rect(float y0, float y1, float z0, float z1, float k, MaterialId m) { rect(2, y0, y1, z0, z1, k, m); }
  void cuboid(Point3 p0, Point3 p1, MaterialId m) {
    const float a[3] = {p0.x, p0.y, p0.z}, b[3] = {p1.x, p1.y, p1.z};
    check(rtw_add_cuboid(s_, a, b, m));
  }
  void triangle(const Point3 v[3], MaterialId m) {  // Triangle::new_flat_shaded
    const float f[9] = {v[0].x, v[0].y, v[0].z, v[1].x, v[1].y, v[1].z, v[2].x, v[2].y, v[2].z};
    check(rtw_add_triangles(s_, 1, f, nullptr, nullptr, nullptr, nullptr, m));
  }
  uint32_t load_wavefront_obj(const std::string& path, uint32_t material_override = UINT32_MAX) {
    uint32_t n = 0;
    check(rtw_load_wavefront_obj(s_, path.c_str(), nullptr, material_override, &n));
    return n;
  }
  template <class F> void list(F&& body) { check(rtw_begin_list(s_)); body(); check(rtw_end(s_)); }
  template <class F> void bvh(float t0, float t1, F&& body) { check(rtw_begin_bvh(s_, t0, t1)); body(); check(rtw_end(s_)); }
  template <class F> void translate(Vec3 off, F&& body) { check(rtw_begin_translate(s_, off.x, off.y, off.z)); body(); check(rtw_end(s_)); }
  template <class F> void rotate_y(float deg, F&& body) { check(rtw_begin_rotate_y(s_, deg)); body(); check(rtw_end(s_)); }
  // ConstantMedium::new(boundary, density, texture): body adds the boundary
  template <class F> void constant_medium(float density, TextureId t, F&& body) {
    check(rtw_begin_constant_medium(s_, density, t, nullptr)); body(); check(rtw_end(s_));
  }

  // console_app/src/scenes.rs presets; returns the camera and background
  void preset(const std::string& name, float aspect, uint64_t seed, const std::string& models, Camera& cam, Color& bg) {
    float b[3];
    check(rtw_scene_preset(s_, name.c_str(), aspect, seed, models.c_str(), &cam.c, b));
    bg = Color{b[0], b[1], b[2]};
  }
  // every camera of a preset (animated-book2-final-scene has 30, scenes.rs:622-667)
  static std::vector<Camera> preset_cameras(const std::string& name, float aspect, const std::string& models) {
    uint32_t n = 0;
    check(rtw_preset_cameras(name.c_str(), aspect, models.c_str(), nullptr, 0, &n));
    std::vector<rtw_camera> raw(n);
    check(rtw_preset_cameras(name.c_str(), aspect, models.c_str(), raw.data(), n, &n));
    std::vector<Camera> out(n);
    for (uint32_t k = 0; k < n; ++k) out[k].c = raw[k];
    return out;
  }
  void commit(int device = -1) { check(rtw_scene_commit(s_, device)); }

 private:
  rtw_scene* s_ = nullptr;
};

// lib.rs:40-95
class Raytracer {
 public:
  Raytracer(World& world, const Camera& cam, Color background, uint32_t w, uint32_t h, uint32_t spp,
            uint64_t seed = 0, uint32_t max_depth = 50)
      : world_(world), cam_(cam), bg_(background), w_(w), h_(h), spp_(spp), seed_(seed), depth_(max_depth) {}

  // Un-normalised per-pixel sums, flat RGB in the reference emission order (lib.rs:58).
  std::vector<float> render_sums(rtw_stats* st = nullptr) const {
    std::vector<float> out((size_t)w_ * h_ * 3);
    const float bg[3] = {bg_.x, bg_.y, bg_.z};
    check(rtw_render(world_.raw(), &cam_.c, bg, w_, h_, spp_, depth_, seed_, out.data(), st));
    return out;
  }
  // Raytracer::render(): Pixel stream, rows h-1..0, columns 0..w-1
  std::vector<Pixel> render(rtw_stats* st = nullptr) const {
    std::vector<float> s = render_sums(st);
    std::vector<Pixel> px;
    px.reserve((size_t)w_ * h_);
    for (uint32_t r = 0; r < h_; ++r)
      for (uint32_t i = 0; i < w_; ++i) {
        const float* c = &s[((size_t)r * w_ + i) * 3];
        px.push_back(Pixel{h_ - 1 - r, i, Color{c[0], c[1], c[2]}});
      }
    return px;
  }

 private:
  World& world_;
  Camera cam_;
  Color bg_;
  uint32_t w_, h_, spp_;
  uint64_t seed_;
  uint32_t depth_;
};

}  // namespace rtw
