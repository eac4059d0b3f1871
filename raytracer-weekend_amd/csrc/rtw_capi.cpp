// rtw_capi.cpp — builder half of the C-ABI (include/rtw.h): textures, materials,
// hierarchy, primitives, camera, tonemap and the scene-text dump used by the tests.
// Render / device entry points live in rtw_kernel.hip.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <new>
#include <set>
#include <string>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_scene.hpp"

namespace rtw {

static thread_local char g_err[512];

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

const char* tuning_env(const char* name) {
  const char* v = getenv(name);
  if (!v) return nullptr;
  const char* gate = getenv("RTW_TUNING");
  if (gate && !strcmp(gate, "1")) return v;
  static std::mutex mu;  // one warning per knob name and process
  static std::set<std::string> warned;
  std::lock_guard<std::mutex> lock(mu);
  if (warned.insert(name).second)
    fprintf(stderr, "rtw: %s=%s ignored (tuning knobs are read only with RTW_TUNING=1)\n", name, v);
  return nullptr;
}

static int check_open(rtw_scene* s) {
  if (!s) return fail(RTW_EINVAL, "scene is NULL");
  if (s->s.committed) return fail(RTW_ESTATE, "scene already committed");
  return RTW_OK;
}

static uint32_t add_node(Scene& sc, Node&& n) {
  uint32_t id = (uint32_t)sc.nodes.size();
  sc.nodes.push_back(std::move(n));
  sc.nodes[sc.open.back()].ch.push_back(id);
  return id;
}

// f32::to_radians: self * (PI / 180.0) with the constant folded in f32.
static inline float to_radians(float deg) { return deg * (3.14159265358979323846f / 180.0f); }

// ---- scene text (DESIGN.md §Scene text): exact hex floats, tree in prefix order
static void put_f(std::string& o, float v) {
  char b[48];
  snprintf(b, sizeof b, " %a", (double)v);
  o += b;
}
static void dump_node(const Scene& s, uint32_t id, std::string& o) {
  const Node& n = s.nodes[id];
  char b[96];
  switch (n.kind) {
    case NK_LIST:
    case NK_BVH:
    case NK_TRANSLATE:
    case NK_ROTY:
    case NK_MEDIUM: {
      if (n.kind == NK_LIST) o += "begin list";
      else if (n.kind == NK_MEDIUM) {
        o += "begin medium";
        put_f(o, n.f[0]);
        snprintf(b, sizeof b, " %u", n.mat);
        o += b;
      }
      else if (n.kind == NK_BVH) { o += "begin bvh"; put_f(o, n.f[0]); put_f(o, n.f[1]); }
      else if (n.kind == NK_TRANSLATE) { o += "begin translate"; for (int k = 0; k < 3; ++k) put_f(o, n.f[k]); }
      else { o += "begin rotate_y"; put_f(o, n.f[0]); }
      o += "\n";
      for (uint32_t c : n.ch) dump_node(s, c, o);
      o += "end\n";
      return;
    }
    case NK_SPHERE:
      o += "sphere";
      for (int k = 0; k < 4; ++k) put_f(o, n.f[k]);
      break;
    case NK_MSPHERE:
      o += "msphere";
      for (int k = 0; k < 9; ++k) put_f(o, n.f[k]);
      break;
    case NK_RECT:
      o += n.axis == 0 ? "rect xy" : (n.axis == 1 ? "rect xz" : "rect yz");
      for (int k = 0; k < 5; ++k) put_f(o, n.f[k]);
      break;
    case NK_CUBOID:
      o += "cuboid";
      for (int k = 0; k < 6; ++k) put_f(o, n.f[k]);
      break;
    case NK_TRI: {
      o += "tri";
      const float* v = &s.tri_v[9 * (size_t)n.tri];
      const float* nn = &s.tri_n[9 * (size_t)n.tri];
      const float* uv = &s.tri_uv[6 * (size_t)n.tri];
      for (int k = 0; k < 9; ++k) put_f(o, v[k]);
      snprintf(b, sizeof b, " %u", (unsigned)s.tri_nm[n.tri]);
      o += b;
      for (int k = 0; k < 9; ++k) put_f(o, nn[k]);
      snprintf(b, sizeof b, " %u", (unsigned)s.tri_uvm[n.tri]);
      o += b;
      for (int k = 0; k < 6; ++k) put_f(o, uv[k]);
      break;
    }
  }
  snprintf(b, sizeof b, " %u\n", n.mat);
  o += b;
}

std::string dump_scene(const Scene& s) {
  std::string o = "rtwscene 1\n";
  char b[96];
  uint32_t img = 0;
  for (size_t k = 0; k < s.tex.size(); ++k) {
    const TexH& t = s.tex[k];
    snprintf(b, sizeof b, "tex %zu ", k);
    o += b;
    if (t.type == TT_SOLID) { o += "solid"; for (int c = 0; c < 3; ++c) put_f(o, t.c[c]); }
    else if (t.type == TT_CHECKER) { snprintf(b, sizeof b, "checker %u %u", t.odd, t.even); o += b; put_f(o, t.freq); }
    else if (t.type == TT_IMAGE) { snprintf(b, sizeof b, "image %u %u %u", t.w, t.h, img++); o += b; }
    else if (t.type == TT_NOISE) {
      o += "noise";
      put_f(o, t.freq);
      for (float g : t.grad) put_f(o, g);
      for (uint32_t q : t.perm) { snprintf(b, sizeof b, " %u", q); o += b; }
    } else o += "uvdebug";
    o += "\n";
  }
  for (size_t k = 0; k < s.mat.size(); ++k) {
    const MatH& m = s.mat[k];
    snprintf(b, sizeof b, "mat %zu ", k);
    o += b;
    if (m.type == MT_LAMBERT) { snprintf(b, sizeof b, "lambertian %u", m.tex); o += b; }
    else if (m.type == MT_METAL) { o += "metal"; for (int c = 0; c < 3; ++c) put_f(o, m.albedo[c]); put_f(o, m.param); }
    else if (m.type == MT_DIELECTRIC) { o += "dielectric"; put_f(o, m.param); }
    else if (m.type == MT_ISOTROPIC) { snprintf(b, sizeof b, "isotropic %u", m.tex); o += b; }
    else { snprintf(b, sizeof b, "light %u", m.tex); o += b; }
    o += "\n";
  }
  for (uint32_t c : s.nodes[0].ch) dump_node(s, c, o);
  return o;
}

}  // namespace rtw

using namespace rtw;

extern "C" {

const char* rtw_last_error(void) { return rtw::g_err; }
int rtw_abi_version(void) { return RTW_ABI_VERSION; }

int rtw_scene_create(rtw_scene** out) {
  if (!out) return fail(RTW_EINVAL, "out is NULL");
  *out = new (std::nothrow) rtw_scene();
  return *out ? RTW_OK : fail(RTW_ENOMEM, "out of memory");
}
void rtw_scene_destroy(rtw_scene* s) {
  if (!s) return;
  release(s->s);
  delete s;
}

// ---------------------------------------------------------------- textures
static int push_tex(rtw_scene* s, TexH&& t, uint32_t* id) {
  if (int e = check_open(s)) return e;
  s->s.tex.push_back(std::move(t));
  if (id) *id = (uint32_t)s->s.tex.size() - 1;
  return RTW_OK;
}
int rtw_texture_solid(rtw_scene* s, float r, float g, float b, uint32_t* id) {
  TexH t;
  t.type = TT_SOLID;
  t.c[0] = r; t.c[1] = g; t.c[2] = b;
  return push_tex(s, std::move(t), id);
}
int rtw_texture_checker(rtw_scene* s, uint32_t odd, uint32_t even, float freq, uint32_t* id) {
  if (s && (odd >= s->s.tex.size() || even >= s->s.tex.size()))
    return fail(RTW_EINVAL, "checker child texture id out of range");
  TexH t;
  t.type = TT_CHECKER;
  t.odd = odd; t.even = even; t.freq = freq;
  return push_tex(s, std::move(t), id);
}
int rtw_texture_image(rtw_scene* s, const uint8_t* rgb8, uint32_t w, uint32_t h, uint32_t* id) {
  if (!rgb8 || w == 0 || h == 0) return fail(RTW_EINVAL, "image texture needs pixels and w, h > 0");
  TexH t;
  t.type = TT_IMAGE;
  t.w = w; t.h = h;
  t.img.assign(rgb8, rgb8 + (size_t)w * h * 3);
  return push_tex(s, std::move(t), id);
}
int rtw_texture_uvdebug(rtw_scene* s, uint32_t* id) {
  TexH t;
  t.type = TT_UVDEBUG;
  return push_tex(s, std::move(t), id);
}
int rtw_texture_noise(rtw_scene* s, const float* grad, const uint32_t* perm, float scale, uint32_t* id) {
  if (!grad || !perm) return fail(RTW_EINVAL, "noise texture needs 256x3 gradients and 3x256 permutations");
  for (int a = 0; a < 3; ++a) {  // perlin.rs:30-48 builds permutations of 0..255; the hash indexes by them
    bool seen[256] = {};
    for (int k = 0; k < 256; ++k) {
      const uint32_t v = perm[256 * a + k];
      if (v > 255 || seen[v]) return fail(RTW_EINVAL, "noise permutation %d is not a permutation of 0..255", a);
      seen[v] = true;
    }
  }
  TexH t;
  t.type = TT_NOISE;
  t.freq = scale;
  t.grad.assign(grad, grad + 768);
  t.perm.assign(perm, perm + 768);
  return push_tex(s, std::move(t), id);
}

// ---------------------------------------------------------------- materials
static int push_mat(rtw_scene* s, MatH&& m, uint32_t* id) {
  if (int e = check_open(s)) return e;
  s->s.mat.push_back(m);
  if (id) *id = (uint32_t)s->s.mat.size() - 1;
  return RTW_OK;
}
int rtw_material_lambertian(rtw_scene* s, uint32_t tex, uint32_t* id) {
  if (s && tex >= s->s.tex.size()) return fail(RTW_EINVAL, "texture id out of range");
  MatH m;
  m.type = MT_LAMBERT; m.tex = tex;
  return push_mat(s, std::move(m), id);
}
int rtw_material_metal(rtw_scene* s, float r, float g, float b, float fuzz, uint32_t* id) {
  if (!(fuzz <= 1.0f)) return fail(RTW_EINVAL, "Metal::new: assertion failed: fuzz <= 1.0 (material.rs:71)");
  MatH m;
  m.type = MT_METAL;
  m.albedo[0] = r; m.albedo[1] = g; m.albedo[2] = b; m.param = fuzz;
  return push_mat(s, std::move(m), id);
}
int rtw_material_dielectric(rtw_scene* s, float ir, uint32_t* id) {
  MatH m;
  m.type = MT_DIELECTRIC; m.param = ir;
  return push_mat(s, std::move(m), id);
}
int rtw_material_isotropic(rtw_scene* s, uint32_t tex, uint32_t* id) {
  if (s && tex >= s->s.tex.size()) return fail(RTW_EINVAL, "texture id out of range");
  MatH m;
  m.type = MT_ISOTROPIC; m.tex = tex;
  return push_mat(s, std::move(m), id);
}
int rtw_material_diffuse_light(rtw_scene* s, uint32_t tex, uint32_t* id) {
  if (s && tex >= s->s.tex.size()) return fail(RTW_EINVAL, "texture id out of range");
  MatH m;
  m.type = MT_LIGHT; m.tex = tex;
  return push_mat(s, std::move(m), id);
}

// ---------------------------------------------------------------- hierarchy
static int begin(rtw_scene* s, Node&& n) {
  if (int e = check_open(s)) return e;
  if (s->s.open.size() > 48) return fail(RTW_EINVAL, "hierarchy nested too deeply");
  uint32_t id = add_node(s->s, std::move(n));
  s->s.open.push_back(id);
  return RTW_OK;
}
int rtw_begin_list(rtw_scene* s) { return begin(s, Node{NK_LIST, {}}); }
int rtw_begin_bvh(rtw_scene* s, float t0, float t1) {
  Node n{NK_BVH, {}};
  n.f[0] = t0; n.f[1] = t1;
  return begin(s, std::move(n));
}
int rtw_begin_translate(rtw_scene* s, float x, float y, float z) {
  Node n{NK_TRANSLATE, {}};
  n.f[0] = x; n.f[1] = y; n.f[2] = z;
  return begin(s, std::move(n));
}
int rtw_begin_rotate_y(rtw_scene* s, float deg) {
  Node n{NK_ROTY, {}};
  n.f[0] = deg;
  float rad = to_radians(deg);  // transformations.rs:60-63
  n.sin_t = sinf(rad);
  n.cos_t = cosf(rad);
  return begin(s, std::move(n));
}
int rtw_begin_constant_medium(rtw_scene* s, float density, uint32_t tex, uint32_t* material) {
  if (int e = check_open(s)) return e;
  if (tex >= s->s.tex.size()) return fail(RTW_EINVAL, "texture id out of range");
  uint32_t m = 0;
  if (int e = rtw_material_isotropic(s, tex, &m)) return e;  // volumes.rs:26 Isotropic::new(texture)
  Node n{NK_MEDIUM, {}};
  n.f[0] = density;
  n.mat = m;
  if (material) *material = m;
  return begin(s, std::move(n));
}
int rtw_end(rtw_scene* s) {
  if (int e = check_open(s)) return e;
  if (s->s.open.size() <= 1) return fail(RTW_ESTATE, "rtw_end without an open group");
  if (s->s.nodes[s->s.open.back()].kind == NK_MEDIUM && s->s.nodes[s->s.open.back()].ch.size() != 1)
    return fail(RTW_EINVAL, "ConstantMedium needs exactly one boundary object (volumes.rs:17-21)");
  s->s.open.pop_back();
  return RTW_OK;
}

// ---------------------------------------------------------------- primitives
static int check_mat(rtw_scene* s, uint32_t m) {
  return m < s->s.mat.size() ? RTW_OK : fail(RTW_EINVAL, "material id %u out of range", m);
}
int rtw_add_spheres(rtw_scene* s, uint32_t n, const float* cx, const float* cy, const float* cz,
                    const float* r, const uint32_t* mat) {
  if (int e = check_open(s)) return e;
  if (n && (!cx || !cy || !cz || !r || !mat)) return fail(RTW_EINVAL, "NULL array");
  for (uint32_t k = 0; k < n; ++k) {
    if (int e = check_mat(s, mat[k])) return e;
    Node nd{NK_SPHERE, {}};
    nd.f[0] = cx[k]; nd.f[1] = cy[k]; nd.f[2] = cz[k]; nd.f[3] = r[k];
    nd.mat = mat[k];
    add_node(s->s, std::move(nd));
  }
  return RTW_OK;
}
int rtw_add_moving_spheres(rtw_scene* s, uint32_t n, const float* c0x, const float* c0y,
                           const float* c0z, const float* t0, const float* c1x, const float* c1y,
                           const float* c1z, const float* t1, const float* r, const uint32_t* mat) {
  if (int e = check_open(s)) return e;
  if (n && (!c0x || !c0y || !c0z || !t0 || !c1x || !c1y || !c1z || !t1 || !r || !mat))
    return fail(RTW_EINVAL, "NULL array");
  for (uint32_t k = 0; k < n; ++k) {
    if (int e = check_mat(s, mat[k])) return e;
    Node nd{NK_MSPHERE, {}};
    float v[9] = {c0x[k], c0y[k], c0z[k], t0[k], c1x[k], c1y[k], c1z[k], t1[k], r[k]};
    memcpy(nd.f, v, sizeof v);
    nd.mat = mat[k];
    add_node(s->s, std::move(nd));
  }
  return RTW_OK;
}
int rtw_add_rects(rtw_scene* s, uint32_t n, const uint32_t* axis, const float* a0, const float* a1,
                  const float* b0, const float* b1, const float* k, const uint32_t* mat) {
  if (int e = check_open(s)) return e;
  if (n && (!axis || !a0 || !a1 || !b0 || !b1 || !k || !mat)) return fail(RTW_EINVAL, "NULL array");
  for (uint32_t q = 0; q < n; ++q) {
    if (int e = check_mat(s, mat[q])) return e;
    if (axis[q] > 2) return fail(RTW_EINVAL, "rect axis must be 0 (XY), 1 (XZ) or 2 (YZ)");
    Node nd{NK_RECT, {}};
    nd.axis = axis[q];
    nd.f[0] = a0[q]; nd.f[1] = a1[q]; nd.f[2] = b0[q]; nd.f[3] = b1[q]; nd.f[4] = k[q];
    nd.mat = mat[q];
    add_node(s->s, std::move(nd));
  }
  return RTW_OK;
}
int rtw_add_cuboid(rtw_scene* s, const float p0[3], const float p1[3], uint32_t mat) {
  if (int e = check_open(s)) return e;
  if (!p0 || !p1) return fail(RTW_EINVAL, "NULL corner");
  if (int e = check_mat(s, mat)) return e;
  Node nd{NK_CUBOID, {}};
  for (int q = 0; q < 3; ++q) { nd.f[q] = p0[q]; nd.f[3 + q] = p1[q]; }
  nd.mat = mat;
  add_node(s->s, std::move(nd));
  return RTW_OK;
}
int rtw_add_triangles(rtw_scene* s, uint32_t n, const float* verts, const float* normals,
                      const uint8_t* nmask, const float* uvs, const uint8_t* uvmask, uint32_t mat) {
  if (int e = check_open(s)) return e;
  if (n && !verts) return fail(RTW_EINVAL, "NULL vertex array");
  if (int e = check_mat(s, mat)) return e;
  Scene& sc = s->s;
  for (uint32_t q = 0; q < n; ++q) {
    uint32_t t = (uint32_t)sc.tri_nm.size();
    sc.tri_v.insert(sc.tri_v.end(), verts + 9 * (size_t)q, verts + 9 * (size_t)q + 9);
    uint8_t nm = normals ? (nmask ? (uint8_t)(nmask[q] & 7) : 7) : 0;
    uint8_t um = uvs ? (uvmask ? (uint8_t)(uvmask[q] & 7) : 7) : 0;
    for (int k = 0; k < 9; ++k) sc.tri_n.push_back(normals ? normals[9 * (size_t)q + k] : 0.f);
    for (int k = 0; k < 6; ++k) sc.tri_uv.push_back(uvs ? uvs[6 * (size_t)q + k] : 0.f);
    sc.tri_nm.push_back(nm);
    sc.tri_uvm.push_back(um);
    Node nd{NK_TRI, {}};
    nd.tri = t;
    nd.mat = mat;
    add_node(sc, std::move(nd));
  }
  return RTW_OK;
}

int rtw_scene_commit(rtw_scene* s, int device) {
  if (!s) return fail(RTW_EINVAL, "scene is NULL");
  if (s->s.committed) return fail(RTW_ESTATE, "scene already committed");
  if (s->s.open.size() != 1) return fail(RTW_ESTATE, "%zu group(s) still open", s->s.open.size() - 1);
  if (int e = flatten(s->s)) return e;
  if (int e = upload(s->s, device)) return e;
  s->s.committed = true;
  return RTW_OK;
}

// ---------------------------------------------------------------- camera (camera.rs:25-64)
int rtw_camera_new(const float lf[3], const float la[3], const float up[3], float vfov,
                   float aspect, float aperture, float focus, float t0, float t1, rtw_camera* c) {
  if (!lf || !la || !up || !c) return fail(RTW_EINVAL, "NULL argument");
  if (!(t0 < t1)) return fail(RTW_EINVAL, "camera needs time0 < time1 (rand gen_range panics otherwise)");
  auto sub = [](const float* a, const float* b, float* o) { for (int k = 0; k < 3; ++k) o[k] = a[k] - b[k]; };
  auto cross = [](const float* a, const float* b, float* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
  };
  auto unit = [](float* a) {
    float l = sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    for (int k = 0; k < 3; ++k) a[k] = a[k] / l;
  };
  float theta = to_radians(vfov);
  float h = tanf(theta / 2.0f);
  float vh = 2.0f * h;
  float vw = aspect * vh;
  float w[3], u[3], v[3];
  sub(lf, la, w);
  unit(w);
  cross(up, w, u);
  unit(u);
  cross(w, u, v);
  float fh = focus * vw, fv = focus * vh;
  for (int k = 0; k < 3; ++k) {
    c->origin[k] = lf[k];
    c->horizontal[k] = u[k] * fh;
    c->vertical[k] = v[k] * fv;
    c->u[k] = u[k];
    c->v[k] = v[k];
    c->w[k] = w[k];
  }
  for (int k = 0; k < 3; ++k)
    c->lower_left_corner[k] = ((lf[k] - c->horizontal[k] / 2.0f) - c->vertical[k] / 2.0f) - w[k] * focus;
  c->lens_radius = aperture / 2.0f;
  c->time0 = t0;
  c->time1 = t1;
  return RTW_OK;
}

// ---------------------------------------------------------------- tonemap (console_app/src/main.rs:78-88)
int rtw_tonemap(const float* sum, uint32_t n, uint32_t spp, uint8_t* out) {
  if ((!sum || !out) && n) return fail(RTW_EINVAL, "NULL buffer");
  if (spp == 0) return fail(RTW_EINVAL, "spp must be > 0");
  float scale = 1.0f / (float)spp;
  for (size_t q = 0; q < (size_t)n * 3; ++q) {
    float c = sqrtf(scale * sum[q]);
    float cl = c < 0.0f ? 0.0f : (c > 0.999f ? 0.999f : c);  // f32::clamp keeps NaN
    float x = 255.999f * cl;
    out[q] = (x != x || x <= 0.0f) ? 0 : (x >= 255.0f ? 255 : (uint8_t)x);  // `as u8` saturates
  }
  return RTW_OK;
}

// ---------------------------------------------------------------- ProgressMessage wire format
// postcard 0.7: varint (LEB128) u32 and enum tags, f32 little-endian; then COBS + 0x00.
static void put_varint(std::vector<uint8_t>& o, uint32_t v) {
  while (v >= 0x80) { o.push_back((uint8_t)(v | 0x80)); v >>= 7; }
  o.push_back((uint8_t)v);
}
static void put_f32(std::vector<uint8_t>& o, float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  for (int k = 0; k < 4; ++k) o.push_back((uint8_t)(b >> (8 * k)));
}
int rtw_progress_encode(const rtw_progress_msg* m, uint8_t* out, size_t cap, size_t* len) {
  if (!m || !len || (!out && cap)) return fail(RTW_EINVAL, "NULL argument");
  std::vector<uint8_t> raw;
  put_varint(raw, m->kind);
  if (m->kind == RTW_MSG_IMAGE_START) {
    put_varint(raw, m->width); put_varint(raw, m->height); put_varint(raw, m->samples_per_pixel);
  } else if (m->kind == RTW_MSG_PIXEL) {
    put_varint(raw, m->pixel.row); put_varint(raw, m->pixel.column);
    for (int c = 0; c < 3; ++c) put_f32(raw, m->pixel.color[c]);
  } else if (m->kind != RTW_MSG_IMAGE_END) {
    return fail(RTW_EINVAL, "unknown ProgressMessage kind %u", m->kind);
  }
  // COBS: each block = (1 + run length of non-zero bytes, max 254) then the run
  std::vector<uint8_t> enc(1, 0);
  size_t code_at = 0;
  uint8_t code = 1;
  for (uint8_t b : raw) {
    if (b == 0) {
      enc[code_at] = code; code_at = enc.size(); enc.push_back(0); code = 1;
    } else {
      enc.push_back(b);
      if (++code == 0xFF) { enc[code_at] = code; code_at = enc.size(); enc.push_back(0); code = 1; }
    }
  }
  enc[code_at] = code;
  enc.push_back(0);  // frame delimiter (to_vec_cobs)
  *len = enc.size();
  if (cap < enc.size()) return fail(RTW_EINVAL, "buffer too small (%zu < %zu)", cap, enc.size());
  memcpy(out, enc.data(), enc.size());
  return RTW_OK;
}
int rtw_progress_decode(const uint8_t* f, size_t n, rtw_progress_msg* m) {
  if (!m || (!f && n)) return fail(RTW_EINVAL, "NULL argument");
  if (n && f[n - 1] == 0) --n;
  std::vector<uint8_t> raw;
  for (size_t i = 0; i < n;) {  // COBS decode
    const uint8_t code = f[i++];
    if (code == 0) return fail(RTW_EIO, "COBS: zero byte inside a frame");
    for (uint8_t k = 1; k < code; ++k) {
      if (i >= n) return fail(RTW_EIO, "COBS: truncated block");
      raw.push_back(f[i++]);
    }
    if (code != 0xFF && i < n) raw.push_back(0);
  }
  size_t at = 0;
  auto varint = [&](uint32_t* v) -> bool {
    uint32_t x = 0;
    for (int sh = 0; sh < 35; sh += 7) {
      if (at >= raw.size()) return false;
      const uint8_t b = raw[at++];
      x |= (uint32_t)(b & 0x7F) << sh;
      if (!(b & 0x80)) { *v = x; return true; }
    }
    return false;
  };
  auto f32 = [&](float* v) -> bool {
    if (at + 4 > raw.size()) return false;
    uint32_t b = 0;
    for (int k = 0; k < 4; ++k) b |= (uint32_t)raw[at++] << (8 * k);
    memcpy(v, &b, 4);
    return true;
  };
  memset(m, 0, sizeof *m);
  if (!varint(&m->kind)) return fail(RTW_EIO, "postcard: unexpected end (DeserializeUnexpectedEnd)");
  bool ok = true;
  if (m->kind == RTW_MSG_IMAGE_START) ok = varint(&m->width) && varint(&m->height) && varint(&m->samples_per_pixel);
  else if (m->kind == RTW_MSG_PIXEL)
    ok = varint(&m->pixel.row) && varint(&m->pixel.column) && f32(&m->pixel.color[0]) && f32(&m->pixel.color[1]) &&
         f32(&m->pixel.color[2]);
  else if (m->kind != RTW_MSG_IMAGE_END) return fail(RTW_EIO, "postcard: bad enum tag %u", m->kind);
  if (!ok) return fail(RTW_EIO, "postcard: unexpected end (DeserializeUnexpectedEnd)");
  return RTW_OK;
}

// ---------------------------------------------------------------- introspection
int rtw_scene_dump(const rtw_scene* s, char* buf, size_t cap, size_t* needed) {
  if (!s) return fail(RTW_EINVAL, "scene is NULL");
  std::string t = dump_scene(s->s);
  if (needed) *needed = t.size() + 1;
  if (buf && cap >= t.size() + 1) memcpy(buf, t.c_str(), t.size() + 1);
  else if (buf) return fail(RTW_EINVAL, "buffer too small (%zu < %zu)", cap, t.size() + 1);
  return RTW_OK;
}
int rtw_scene_image(const rtw_scene* s, uint32_t k, const uint8_t** px, uint32_t* w, uint32_t* h) {
  if (!s || !px || !w || !h) return fail(RTW_EINVAL, "NULL argument");
  uint32_t seen = 0;
  for (const TexH& t : s->s.tex) {
    if (t.type != TT_IMAGE) continue;
    if (seen++ == k) { *px = t.img.data(); *w = t.w; *h = t.h; return RTW_OK; }
  }
  return fail(RTW_EINVAL, "no image texture #%u", k);
}
int rtw_scene_nodes(const rtw_scene* s, const void** nodes, uint32_t* n_nodes) {
  if (!s || !nodes || !n_nodes) return fail(RTW_EINVAL, "NULL argument");
  *nodes = s->s.flat.nodes4.empty() ? nullptr : (const void*)s->s.flat.nodes4.data();
  *n_nodes = (uint32_t)s->s.flat.nodes4.size();
  return RTW_OK;
}
int rtw_scene_nodes_half(const rtw_scene* s, const void** nodes, uint32_t* n_nodes) {
  if (!s || !nodes || !n_nodes) return fail(RTW_EINVAL, "NULL argument");
  *nodes = s->s.flat.nodes4h.empty() ? nullptr : (const void*)s->s.flat.nodes4h.data();
  *n_nodes = (uint32_t)s->s.flat.nodes4h.size();
  return RTW_OK;
}
int64_t rtw_scene_info(const rtw_scene* s, int what) {
  if (!s) return -1;
  const Scene& sc = s->s;
  switch (what) {
    case 1: return (int64_t)sc.mat.size();
    case 2: return (int64_t)sc.tex.size();
    case 3: return (int64_t)sc.flat.nodes4.size();
    case 7: return (int64_t)sc.flat.nodes.size();
    case 8: return (int64_t)sc.flat.stack_need;
    case 9: return (int64_t)sc.flat.features;
    case 10: return (int64_t)sc.flat.perlins.size();
    case 11: return (int64_t)sc.flat.stack_need4;
    case 12: return (int64_t)sc.flat.lgroups.size();
    case 13: return (int64_t)sc.flat.rect_fast;
    case 14: return (int64_t)sc.flat.far_check;
    case 15: return (int64_t)llround(1000.0 * (double)sc.flat.far_d0);
    case 4: return (int64_t)sc.flat.depth;
    case 5: return (int64_t)sc.flat.always.size();
    case 6: return (int64_t)sc.flat.insts.size();
    default: {
      if (sc.committed) return (int64_t)sc.flat.prims.size();
      // world leaves in DFS order: a cuboid is six rects, a ConstantMedium one leaf (its boundary
      // is not part of the world)
      int64_t n = 0;
      std::vector<uint32_t> todo{0};
      while (!todo.empty()) {
        const Node& nd = sc.nodes[todo.back()];
        todo.pop_back();
        if (nd.kind == NK_CUBOID) n += 6;
        else if (nd.kind == NK_MEDIUM || nd.kind >= NK_SPHERE) n += 1;
        else todo.insert(todo.end(), nd.ch.begin(), nd.ch.end());
      }
      return n;
    }
  }
}

}  // extern "C"
