// rtw_obj.cpp — load_wavefront_obj (triangular.rs:151-312) for the C-ABI, plus this
// build's `.rtwm` binary mesh format (the OBJ assets re-encoded so the GPU box, which has
// no copy of the reference, can load them).
//
// OBJ semantics kept from the reference: vertex coordinates parsed as f64 and cast to f32
// (triangular.rs:153-166, the wavefront_obj crate stores f64); faces without `usemtl` get
// DiffuseLight(SolidColor(1, 0, 1)) (:177-182); `usemtl` needs the `mtllib` (:176, unwrap);
// MTL materials must be illum 1 with a map_Kd image (:299-312, else panic); every face set
// becomes one BvhNode::new(triangles, 0, 1, rng) (:257-259).  Polygons with more than three
// vertices are fan-triangulated (the wavefront_obj crate's behaviour; parity unpinned).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_scene.hpp"

namespace rtw {
namespace {

bool read_file(const char* path, std::string& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  fclose(f);
  return true;
}

std::string dir_of(const std::string& p) {
  size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

struct FaceSet {
  std::string material;  // "" = none
  std::vector<float> v, n, uv;
  std::vector<uint8_t> nm, um;
};

struct MtlEntry {
  int illum = -1;
  std::string map_kd;
};

int parse_mtl(const std::string& path, std::map<std::string, MtlEntry>& out) {
  std::string text;
  if (!read_file(path.c_str(), text)) return fail(RTW_EIO, "cannot read MTL '%s'", path.c_str());
  std::string cur;
  size_t pos = 0;
  while (pos < text.size()) {
    size_t e = text.find('\n', pos);
    if (e == std::string::npos) e = text.size();
    std::string line = text.substr(pos, e - pos);
    pos = e + 1;
    while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
    char key[64] = {0};
    if (sscanf(line.c_str(), "%63s", key) != 1) continue;
    const char* rest = line.c_str() + strlen(key);
    while (*rest == ' ' || *rest == '\t') ++rest;
    if (!strcmp(key, "newmtl")) { cur = rest; out[cur] = MtlEntry(); }
    else if (!strcmp(key, "illum") && !cur.empty()) out[cur].illum = atoi(rest);
    else if (!strcmp(key, "map_Kd") && !cur.empty()) out[cur].map_kd = rest;
  }
  return RTW_OK;
}

}  // namespace

int load_rtwm(rtw_scene* hs, const char* path, uint32_t mat, uint32_t* ntri_out);

}  // namespace rtw

using namespace rtw;

extern "C" int rtw_load_wavefront_obj(rtw_scene* s, const char* path, rtw_image_loader loader,
                                      uint32_t fallback_material, uint32_t* n_triangles) {
  if (!s || !path) return fail(RTW_EINVAL, "NULL argument");
  if (s->s.committed) return fail(RTW_ESTATE, "scene already committed");
  size_t L = strlen(path);
  if (L > 5 && !strcmp(path + L - 5, ".rtwm")) {
    uint32_t mat = fallback_material;
    if (mat == UINT32_MAX) {  // the reference's no-material fallback, triangular.rs:177-182
      uint32_t t;
      if (int e = rtw_texture_solid(s, 1.0f, 0.0f, 1.0f, &t)) return e;
      if (int e = rtw_material_diffuse_light(s, t, &mat)) return e;
    }
    return load_rtwm(s, path, mat, n_triangles);
  }
  std::string text;
  if (!read_file(path, text)) return fail(RTW_EIO, "cannot read OBJ '%s'", path);
  std::vector<double> V, VT, VN;  // f64 storage as the wavefront_obj crate
  std::vector<FaceSet> sets(1);
  std::string mtllib;
  size_t pos = 0;
  int line_no = 0;
  while (pos < text.size()) {
    size_t e = text.find('\n', pos);
    if (e == std::string::npos) e = text.size();
    const char* p = text.c_str() + pos;
    const char* end = text.c_str() + e;
    pos = e + 1;
    ++line_no;
    while (p < end && (*p == ' ' || *p == '\t')) ++p;
    if (p >= end || *p == '#') continue;
    std::string line(p, end);
    while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
    char key[32] = {0};
    if (sscanf(line.c_str(), "%31s", key) != 1) continue;
    const char* rest = line.c_str() + strlen(key);
    if (!strcmp(key, "v") || !strcmp(key, "vn")) {
      double a, b, c;
      if (sscanf(rest, "%lf %lf %lf", &a, &b, &c) != 3) return fail(RTW_EIO, "%s:%d: bad vertex", path, line_no);
      std::vector<double>& dst = key[1] ? VN : V;
      dst.push_back(a); dst.push_back(b); dst.push_back(c);
    } else if (!strcmp(key, "vt")) {
      double a, b = 0.0;
      if (sscanf(rest, "%lf %lf", &a, &b) < 1) return fail(RTW_EIO, "%s:%d: bad texture vertex", path, line_no);
      VT.push_back(a); VT.push_back(b);
    } else if (!strcmp(key, "mtllib")) {
      while (*rest == ' ' || *rest == '\t') ++rest;
      mtllib = rest;
    } else if (!strcmp(key, "usemtl")) {
      while (*rest == ' ' || *rest == '\t') ++rest;
      sets.emplace_back();
      sets.back().material = rest;
    } else if (!strcmp(key, "f")) {
      struct Idx { long v, t, n; };
      std::vector<Idx> poly;
      const char* q = rest;
      while (*q) {
        while (*q == ' ' || *q == '\t') ++q;
        if (!*q) break;
        Idx ix{0, 0, 0};
        char* nx;
        ix.v = strtol(q, &nx, 10);
        q = nx;
        if (*q == '/') {
          ++q;
          if (*q != '/') { ix.t = strtol(q, &nx, 10); q = nx; }
          if (*q == '/') { ++q; ix.n = strtol(q, &nx, 10); q = nx; }
        }
        while (*q && *q != ' ' && *q != '\t') ++q;
        poly.push_back(ix);
      }
      if (poly.size() < 3) return fail(RTW_EIO, "%s:%d: face with < 3 vertices (triangular.rs:186-191 panics)", path, line_no);
      auto resolve = [](long i, size_t n) -> long { return i > 0 ? i - 1 : (i < 0 ? (long)n + i : -1); };
      FaceSet& fs = sets.back();
      for (size_t k = 1; k + 1 < poly.size(); ++k) {
        const Idx tri[3] = {poly[0], poly[k], poly[k + 1]};
        uint8_t nm = 0, um = 0;
        float vv[9], nn[9] = {0}, uu[6] = {0};
        for (int c = 0; c < 3; ++c) {
          long vi = resolve(tri[c].v, V.size() / 3);
          if (vi < 0 || (size_t)vi >= V.size() / 3) return fail(RTW_EIO, "%s:%d: vertex index out of range", path, line_no);
          for (int a = 0; a < 3; ++a) vv[3 * c + a] = (float)V[3 * vi + a];
          if (tri[c].t) {
            long ti = resolve(tri[c].t, VT.size() / 2);
            if (ti < 0 || (size_t)ti >= VT.size() / 2) return fail(RTW_EIO, "%s:%d: uv index out of range", path, line_no);
            uu[2 * c] = (float)VT[2 * ti];
            uu[2 * c + 1] = (float)VT[2 * ti + 1];
            um |= (uint8_t)(1u << c);
          }
          if (tri[c].n) {
            long ni = resolve(tri[c].n, VN.size() / 3);
            if (ni < 0 || (size_t)ni >= VN.size() / 3) return fail(RTW_EIO, "%s:%d: normal index out of range", path, line_no);
            for (int a = 0; a < 3; ++a) nn[3 * c + a] = (float)VN[3 * ni + a];
            nm |= (uint8_t)(1u << c);
          }
        }
        fs.v.insert(fs.v.end(), vv, vv + 9);
        fs.n.insert(fs.n.end(), nn, nn + 9);
        fs.uv.insert(fs.uv.end(), uu, uu + 6);
        fs.nm.push_back(nm);
        fs.um.push_back(um);
      }
    }
    // o, g, s, l and anything else: ignored (no geometry for the render path)
  }

  // resolve materials (triangular.rs:175-183, :280-312)
  std::map<std::string, MtlEntry> mtl;
  bool need_mtl = false;
  for (const FaceSet& fs : sets) need_mtl |= !fs.material.empty() && !fs.v.empty();
  if (need_mtl && fallback_material == UINT32_MAX) {
    if (mtllib.empty()) return fail(RTW_EIO, "%s: usemtl without mtllib (triangular.rs:176 unwrap)", path);
    if (int e = parse_mtl(dir_of(path) + "/" + mtllib, mtl)) return e;
  }
  // every material is resolved before the BvhNode group opens, so a parse / texture error leaves
  // the caller's scene without a dangling open group
  std::map<std::string, uint32_t> mat_ids;
  uint32_t magenta = UINT32_MAX;
  std::vector<uint32_t> set_mat(sets.size(), UINT32_MAX);
  for (size_t q = 0; q < sets.size(); ++q) {
    const FaceSet& fs = sets[q];
    if (fs.nm.empty()) continue;
    uint32_t mat;
    if (fallback_material != UINT32_MAX) {
      mat = fallback_material;
    } else if (fs.material.empty()) {
      if (magenta == UINT32_MAX) {
        uint32_t t;
        if (int e = rtw_texture_solid(s, 1.0f, 0.0f, 1.0f, &t)) return e;
        if (int e = rtw_material_diffuse_light(s, t, &magenta)) return e;
      }
      mat = magenta;
    } else {
      auto it = mat_ids.find(fs.material);
      if (it != mat_ids.end()) {
        mat = it->second;
      } else {
        auto m = mtl.find(fs.material);
        if (m == mtl.end()) return fail(RTW_EIO, "material '%s' not in MTL", fs.material.c_str());
        if (m->second.illum != 1) return fail(RTW_EIO, "material '%s': illum != 1 (triangular.rs:300 panics)", fs.material.c_str());
        if (m->second.map_kd.empty()) return fail(RTW_EIO, "material '%s' has no map_Kd (triangular.rs:309 unwrap)", fs.material.c_str());
        if (!loader) return fail(RTW_EIO, "no image loader for '%s' (the build ships no JPEG/PNG decoder)", m->second.map_kd.c_str());
        uint8_t* px = nullptr;
        uint32_t w = 0, h = 0;
        std::string ip = dir_of(path) + "/" + m->second.map_kd;
        if (loader(ip.c_str(), &px, &w, &h) != 0 || !px)
          return fail(RTW_EIO, "cannot load texture '%s' (image_texture.rs:24 / triangular.rs:308 unwrap)", ip.c_str());
        uint32_t t;
        int e = rtw_texture_image(s, px, w, h, &t);
        free(px);
        if (e) return e;
        if ((e = rtw_material_lambertian(s, t, &mat))) return e;
        mat_ids[fs.material] = mat;
      }
    }
    set_mat[q] = mat;
  }
  uint32_t total = 0;
  if (int e = rtw_begin_bvh(s, 0.0f, 1.0f)) return e;
  for (size_t q = 0; q < sets.size(); ++q) {
    const FaceSet& fs = sets[q];
    const uint32_t n = (uint32_t)fs.nm.size();
    if (!n) continue;
    if (int e = rtw_add_triangles(s, n, fs.v.data(), fs.n.data(), fs.nm.data(), fs.uv.data(), fs.um.data(), set_mat[q])) {
      rtw_end(s);  // close the group: the caller sees this error, not "group(s) still open" at commit
      return e;
    }
    total += n;
  }
  if (int e = rtw_end(s)) return e;
  if (n_triangles) *n_triangles = total;
  return RTW_OK;
}

namespace rtw {
// .rtwm: "RTWM" u32 version(1) u32 ntri u32 flags(1 normals, 2 uvs) | f32 v[9n] |
//        [f32 n[9n] u8 nmask[n]] | [f32 uv[6n] u8 uvmask[n]]   (little endian)
int load_rtwm(rtw_scene* hs, const char* path, uint32_t mat, uint32_t* ntri_out) {
  std::string b;
  if (!read_file(path, b)) return fail(RTW_EIO, "cannot read mesh '%s'", path);
  if (b.size() < 16 || memcmp(b.data(), "RTWM", 4)) return fail(RTW_EIO, "'%s' is not an .rtwm mesh", path);
  uint32_t hdr[3];
  memcpy(hdr, b.data() + 4, 12);
  const uint32_t n = hdr[1], flags = hdr[2];
  size_t need = 16 + (size_t)n * 36 + ((flags & 1) ? (size_t)n * 37 : 0) + ((flags & 2) ? (size_t)n * 25 : 0);
  if (hdr[0] != 1 || b.size() < need) return fail(RTW_EIO, "'%s': bad .rtwm header or size", path);
  const char* p = b.data() + 16;
  std::vector<float> v(9 * (size_t)n), nn, uv;
  std::vector<uint8_t> nm, um;
  memcpy(v.data(), p, 36 * (size_t)n);
  p += 36 * (size_t)n;
  if (flags & 1) {
    nn.resize(9 * (size_t)n);
    nm.resize(n);
    memcpy(nn.data(), p, 36 * (size_t)n);
    p += 36 * (size_t)n;
    memcpy(nm.data(), p, n);
    p += n;
  }
  if (flags & 2) {
    uv.resize(6 * (size_t)n);
    um.resize(n);
    memcpy(uv.data(), p, 24 * (size_t)n);
    p += 24 * (size_t)n;
    memcpy(um.data(), p, n);
  }
  if (int e = rtw_begin_bvh(hs, 0.0f, 1.0f)) return e;
  if (int e = rtw_add_triangles(hs, n, v.data(), (flags & 1) ? nn.data() : nullptr, (flags & 1) ? nm.data() : nullptr,
                                (flags & 2) ? uv.data() : nullptr, (flags & 2) ? um.data() : nullptr, mat)) {
    rtw_end(hs);  // close the group (see rtw_load_wavefront_obj)
    return e;
  }
  if (int e = rtw_end(hs)) return e;
  if (ntri_out) *ntri_out = n;
  return RTW_OK;
}
}  // namespace rtw
