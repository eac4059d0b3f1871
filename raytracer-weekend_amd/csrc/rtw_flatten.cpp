// rtw_flatten.cpp — turns the reference-shaped Hittable tree into the device layout
// (rtw_device.hpp): one BVH2 over every leaf primitive in world space, each primitive
// tagged with its wrapper chain (instance) and its DFS key.
//
// Why this is exact w.r.t. the reference's nested closest-hit (hittable/mod.rs:57-69):
// every reference set (Vec list, Cuboid sides, BvhNode) returns the closest hit of its
// children and a later child wins an exact tie, and t is the same number in every
// wrapper space (Translation/YRotation do not rescale the ray).  So the world's answer is
// "smallest candidate t over all leaves, ties to the largest DFS key", which is a
// commutative reduction any traversal order reproduces, provided culling never drops a
// leaf whose candidate could win.  Primitives whose box is huge next to the rest (the
// r = 1000 ground sphere, scenes.rs:74-78) are kept out of the BVH and tested for every ray
// ("always" list): it keeps the tree tight.
//
// Culling is conservative because every candidate hit point lies inside its leaf's box as padded here, and
// the kernel's slab test covers [0, best t · (1 + 1e-5) + 1e-5]:
//  * pad_box (1e-4 + 4e-5 · the box's largest |coordinate|) covers the rounding of the slab test, of the
//    wrapper transforms and of the linear primitive tests (rects; triangles hit at a non-grazing angle);
//  * the f32 sphere test (spherical.rs:26-44) is NOT local: hb² - a·c cancels, so a ray whose origin is
//    |oc| from the centre "hits" at points up to R'(|oc|) = sqrt(r² + 37u(|oc|² + r²)) + u|oc| from it
//    (u = 2^-24, the first-order bound derived in DESIGN.md §2; the spurious band grows with |oc|², a ray
//    from inside the r = 1000 ground sphere hits a 0.2 ball 2.5 r from its centre).  far_bound() pads
//    every sphere leaf (and sphere-bounded medium) for origins within D0 of every BVH point (D0 = the
//    diagonal of the BVH's box B: any origin inside B, jumpy-balls' camera too), and the kernel sends
//    rays from farther away (DevScene::far_*, trace_begin) through a walk whose boxes grow by the bound
//    at their own distance, after one test of B grown the same way (most such rays miss it).
#include <math.h>

#include <cmath>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_scene.hpp"

namespace rtw {
namespace {

struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float p[3]) {
    for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], p[a]); hi[a] = fmaxf(hi[a], p[a]); }
  }
  void grow(const Box& b) {
    for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], b.lo[a]); hi[a] = fmaxf(hi[a], b.hi[a]); }
  }
  bool valid() const { return lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2]; }
  float area() const {
    if (!valid()) return 0.f;
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.f * (dx * dy + dy * dz + dz * dx);
  }
  float diag() const {
    if (!valid()) return 0.f;
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return sqrtf(dx * dx + dy * dy + dz * dz);
  }
};

// Conservative padding: covers the rounding of the primitive tests and of the slab test
// (errors scale with coordinate magnitude, ~1e-6 relative for well-conditioned hits).
void pad_box(Box& b) {
  float m = 0.f;
  for (int a = 0; a < 3; ++a) m = fmaxf(m, fmaxf(fabsf(b.lo[a]), fabsf(b.hi[a])));
  float e = 1e-4f + 4e-5f * m;
  for (int a = 0; a < 3; ++a) { b.lo[a] -= e; b.hi[a] += e; }
}

struct Leaf {
  DevPrim p;
  Box wbox;
  float c[3];
};

// ---- the far-origin bound of the sphere test (header comment)
constexpr double U24 = 0x1p-24;
constexpr double KU = 40.0 * U24;  // 37u of the first-order bound, rounded up to cover second-order terms
// R'(D) - r for a sphere of radius r (>= 0) and an origin at most D from its centre: an upper bound
double sphere_reach(double D, double r) {
  const double x = KU * (D * D + r * r);
  const double q = r > 0.0 ? x / (2.0 * r) : INFINITY;  // sqrt(r² + x) - r <= x / 2r, and <= sqrt(x)
  return std::min(q, sqrt(x)) + U24 * D;
}
// the linear terms for an origin D away from a scene whose coordinates are at most M (slab test, wrapper
// transforms, rect hit points: a few roundings of |o| and |p| each)
double linear_reach(double D, double M) { return 16.0 * U24 * (D + M); }
// |r| of a leaf whose test is the quadratic sphere test, or -1
float quad_radius(const DevPrim& p) {
  const uint32_t t = p.type_inst & 0xffu;
  if (t == PT_SPHERE || t == PT_MSPHERE) return fabsf(p.q2[2]);
  if (t == PT_MEDIUM && p.q2[1] == 0.0f) return fabsf(p.q0[3]);  // a sphere boundary
  return -1.0f;
}

// Pads the BVH's sphere leaves for near origins and fills Flat::far_* for the kernel's far-origin walk.
// Knob RTW_FAR_D0 (tuning): D0 as a multiple of B's diagonal.
void far_bound(std::vector<Leaf>& rest, Flat& f) {
  f.far_check = 0;
  Box B;
  float rmin = INFINITY, rmax = 0.0f;
  for (const Leaf& L : rest) {
    B.grow(L.wbox);
    const float r = quad_radius(L.p);
    if (r >= 0.0f) { rmin = std::min(rmin, r); rmax = std::max(rmax, r); }
  }
  if (!(rmin <= rmax) || !B.valid()) return;  // no sphere in the BVH: pad_box's linear bound suffices
  double scale = 1.0;
  if (const char* e = tuning_env("RTW_FAR_D0")) scale = std::min(8.0, std::max(0.05, atof(e)));
  double M = 0.0;
  for (int a = 0; a < 3; ++a) M = std::max(M, (double)std::max(fabsf(B.lo[a]), fabsf(B.hi[a])));
  const double D0 = scale * (double)B.diag();
  // near origins: every sphere centre c lies in B, so |o - c| <= D(o) = the farthest corner of B <= D0
  for (Leaf& L : rest) {
    const float r = quad_radius(L.p);
    if (r < 0.0f) continue;
    const float e = (float)((sphere_reach(D0, r) + linear_reach(D0, M)) * 1.01);
    for (int a = 0; a < 3; ++a) { L.wbox.lo[a] -= e; L.wbox.hi[a] += e; }
  }
  // far origins: delta(D) = min(q D² + q0, s D + s0) + l D + l0 bounds sphere_reach(D, r) + linear_reach(D, M)
  // over r in [rmin, rmax] (KU/2 (D²/r + r) and sqrt(KU (D² + r²)) <= sqrt(KU) (D + r)); 1% up for the
  // kernel's f32 evaluation
  f.far_check = 1;
  DevFar& F = f.far;
  memset(&F, 0, sizeof F);
  for (int a = 0; a < 3; ++a) {
    F.mid[a] = 0.5f * (B.lo[a] + B.hi[a]);
    // half extent rounded up, so |o - mid| + half >= the farthest corner's distance on this axis
    F.half[a] = nextafterf(std::max(B.hi[a] - F.mid[a], F.mid[a] - B.lo[a]), INFINITY);
    F.lo[a] = B.lo[a];
    F.hi[a] = B.hi[a];
  }
  f.far_d0 = (float)D0;
  F.d2 = (float)(D0 * D0 * (1.0 - 1e-5));  // rounded down: an origin near D0 takes the far path
  const double up = 1.01;
  F.q = rmin > 0.0f ? (float)(up * KU / (2.0 * rmin)) : INFINITY;
  F.q0 = (float)(up * KU * rmax / 2.0);
  F.s = (float)(up * sqrt(KU));
  F.s0 = (float)(up * sqrt(KU) * rmax);
  F.l = (float)(up * (16.0 + 1.0) * U24);
  F.l0 = (float)(up * 16.0 * U24 * M);
  F.n_bvh = (uint32_t)rest.size();  // (nodes_back: set at upload)
}

struct Builder {
  const Scene& s;
  Flat& f;
  std::map<std::vector<uint32_t>, uint32_t> inst_of;
  std::vector<Leaf> leaves;
  uint32_t key = 0;
  int err = RTW_OK;

  Builder(const Scene& sc, Flat& fl) : s(sc), f(fl) {}

  uint32_t instance(const std::vector<uint32_t>& chain) {
    if (chain.empty()) return 0;
    auto it = inst_of.find(chain);
    if (it != inst_of.end()) return it->second;
    if (chain.size() > (size_t)MAX_INST_OPS) {
      err = fail(RTW_EINVAL, "wrapper chain deeper than %d", MAX_INST_OPS);
      return 0;
    }
    DevInst in;
    memset(&in, 0, sizeof in);
    in.nops = (uint32_t)chain.size();
    for (size_t k = 0; k < chain.size(); ++k) {
      const Node& n = s.nodes[chain[k]];
      if (n.kind == NK_TRANSLATE) {
        in.op[k][0] = (float)IO_TRANSLATE;
        in.op[k][1] = n.f[0]; in.op[k][2] = n.f[1]; in.op[k][3] = n.f[2];
      } else {
        in.op[k][0] = (float)IO_ROTY;
        in.op[k][1] = n.sin_t; in.op[k][2] = n.cos_t;
      }
    }
    uint32_t id = (uint32_t)f.insts.size();
    f.insts.push_back(in);
    inst_of[chain] = id;
    return id;
  }

  // object-space box -> world box through the wrapper chain (inner -> outer)
  Box to_world(Box b, const std::vector<uint32_t>& chain) {
    pad_box(b);
    for (size_t k = chain.size(); k-- > 0;) {
      const Node& n = s.nodes[chain[k]];
      if (n.kind == NK_TRANSLATE) {
        for (int a = 0; a < 3; ++a) { b.lo[a] += n.f[a]; b.hi[a] += n.f[a]; }
      } else {  // object -> world of YRotation::hit (transformations.rs:137-141)
        Box r;
        for (int q = 0; q < 8; ++q) {
          float x = (q & 1) ? b.hi[0] : b.lo[0], y = (q & 2) ? b.hi[1] : b.lo[1], z = (q & 4) ? b.hi[2] : b.lo[2];
          float p[3] = {n.cos_t * x + n.sin_t * z, y, -n.sin_t * x + n.cos_t * z};
          r.grow(p);
        }
        b = r;
      }
      pad_box(b);
    }
    return b;
  }

  // box_chain: the wrappers between the box's space and the world (default: the prim's chain)
  void emit(DevPrim p, Box local, const std::vector<uint32_t>& chain,
            const std::vector<uint32_t>* box_chain = nullptr) {
    p.type_inst |= instance(chain) << 8;
    p.key = key++;
    Leaf L;
    L.p = p;
    L.wbox = to_world(local, box_chain ? *box_chain : chain);
    for (int a = 0; a < 3; ++a) L.c[a] = 0.5f * (L.wbox.lo[a] + L.wbox.hi[a]);
    leaves.push_back(L);
  }

  void rect(uint32_t axis, float a0, float a1, float b0, float b1, float k, uint32_t mat,
            const std::vector<uint32_t>& chain) {
    DevPrim p;
    memset(&p, 0, sizeof p);
    p.type_inst = PT_RECT_XY + axis;
    p.q0[0] = a0; p.q0[1] = a1; p.q0[2] = b0; p.q0[3] = b1; p.q1[0] = k;
    p.mat = mat;
    Box b;
    float lo[3], hi[3];
    int kax = axis == 0 ? 2 : (axis == 1 ? 1 : 0), aax = axis == 2 ? 1 : 0, bax = axis == 0 ? 1 : 2;
    lo[aax] = fminf(a0, a1); hi[aax] = fmaxf(a0, a1);
    lo[bax] = fminf(b0, b1); hi[bax] = fmaxf(b0, b1);
    lo[kax] = k; hi[kax] = k;
    b.grow(lo); b.grow(hi);
    emit(p, b, chain);
  }

  void walk(uint32_t id, std::vector<uint32_t>& chain) {
    const Node& n = s.nodes[id];
    switch (n.kind) {
      case NK_LIST:
      case NK_BVH:
        for (uint32_t c : n.ch) walk(c, chain);
        return;
      case NK_TRANSLATE:
      case NK_ROTY:
        chain.push_back(id);
        for (uint32_t c : n.ch) walk(c, chain);
        chain.pop_back();
        return;
      case NK_SPHERE: {
        DevPrim p;
        memset(&p, 0, sizeof p);
        p.type_inst = PT_SPHERE;
        // q0 = (c, r * r), q1 = (0, 0, 0, key bits), q2 = (0, 1, r): the layout of a moving sphere
        // with c1 - c0 = 0 over the unit shutter (rtw_device.hpp), so sphere-only kernels test both
        // kinds alike; r * r is the f32 product spherical.rs:29 forms per call
        memcpy(p.q0, n.f, 3 * sizeof(float));
        {
          const volatile float r = n.f[3];
          p.q0[3] = r * r;
        }
        p.q2[0] = 0.0f;
        p.q2[1] = 1.0f;
        p.q2[2] = n.f[3];
        {
          const volatile float r = n.f[3];
          p.q2[3] = 1.0f / r;  // RN(1 / r): the outward normal (p - c) / r by Markstein's correction (kernel)
        }
        p.mat = n.mat;
        float r = fabsf(n.f[3]);  // |r|: spherical.rs:98-103 inverts the box for r < 0
        Box b;
        float lo[3] = {n.f[0] - r, n.f[1] - r, n.f[2] - r}, hi[3] = {n.f[0] + r, n.f[1] + r, n.f[2] + r};
        b.grow(lo); b.grow(hi);
        emit(p, b, chain);
        return;
      }
      case NK_MSPHERE: {
        DevPrim p;
        memset(&p, 0, sizeof p);
        p.type_inst = PT_MSPHERE;
        // q0 = (c0, r * r), q1 = (c1 - c0, r), q2 = (t0, t1): the f32 subtraction and product the
        // reference evaluates per call (spherical.rs:29, :117-123), done once here (same IEEE ops).
        // aux = 1 for the shutter [+0, 1], where (time - t0) / (t1 - t0) is `time` exactly; when every
        // moving sphere has it (Flat::msphere_unit) the test needs q0, q1 and meta only (one round trip)
        memcpy(p.q0, n.f, 3 * sizeof(float));
        p.q0[3] = n.f[8] * n.f[8];
        for (int a = 0; a < 3; ++a) p.q1[a] = n.f[4 + a] - n.f[a];
        p.q2[0] = n.f[3];
        p.q2[1] = n.f[7];
        p.q2[2] = n.f[8];  // r; q1[3] gets the key bits once keys are assigned
        {
          const volatile float r = n.f[8];
          p.q2[3] = 1.0f / r;  // RN(1 / r) for the outward normal
        }
        uint32_t t0_bits;
        memcpy(&t0_bits, &n.f[3], 4);
        p.aux = (t0_bits == 0u && n.f[7] == 1.0f) ? 1u : 0u;
        p.mat = n.mat;
        float r = fabsf(n.f[8]);
        Box b;
        // center_at_time (spherical.rs:117-123) is linear in t: the shutter interval's end
        // points bound it.  The kernel refuses cameras outside [time_lo, time_hi].
        for (float t : {f.time_lo, f.time_hi}) {
          float c[3];
          for (int a = 0; a < 3; ++a) c[a] = n.f[a] + ((t - n.f[3]) / (n.f[7] - n.f[3])) * (n.f[4 + a] - n.f[a]);
          float lo[3] = {c[0] - r, c[1] - r, c[2] - r}, hi[3] = {c[0] + r, c[1] + r, c[2] + r};
          b.grow(lo); b.grow(hi);
        }
        emit(p, b, chain);
        return;
      }
      case NK_RECT:
        rect(n.axis, n.f[0], n.f[1], n.f[2], n.f[3], n.f[4], n.mat, chain);
        return;
      case NK_CUBOID: {  // rectangular.rs:177-234, sides in this order
        const float* p0 = n.f;
        const float* p1 = n.f + 3;
        rect(0, p0[0], p1[0], p0[1], p1[1], p1[2], n.mat, chain);
        rect(0, p0[0], p1[0], p0[1], p1[1], p0[2], n.mat, chain);
        rect(1, p0[0], p1[0], p0[2], p1[2], p1[1], n.mat, chain);
        rect(1, p0[0], p1[0], p0[2], p1[2], p0[1], n.mat, chain);
        rect(2, p0[1], p1[1], p0[2], p1[2], p1[0], n.mat, chain);
        rect(2, p0[1], p1[1], p0[2], p1[2], p0[0], n.mat, chain);
        return;
      }
      case NK_MEDIUM: {  // volumes.rs:17-83: one leaf; the boundary is geometry of the medium
        if (n.ch.size() != 1) { err = fail(RTW_EINVAL, "ConstantMedium needs exactly one boundary object"); return; }
        std::vector<uint32_t> inner;  // wrappers inside the medium, outer -> inner
        uint32_t b = n.ch[0];
        for (int guard = 0; guard < 64; ++guard) {
          const Node& m = s.nodes[b];
          if ((m.kind == NK_TRANSLATE || m.kind == NK_ROTY || m.kind == NK_LIST || m.kind == NK_BVH) && m.ch.size() == 1) {
            if (m.kind == NK_TRANSLATE || m.kind == NK_ROTY) inner.push_back(b);
            b = m.ch[0];
            continue;
          }
          break;
        }
        const Node& bd = s.nodes[b];
        DevPrim p;
        memset(&p, 0, sizeof p);
        p.type_inst = PT_MEDIUM;
        p.q2[0] = -1.0f / n.f[0];  // volumes.rs:25 neg_inv_density
        p.mat = n.mat;
        p.aux = instance(inner);
        Box lb;
        if (bd.kind == NK_SPHERE) {
          memcpy(p.q0, bd.f, 4 * sizeof(float));
          p.q2[1] = 0.0f;
          float r = fabsf(bd.f[3]);
          float lo[3] = {bd.f[0] - r, bd.f[1] - r, bd.f[2] - r}, hi[3] = {bd.f[0] + r, bd.f[1] + r, bd.f[2] + r};
          lb.grow(lo); lb.grow(hi);
        } else if (bd.kind == NK_CUBOID) {
          memcpy(p.q0, bd.f, 3 * sizeof(float));
          memcpy(p.q1, bd.f + 3, 3 * sizeof(float));
          p.q2[1] = 1.0f;
          lb.grow(bd.f); lb.grow(bd.f + 3);
        } else {
          err = fail(RTW_EINVAL, "ConstantMedium boundary must be a Sphere or a Cuboid (optionally translated / "
                                 "rotated) in this build");
          return;
        }
        std::vector<uint32_t> full = chain;
        full.insert(full.end(), inner.begin(), inner.end());
        emit(p, lb, chain, &full);
        return;
      }
      case NK_TRI: {
        const float* v = &s.tri_v[9 * (size_t)n.tri];
        DevPrim p;
        memset(&p, 0, sizeof p);
        p.type_inst = PT_TRI;
        // triangular.rs:101-105: ab = b - a, ac = c - a, n = ab x ac (precomputed, bit-identical)
        float ab[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        float ac[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        float nn[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]};
        float q[12] = {v[0], v[1], v[2], ab[0], ab[1], ab[2], ac[0], ac[1], ac[2], nn[0], nn[1], nn[2]};
        memcpy(p.q0, q, 4 * sizeof(float));
        memcpy(p.q1, q + 4, 4 * sizeof(float));
        memcpy(p.q2, q + 8, 4 * sizeof(float));
        p.mat = n.mat;
        p.aux = (uint32_t)f.tshade.size();
        DevTriShade sh;
        memset(&sh, 0, sizeof sh);
        const float* vn = &s.tri_n[9 * (size_t)n.tri];
        const float* uv = &s.tri_uv[6 * (size_t)n.tri];
        const float defuv[6] = {0, 0, 1, 0, 0, 1};  // triangular.rs:57-61
        uint8_t nm = s.tri_nm[n.tri], um = s.tri_uvm[n.tri];
        for (int k = 0; k < 3; ++k) {
          for (int a = 0; a < 3; ++a) sh.n[3 * k + a] = ((nm >> k) & 1) ? vn[3 * k + a] : nn[a];  // :55
          for (int a = 0; a < 2; ++a) sh.uv[2 * k + a] = ((um >> k) & 1) ? uv[2 * k + a] : defuv[2 * k + a];
        }
        f.tshade.push_back(sh);
        Box b;
        for (int k = 0; k < 3; ++k) b.grow(v + 3 * k);
        emit(p, b, chain);
        return;
      }
    }
  }
};

// ---------------------------------------------------------------- binned SAH BVH2
// Build parameters (tuning knobs RTW_BVH_LEAF 1..7, RTW_BVH_TRAV = SAH cost of a BVH2 traversal step
// relative to one primitive test, RTW_BVH_BINS 4..64)
struct BuildParams {
  int leaf_max = 4;
  float trav = 0.5f;
  int bins = 16;
  uint32_t pair = 2;  // ranges of at most this many prims become leaves without a SAH decision
  BuildParams() {
    if (const char* e = tuning_env("RTW_BVH_PAIR")) pair = (uint32_t)std::min(4, std::max(1, atoi(e)));
    if (const char* e = tuning_env("RTW_BVH_LEAF")) leaf_max = std::min(7, std::max(1, atoi(e)));
    if (const char* e = tuning_env("RTW_BVH_TRAV")) trav = (float)atof(e);
    if (const char* e = tuning_env("RTW_BVH_BINS")) bins = std::min(64, std::max(4, atoi(e)));
  }
};
constexpr int NBINS_MAX = 64;
constexpr uint32_t MAX_DEPTH = 31;  // the kernel's traversal stack holds 32 entries

struct Ref {
  Box box;
  int32_t idx;     // node index (count == 0) or first prim
  uint32_t count;  // prims in leaf
};

struct BvhBuild {
  std::vector<Leaf>& L;
  std::vector<DevNode>& nodes;
  uint32_t median_depth;  // from here on: median splits, so depth <= MAX_DEPTH
  BuildParams P;
  uint32_t max_depth = 0;

  Ref build(uint32_t b, uint32_t e, uint32_t depth) {
    Box box, cbox;
    for (uint32_t k = b; k < e; ++k) { box.grow(L[k].wbox); cbox.grow(L[k].c); }
    uint32_t n = e - b;
    if (depth > max_depth) max_depth = depth;
    if (n <= P.pair) return Ref{box, (int32_t)b, n};

    // choose split
    int best_axis = -1;
    int best_bin = 0;
    float best_cost = INFINITY;
    if (depth < median_depth) {
      for (int a = 0; a < 3; ++a) {
        float lo = cbox.lo[a], hi = cbox.hi[a];
        if (!(hi > lo)) continue;
        Box bb[NBINS_MAX];
        uint32_t cnt[NBINS_MAX] = {0};
        const int NBINS = P.bins;
        float sc = NBINS / (hi - lo);
        for (uint32_t k = b; k < e; ++k) {
          int bi = std::min(NBINS - 1, (int)((L[k].c[a] - lo) * sc));
          cnt[bi]++;
          bb[bi].grow(L[k].wbox);
        }
        Box left[NBINS_MAX];
        uint32_t lc[NBINS_MAX];
        Box acc;
        uint32_t c = 0;
        for (int q = 0; q < NBINS; ++q) { acc.grow(bb[q]); c += cnt[q]; left[q] = acc; lc[q] = c; }
        acc = Box();
        c = 0;
        for (int q = NBINS - 1; q > 0; --q) {
          acc.grow(bb[q]);
          c += cnt[q];
          if (lc[q - 1] == 0 || c == 0) continue;
          float cost = left[q - 1].area() * lc[q - 1] + acc.area() * c;
          if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = q; }
        }
      }
      float leaf_cost = box.area() * n;
      float split_cost = box.area() * P.trav + best_cost;  // traversal step vs prim test
      if (n <= (uint32_t)P.leaf_max && (best_axis < 0 || split_cost >= leaf_cost))
        return Ref{box, (int32_t)b, n};
    }
    uint32_t mid;
    if (best_axis >= 0) {
      const int NBINS = P.bins;
      float lo = cbox.lo[best_axis], sc = NBINS / (cbox.hi[best_axis] - lo);
      auto it = std::partition(L.begin() + b, L.begin() + e, [&](const Leaf& x) {
        return std::min(NBINS - 1, (int)((x.c[best_axis] - lo) * sc)) < best_bin;
      });
      mid = (uint32_t)(it - L.begin());
      if (mid == b || mid == e) best_axis = -1;
    }
    if (best_axis < 0) {  // median split on the widest centroid axis
      int a = 0;
      for (int q = 1; q < 3; ++q)
        if (cbox.hi[q] - cbox.lo[q] > cbox.hi[a] - cbox.lo[a]) a = q;
      mid = b + n / 2;
      std::nth_element(L.begin() + b, L.begin() + mid, L.begin() + e,
                       [a](const Leaf& x, const Leaf& y) { return x.c[a] < y.c[a]; });
    }
    int32_t id = (int32_t)nodes.size();
    nodes.push_back(DevNode{});
    Ref l = build(b, mid, depth + 1);
    Ref r = build(mid, e, depth + 1);
    DevNode& nd = nodes[id];
    for (int a = 0; a < 3; ++a) {
      nd.b0lo[a] = l.box.lo[a]; nd.b0hi[a] = l.box.hi[a];
      nd.b1lo[a] = r.box.lo[a]; nd.b1hi[a] = r.box.hi[a];
    }
    nd.c0 = l.idx; nd.n0 = l.count;
    nd.c1 = r.idx; nd.n1 = r.count;
    return Ref{box, id, 0};
  }
};

// ---------------------------------------------------------------- BVH2 -> BVH4 collapse
// Each 4-wide node absorbs up to two BVH2 levels: starting from a BVH2 node's two children, the
// internal child with the largest surface area is repeatedly replaced by its own two children
// until there are four.  Leaves keep their prim ranges (leaf word ~(first << 3 | count)).
struct Collapse {
  const std::vector<DevNode>& n2;
  std::vector<DevNode4>& out;

  struct C {
    Box box;
    int32_t idx;     // BVH2 node (internal) or first prim (leaf)
    uint32_t count;  // 0 = internal
  };
  static C child(const DevNode& n, int k) {
    C c;
    for (int a = 0; a < 3; ++a) {
      c.box.lo[a] = k ? n.b1lo[a] : n.b0lo[a];
      c.box.hi[a] = k ? n.b1hi[a] : n.b0hi[a];
    }
    c.idx = k ? n.c1 : n.c0;
    c.count = k ? n.n1 : n.n0;
    return c;
  }
  // returns the node4 index; *bound = worst-case stack entries pushed below (and at) this node
  // *bound4: the same for the sorted-push walk of the LDS-node kernels (trace_run, K16), which writes
  // a 4-entry window at the stack top on every visit and walks into the nearest hit child: rows
  // needed = max over root-to-node paths of sum(children - 1) over the ancestors + 4
  int32_t build(int32_t root2, uint32_t* bound, uint32_t* bound4) {
    std::vector<C> ch;
    const DevNode& r = n2[root2];
    ch.push_back(child(r, 0));
    if (r.c1 >= 0 || r.n1) ch.push_back(child(r, 1));
    while (ch.size() < 4) {
      int best = -1;
      float area = -1.f;
      for (size_t k = 0; k < ch.size(); ++k)
        if (ch[k].count == 0 && ch[k].box.area() > area) { area = ch[k].box.area(); best = (int)k; }
      if (best < 0) break;
      const DevNode& m = n2[ch[best].idx];
      C a = child(m, 0);
      ch[best] = a;
      if (m.c1 >= 0 || m.n1) ch.push_back(child(m, 1));
    }
    const int32_t id = (int32_t)out.size();
    DevNode4 nd;
    memset(&nd, 0, sizeof nd);
    for (int k = 0; k < 4; ++k) {
      nd.lo_x[k] = nd.lo_y[k] = nd.lo_z[k] = INFINITY;
      nd.hi_x[k] = nd.hi_y[k] = nd.hi_z[k] = -INFINITY;
    }
    out.push_back(nd);
    uint32_t below = 0, below4 = 0;
    bool inner = false;
    for (size_t k = 0; k < ch.size(); ++k) {
      int32_t word;
      if (ch[k].count) {
        word = (int32_t)~(((uint32_t)ch[k].idx << 3) | ch[k].count);
      } else {
        uint32_t b = 0, b4 = 0;
        word = build(ch[k].idx, &b, &b4);
        below = std::max(below, b);
        below4 = std::max(below4, b4);
        inner = true;
      }
      DevNode4& o = out[id];
      o.lo_x[k] = ch[k].box.lo[0]; o.hi_x[k] = ch[k].box.hi[0];
      o.lo_y[k] = ch[k].box.lo[1]; o.hi_y[k] = ch[k].box.hi[1];
      o.lo_z[k] = ch[k].box.lo[2]; o.hi_z[k] = ch[k].box.hi[2];
      o.child[k] = word;
    }
    // a visit pushes every hit child except the nearest internal one, which it walks into next
    // (trace_run); with no internal child it may push them all
    *bound = inner ? (uint32_t)ch.size() - 1 + below : (uint32_t)ch.size();
    *bound4 = std::max(4u, inner ? (uint32_t)ch.size() - 1 + below4 : 4u);
    return id;
  }
};

// ---- f16 with directed rounding (DevNode4h): binary search over the ordered f16 values
double h2d(uint16_t h) {
  const int e = (h >> 10) & 31, m = h & 1023;
  const double v = e == 0 ? ldexp((double)m, -24) : (e == 31 ? (m ? NAN : INFINITY) : ldexp(1024.0 + m, e - 25));
  return (h & 0x8000) ? -v : v;
}
uint16_t h_of_key(int32_t k) { return k >= 0 ? (uint16_t)k : (uint16_t)(0x8000 | -k); }
// the largest f16 <= x (down) or the smallest f16 >= x (up); -inf / +inf beyond the range
uint16_t h_round(double x, bool up) {
  int32_t lo = -0x7C00, hi = 0x7C00;  // ordered keys of -inf .. +inf
  if (up) {  // smallest key with h2d >= x
    while (lo < hi) {
      const int32_t mid = lo + (hi - lo) / 2;
      if (h2d(h_of_key(mid)) >= x) hi = mid; else lo = mid + 1;
    }
  } else {  // largest key with h2d <= x
    while (lo < hi) {
      const int32_t mid = lo + (hi - lo + 1) / 2;
      if (h2d(h_of_key(mid)) <= x) lo = mid; else hi = mid - 1;
    }
  }
  return h_of_key(lo);
}
bool h_subnormal(uint16_t h) { return ((h >> 10) & 31) == 0 && (h & 1023) != 0; }
// outward-rounded f16 offsets from a normal-or-zero f16 origin: no subnormal operand reaches the kernel.
// false when a child's lower bound is below -65504: the origin would round down to -inf, every offset on
// that axis would be +inf and the planes NaN (the caller then builds no half-precision table)
bool half_node(const DevNode4& n, DevNode4h& o) {
  memset(&o, 0, sizeof o);
  const float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
  const float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
  uint16_t* ax[3] = {&o.x[0][0], &o.y[0][0], &o.z[0][0]};
  for (int a = 0; a < 3; ++a) {
    double mn = INFINITY;
    for (int k = 0; k < 4; ++k)
      if (n.lo_x[k] <= n.hi_x[k]) mn = std::min(mn, (double)lo[a][k]);
    if (mn < -65504.0) return false;
    uint16_t org = mn == INFINITY ? 0 : h_round(mn, false);
    if (h_subnormal(org)) org = (org & 0x8000) ? 0x8400 : 0;  // -2^-14 or +0: still <= mn
    o.origin[a] = org;
    const double od = h2d(org);
    for (int k = 0; k < 4; ++k) {
      uint16_t l = 0x7C00, h = 0xFC00;  // empty slot: +inf, -inf
      if (n.lo_x[k] <= n.hi_x[k]) {
        l = h_round((double)lo[a][k] - od, false);  // >= 0 (od <= lo), rounded down
        h = h_round((double)hi[a][k] - od, true);   // rounded up (+inf past 65504: conservative)
        if (h_subnormal(l)) l = 0;
        if (h_subnormal(h)) h = 0x0400;  // 2^-14
      }
      ax[a][k] = l;
      ax[a][4 + k] = h;
      ax[a][8 + k] = h;
      ax[a][12 + k] = l;
    }
  }
  for (int k = 0; k < 4; ++k) o.code[k] = (uint16_t)n.code[k];
  return true;
}

bool texture_reads_uv(const Scene& s, uint32_t t, int guard = 0) {
  if (guard > 64) return false;
  const TexH& x = s.tex[t];
  if (x.type == TT_IMAGE || x.type == TT_UVDEBUG) return true;
  if (x.type == TT_CHECKER) return texture_reads_uv(s, x.odd, guard + 1) || texture_reads_uv(s, x.even, guard + 1);
  return false;
}

}  // namespace

int flatten(Scene& s) {
  Flat& f = s.flat;
  f = Flat();
  // tables
  for (const MatH& m : s.mat) {
    DevMat d;
    memset(&d, 0, sizeof d);
    d.type = m.type; d.tex = m.tex; d.param = m.param;
    memcpy(d.albedo, m.albedo, sizeof d.albedo);
    d.needs_uv = (m.type == MT_LAMBERT || m.type == MT_LIGHT || m.type == MT_ISOTROPIC) ? texture_reads_uv(s, m.tex) : 0;
    f.mats.push_back(d);
  }
  for (const TexH& t : s.tex) {
    DevTex d;
    memset(&d, 0, sizeof d);
    d.type = t.type; d.odd = t.odd; d.even = t.even; d.freq = t.freq;
    memcpy(d.c, t.c, sizeof d.c);
    if (t.type == TT_IMAGE) {
      // RGBX8 on the device: one aligned 4-byte load per lookup instead of three byte loads
      if (f.texels.size() + 4ull * t.w * t.h >= (1ull << 32)) return fail(RTW_EINVAL, "image textures exceed 4 GiB");
      d.off = (uint32_t)f.texels.size();
      d.w = t.w; d.h = t.h;
      const size_t n = (size_t)t.w * t.h;
      f.texels.resize(f.texels.size() + 4 * n, 0);
      uint8_t* o = f.texels.data() + d.off;
      for (size_t q = 0; q < n; ++q) memcpy(o + 4 * q, t.img.data() + 3 * q, 3);
    }
    if (t.type == TT_NOISE) {
      d.off = (uint32_t)f.perlins.size();
      DevPerlin P;
      memset(&P, 0, sizeof P);
      for (int k = 0; k < 256; ++k) {
        for (int a = 0; a < 3; ++a) P.g[k][a] = t.grad[3 * k + a];
        for (int a = 0; a < 3; ++a) P.perm[a][k] = (uint8_t)t.perm[256 * a + k];
      }
      f.perlins.push_back(P);
    }
    f.texs.push_back(d);
  }
  if (f.texels.empty()) f.texels.resize(4, 0);
  if (f.perlins.empty()) f.perlins.resize(1);
  if (f.mats.empty()) f.mats.push_back(DevMat{});
  if (f.texs.empty()) f.texs.push_back(DevTex{});

  DevInst ident;
  memset(&ident, 0, sizeof ident);
  f.insts.push_back(ident);

  Builder B(s, f);
  std::vector<uint32_t> chain;
  B.walk(0, chain);
  if (B.err) return B.err;
  if (B.leaves.size() >= (1u << 31)) return fail(RTW_EINVAL, "too many primitives");

  // split off huge primitives (tested for every ray)
  std::vector<Leaf> huge, rest;
  // list mode: a world of at most list_max primitives skips the BVH and every ray tests all of
  // them, as the reference's flat list does (hittable/mod.rs:57-69).  The loop index is
  // wave-uniform, so every lane tests the same primitive (scalar loads, no divergence): on
  // MI355X cornell-box (18 rects) renders 23% faster than through its 4-node BVH4 (14.6k ->
  // 17.9k Mrays/s).  Tuning knob RTW_LIST_MAX (0 = always build the BVH).
  uint32_t list_max = 32;
  if (const char* e = tuning_env("RTW_LIST_MAX")) list_max = (uint32_t)std::min(64, std::max(0, atoi(e)));
  if (B.leaves.size() <= list_max) {
    huge = B.leaves;
  } else if (B.leaves.size() > 16) {
    std::vector<float> d;
    for (const Leaf& L : B.leaves) d.push_back(L.wbox.diag());
    std::vector<float> sorted = d;
    size_t q = (size_t)(0.95 * (sorted.size() - 1));
    std::nth_element(sorted.begin(), sorted.begin() + q, sorted.end());
    float thr = 20.f * sorted[q];
    size_t nh = 0;
    for (float x : d) nh += x > thr;
    for (size_t k = 0; k < B.leaves.size(); ++k)
      ((nh <= 8 && d[k] > thr) ? huge : rest).push_back(B.leaves[k]);
  } else {
    rest = B.leaves;
  }

  // Triangle meshes: when the BVH part is all triangles of ONE wrapper chain but for a few other
  // primitives (the cow's light rect), those few join the always-tested list, so every BVH leaf is a
  // triangle of that chain (Flat::bvh_tri): the kernel's leaf test then skips the type dispatch and the
  // per-test wrapper transform, and loads 3 x 16 B instead of 4 (the tie key only on a candidate hit).
  // Which leaves are tested where never changes the answer (closest t, ties to the larger key).
  {
    size_t ntri = 0;
    uint32_t inst = UINT32_MAX;
    bool one_inst = true;
    for (const Leaf& L : rest)
      if ((L.p.type_inst & 0xffu) == PT_TRI) {
        ++ntri;
        const uint32_t i = L.p.type_inst >> 8;
        if (inst == UINT32_MAX) inst = i;
        one_inst = one_inst && i == inst;
      }
    const char* knob = tuning_env("RTW_TRI_LEAF");  // 0 = keep the mixed BVH and the generic leaf test
    if ((!knob || atoi(knob)) && ntri > 16 && one_inst && rest.size() - ntri <= 4 &&
        huge.size() + (rest.size() - ntri) <= 8) {
      std::vector<Leaf> tris;
      for (const Leaf& L : rest) ((L.p.type_inst & 0xffu) == PT_TRI ? tris : huge).push_back(L);
      rest.swap(tris);
      f.bvh_tri = 1;
      f.tri_inst = inst;
    }
  }
  far_bound(rest, f);  // sphere leaves padded for near origins, the far-origin walk's bound (header)
  if (!rest.empty()) {
    uint32_t lg = 0;
    while ((1ull << lg) < rest.size()) ++lg;
    BvhBuild bb{rest, f.nodes, lg + 4 < MAX_DEPTH ? MAX_DEPTH - lg - 1 : 3};
    Ref root = bb.build(0, (uint32_t)rest.size(), 0);
    if (root.count > 0) {  // whole set is one leaf: wrap it in a root node
      DevNode nd;
      for (int a = 0; a < 3; ++a) {
        nd.b0lo[a] = root.box.lo[a]; nd.b0hi[a] = root.box.hi[a];
        nd.b1lo[a] = INFINITY; nd.b1hi[a] = -INFINITY;
      }
      nd.c0 = root.idx; nd.n0 = root.count;
      nd.c1 = -1; nd.n1 = 0;  // no second child (the kernel tests c1 >= 0)
      f.nodes.push_back(nd);
    }
    f.depth = bb.max_depth;
  }
  for (const Leaf& L : rest) f.prims.push_back(L.p);
  for (const Leaf& L : huge) {  // the kernels rely on this: always[k] = prims.size() - always.size() + k
    f.always.push_back((uint32_t)f.prims.size());
    f.prims.push_back(L.p);
  }
  if (f.depth > MAX_DEPTH) return fail(RTW_EINVAL, "BVH deeper than the traversal stack (%u)", f.depth);
  // the list-mode rect loop (rtw_kernel.hip trace_rect_list) accepts t <= best: a later prim of the list must
  // have the larger DFS key, which holds because list mode keeps the leaves in walk (= key) order
  if (f.nodes.empty())
    for (size_t k = 1; k < f.always.size(); ++k)
      if (!(f.prims[f.always[k]].key > f.prims[f.always[k - 1]].key))
        return fail(RTW_EINVAL, "internal: list-mode prims out of key order");
  // triangle shading data re-indexed by prim (tshade[k] belongs to prims[k]): the winner's
  // normals / uvs load straight from the hit's prim index, beside its geometry
  if (!f.tshade.empty()) {
    std::vector<DevTriShade> by_prim(f.prims.size());
    memset(by_prim.data(), 0, by_prim.size() * sizeof(DevTriShade));
    for (size_t k = 0; k < f.prims.size(); ++k)
      if ((f.prims[k].type_inst & 0xffu) == PT_TRI) {
        by_prim[k] = f.tshade[f.prims[k].aux];
        f.prims[k].aux = (uint32_t)k;
      }
    f.tshade.swap(by_prim);
  }
  // the list-mode rect loop's fast path (rtw_kernel.hip trace_rect_list) divides by Markstein's correction, exact
  // where |k - o| < 2^64: |o| < 2^62 per lane (checked by the kernel) and |k| < 2^62 for every rect plane (here);
  // and it tests the bounds as med3(x, a0, a1) == x, the reference's !(x < a0 || x > a1) for finite x when
  // a0 <= a1 (here; NaN bounds fail it too)
  f.rect_fast = 1;
  for (const DevPrim& p : f.prims) {
    const uint32_t t = p.type_inst & 0xffu;
    // (finite bounds too: x = o + t d can reach +-inf, and med3(inf, a0, inf) - inf is NaN, which the one-compare
    // accept would then have to lose through fmaxf)
    if ((t == PT_RECT_XY || t == PT_RECT_XZ || t == PT_RECT_YZ) &&
        !(fabsf(p.q1[0]) < 0x1p62f && p.q0[0] <= p.q0[1] && p.q0[2] <= p.q0[3] && std::isfinite(p.q0[0]) &&
          std::isfinite(p.q0[1]) && std::isfinite(p.q0[2]) && std::isfinite(p.q0[3])))
      f.rect_fast = 0;
  }
  // the always list as runs of one wrapper chain and one kind (DevScene::lgroups), in list order
  for (size_t k = 0; k < f.always.size(); ++k) {
    const DevPrim& p = f.prims[f.always[k]];
    const uint32_t inst = p.type_inst >> 8, type = p.type_inst & 0xffu;
    if (!f.lgroups.empty() && f.lgroups.back().inst == inst && f.lgroups.back().type == type &&
        f.lgroups.back().first + f.lgroups.back().count == f.always[k])
      ++f.lgroups.back().count;
    else
      f.lgroups.push_back(DevGroup{f.always[k], 1u, inst, type});
  }
  {  // a Cuboid's three pair runs as one (GK_BOX6): one dispatch in the kernel's run loop instead of three
    std::vector<DevGroup> g2;
    for (size_t g = 0; g < f.lgroups.size(); ++g) {
      const DevGroup& a = f.lgroups[g];
      if (g + 2 < f.lgroups.size()) {
        const DevGroup &b = f.lgroups[g + 1], &c = f.lgroups[g + 2];
        if (a.type == PT_RECT_XY && b.type == PT_RECT_XZ && c.type == PT_RECT_YZ && a.count == 2u && b.count == 2u &&
            c.count == 2u && a.inst == b.inst && b.inst == c.inst && b.first == a.first + 2u && c.first == b.first + 2u) {
          g2.push_back(DevGroup{a.first, 6u, a.inst, GK_BOX6});
          g += 2;
          continue;
        }
      }
      g2.push_back(a);
    }
    f.lgroups.swap(g2);
  }
  // spheres carry their DFS key in q1[3] too (the sphere-only kernels' 32-B test, rtw_device.hpp)
  for (DevPrim& p : f.prims) {
    const uint32_t t = p.type_inst & 0xffu;
    if (t == PT_SPHERE || t == PT_MSPHERE) memcpy(&p.q1[3], &p.key, sizeof p.key);
  }
  // shading records (one per prim, same order)
  for (const DevPrim& p : f.prims) {
    const DevMat& m = f.mats[p.mat];
    DevShade d;
    memset(&d, 0, sizeof d);
    uint32_t mode = SM_GENERIC;
    if (m.type == MT_METAL) {
      mode = SM_SOLID;
      memcpy(d.a, m.albedo, sizeof d.a);
      d.param = m.param;
    } else if (m.type == MT_DIELECTRIC) {
      mode = SM_SOLID;  // attenuation (1, 1, 1), no texture
      d.param = m.param;
      // material.rs:120 (1.0 / ir) and :108-112 (Schlick r0) for both refraction ratios: the kernel's
      // f32 operations, evaluated once here (IEEE f32 on the host as on the device)
      const volatile float one = 1.0f;
      auto r0 = [&](float ri) {
        const float x = (one - ri) / (one + ri);
        return x * x;
      };
      d.a[0] = one / m.param;
      d.a[1] = r0(d.a[0]);
      d.a[2] = r0(m.param);
    } else {  // Lambertian, DiffuseLight, Isotropic: a texture
      const DevTex& t = f.texs[m.tex];
      if (t.type == TT_SOLID) {
        mode = SM_SOLID;
        memcpy(d.a, t.c, sizeof d.a);
      } else if (t.type == TT_CHECKER && f.texs[t.odd].type == TT_SOLID && f.texs[t.even].type == TT_SOLID) {
        mode = SM_CHECKER;
        memcpy(d.a, f.texs[t.odd].c, sizeof d.a);
        memcpy(d.b, f.texs[t.even].c, sizeof d.b);
        d.param = t.freq;
      } else if (t.type == TT_IMAGE) {  // the texel lookup needs no material / texture record loads
        mode = SM_IMAGE;
        const uint32_t img[3] = {t.off, t.w, t.h};
        memcpy(d.a, img, sizeof d.a);
      }
    }
    d.kind = m.type | (mode << 8) | (m.needs_uv ? 1u << 12 : 0u);
    f.shade.push_back(d);
    if (mode == SM_GENERIC) f.features |= F_TEXGEN;
  }
  // 4-wide tree for the kernel
  if (!f.nodes.empty()) {
    if (rest.size() >= (1u << 28)) return fail(RTW_EINVAL, "too many BVH primitives for leaf words");
    Collapse col{f.nodes, f.nodes4};
    uint32_t bound = 0, bound4 = 0;
    col.build(0, &bound, &bound4);
    f.stack_need4 = bound4;
    if (f.nodes4.size() >= (1u << 25)) return fail(RTW_EINVAL, "BVH4 too large for 32-bit node offsets");
    f.stack_need = bound;  // entries beyond the kernel's LDS stack spill to a per-lane HBM area
    if (f.stack_need > 4096) return fail(RTW_EINVAL, "BVH4 stack bound %u is unreasonable", f.stack_need);
    // self-check: every node4 reached once, every BVH prim covered once
    std::vector<uint8_t> seen4(f.nodes4.size(), 0), seenp(rest.size(), 0);
    std::vector<int32_t> todo{0};
    seen4[0] = 1;
    while (!todo.empty()) {
      const DevNode4 nd = f.nodes4[todo.back()];
      todo.pop_back();
      for (int k = 0; k < 4; ++k) {
        if (nd.lo_x[k] > nd.hi_x[k]) continue;  // empty slot
        const int32_t w = nd.child[k];
        if (w >= 0) {
          if ((size_t)w >= f.nodes4.size() || seen4[w]++) return fail(RTW_EINVAL, "BVH4 node cycle/range");
          todo.push_back(w);
        } else {
          const uint32_t v = ~(uint32_t)w, first = v >> 3, cnt = v & 7u;
          if (!cnt || (size_t)first + cnt > rest.size()) return fail(RTW_EINVAL, "BVH4 leaf out of range");
          for (uint32_t q = 0; q < cnt; ++q)
            if (seenp[first + q]++) return fail(RTW_EINVAL, "BVH4 prim referenced twice");
        }
      }
    }
    for (uint8_t x : seenp)
      if (!x) return fail(RTW_EINVAL, "BVH4 misses a primitive");
    // Breadth-first node numbering: the nodes every ray visits (the top levels) come first, so a
    // kernel that keeps only the first K node4s in LDS caches the K most visited ones.  Renumbering
    // never changes the answer (closest hit over the leaves not culled).
    {
      std::vector<int32_t> order{0}, renum(f.nodes4.size(), -1);
      renum[0] = 0;
      for (size_t q = 0; q < order.size(); ++q) {
        const DevNode4& nd = f.nodes4[order[q]];
        for (int k = 0; k < 4; ++k) {
          if (nd.lo_x[k] > nd.hi_x[k] || nd.child[k] < 0) continue;
          renum[nd.child[k]] = (int32_t)order.size();
          order.push_back(nd.child[k]);
        }
      }
      std::vector<DevNode4> bfs(order.size());
      for (size_t q = 0; q < order.size(); ++q) {
        bfs[q] = f.nodes4[order[q]];
        for (int k = 0; k < 4; ++k)
          if (bfs[q].lo_x[k] <= bfs[q].hi_x[k] && bfs[q].child[k] >= 0) bfs[q].child[k] = renum[bfs[q].child[k]];
      }
      f.nodes4.swap(bfs);
    }
    // 16-bit child codes of the sorted-push walk (DevNode4::code): possible when node4 indices fit
    // 15 bits and every leaf has <= 4 prims starting below 8192
    f.codes16 = f.nodes4.size() < 0x8000u;
    for (DevNode4& nd : f.nodes4)
      for (int k = 0; k < 4; ++k) {
        nd.code[k] = 0;
        if (nd.lo_x[k] > nd.hi_x[k]) continue;  // empty slot: 0, its inverted box never hits
        const int32_t w = nd.child[k];
        if (w >= 0) {
          nd.code[k] = (uint32_t)w;
        } else {
          const uint32_t v = ~(uint32_t)w, first = v >> 3, cnt = v & 7u;
          if (cnt > 4u || first >= 0x2000u) f.codes16 = false;
          nd.code[k] = 0x8000u | ((first & 0x1FFFu) << 2) | ((cnt - 1u) & 3u);
        }
      }
    if (f.codes16) {
      f.nodes4h.resize(f.nodes4.size());
      for (size_t q = 0; q < f.nodes4.size(); ++q)
        if (!half_node(f.nodes4[q], f.nodes4h[q])) {  // bounds beyond f16: the f32 table only
          f.nodes4h.clear();
          break;
        }
    }
  }
  // feature set (selects the specialised kernel)
  uint32_t F = 0;
  // one translate-only wrapper for every instanced prim (cow, monument: the mesh under one
  // Translation): the kernel subtracts its kernel-uniform offset instead of loading the chain
  f.uni_inst = 0;
  if (f.insts.size() == 2 && f.insts[1].nops == 1 && f.insts[1].op[0][0] == (float)IO_TRANSLATE) {
    f.uni_inst = 1;
    for (int a = 0; a < 3; ++a) f.uni_off[a] = f.insts[1].op[0][1 + a];
  }
  f.msphere_unit = 1;
  for (const DevPrim& p : f.prims)
    if ((p.type_inst & 0xffu) == PT_MSPHERE && !p.aux) f.msphere_unit = 0;
  for (const DevPrim& p : f.prims) {
    const uint32_t t = p.type_inst & 0xffu;
    F |= t == PT_SPHERE ? F_SPHERE : t == PT_MSPHERE ? F_MSPHERE : t == PT_TRI ? F_TRI : t == PT_MEDIUM ? F_MEDIUM : F_RECT;
    if ((p.type_inst >> 8) || (t == PT_MEDIUM && p.aux)) F |= F_INST;
    if ((t == PT_SPHERE || t == PT_MSPHERE) && f.mats[p.mat].needs_uv) F |= F_UV;
  }
  for (const DevMat& m : f.mats)
    F |= m.type == MT_LAMBERT ? F_LAMBERT : m.type == MT_METAL ? F_METAL : m.type == MT_DIELECTRIC ? F_DIEL :
         m.type == MT_ISOTROPIC ? F_ISO : F_LIGHT;
  for (const DevTex& t : f.texs)
    F |= t.type == TT_CHECKER ? F_CHECKER : t.type == TT_IMAGE ? F_IMAGE : t.type == TT_UVDEBUG ? F_UVDEBUG :
         t.type == TT_NOISE ? F_NOISE : 0u;
  f.features |= F;
  // structural self-check: every internal node reached exactly once from the root, every
  // leaf range inside the BVH part of prims[], every BVH prim covered exactly once
  if (!f.nodes.empty()) {
    std::vector<uint8_t> seen_node(f.nodes.size(), 0), seen_prim(rest.size(), 0);
    std::vector<int32_t> todo{0};
    seen_node[0] = 1;
    while (!todo.empty()) {
      const DevNode nd = f.nodes[todo.back()];
      todo.pop_back();
      const int32_t c[2] = {nd.c0, nd.c1};
      const uint32_t n[2] = {nd.n0, nd.n1};
      for (int k = 0; k < 2; ++k) {
        if (c[k] < 0 && n[k] == 0) continue;  // absent child
        if (n[k]) {
          if (c[k] < 0 || (size_t)c[k] + n[k] > rest.size()) return fail(RTW_EINVAL, "BVH leaf out of range");
          for (uint32_t q = 0; q < n[k]; ++q)
            if (seen_prim[c[k] + q]++) return fail(RTW_EINVAL, "BVH prim referenced twice");
        } else {
          if ((size_t)c[k] >= f.nodes.size() || seen_node[c[k]]++) return fail(RTW_EINVAL, "BVH node cycle/range");
          todo.push_back(c[k]);
        }
      }
    }
    for (uint8_t x : seen_prim)
      if (!x) return fail(RTW_EINVAL, "BVH misses a primitive");
  }
  return RTW_OK;
}

}  // namespace rtw
