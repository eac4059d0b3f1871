// rtw_device.hpp — flattened scene layout in HBM, shared by the host flattener
// (rtw_flatten.cpp) and the gfx950 kernels (rtw_kernel.hip).  Plain PODs only.
//
// Layout (DESIGN.md §Data layout):
//   nodes   : DevNode[]   BVH2, 64 B per node = both children's boxes + child refs,
//                         so one 64-B fetch (4 x dwordx4) tests two boxes.
//   prims   : DevPrim[]   64 B per leaf primitive, stored in BVH leaf order so a leaf
//                         is a contiguous run; geometry in q0..q2, meta in the last 16 B.
//   always  : uint32[]    primitives tested for every ray (huge boxes, e.g. the
//                         r=1000 ground sphere) instead of polluting the BVH.
//   tshade  : DevTriShade per prim (triangles only filled): vertex normals + uvs, read only for the winner.
//   insts   : DevInst[]   wrapper chains (Translation / YRotation), outer -> inner.
//   mats, texs, texels   : material / texture tables and image data (RGBX8: 4 B per texel).
#pragma once
#include <stdint.h>

namespace rtw {

enum PrimType : uint32_t {
  PT_SPHERE = 0,
  PT_MSPHERE = 1,
  PT_RECT_XY = 2,
  PT_RECT_XZ = 3,
  PT_RECT_YZ = 4,
  PT_TRI = 5,
  PT_MEDIUM = 6,  // ConstantMedium (volumes.rs): boundary sphere / cuboid + density
};

struct alignas(16) DevPrim {
  // sphere : q0 = (cx, cy, cz, r*r), q1 = (0, 0, 0, key bits), q2 = (0, 1, r, RN(1/r)): a moving sphere
  //          that does not move, so sphere-only kernels test both kinds with one 32-B branch-free test
  // msphere: q0 = (c0x, c0y, c0z, r*r), q1 = (c1-c0 xyz, key bits), q2 = (t0, t1, r, RN(1/r)), aux = 1 if
  //          the shutter is [+0, 1] (center_at then needs no division and no q2)
  // rect   : q0 = (a0, a1, b0, b1), q1.x = k
  // tri    : q0 = (ax, ay, az, abx), q1 = (aby, abz, acx, acy), q2 = (acz, nx, ny, nz)
  //          ab = b - a, ac = c - a, n = ab x ac (bit-identical to triangular.rs:101-105)
  // medium : q0 = sphere (cx, cy, cz, r) | cuboid p0 (x, y, z, -), q1 = cuboid p1, q2 = (neg_inv_density,
  //          boundary kind 0 sphere / 1 cuboid); aux = instance id of the wrappers inside the medium
  float q0[4], q1[4], q2[4];
  uint32_t type_inst;  // bits 0..7 PrimType, bits 8..31 instance id (0 = identity)
  uint32_t key;        // global DFS leaf index: the tie-break (later object wins, mod.rs:61-65)
  uint32_t mat;        // material id
  uint32_t aux;        // triangle: index into tshade (= its prim index); medium: inner (boundary) instance id; msphere: unit shutter
};
static_assert(sizeof(DevPrim) == 64, "DevPrim must be 64 B");

// A run of consecutive always-tested prims with one wrapper chain and one PrimType: the list-mode rect loop walks
// these (no per-prim chain check or type dispatch; rtw_kernel.hip trace_rect_list)
struct alignas(16) DevGroup {
  uint32_t first, count, inst, type;
};
// DevGroup::type of a whole Cuboid (rectangular.rs:177-240: xy, xy, xz, xz, yz, yz, one chain) as one run
constexpr uint32_t GK_BOX6 = 16u;
static_assert(sizeof(DevGroup) == 16, "DevGroup must be 16 B");

struct alignas(16) DevNode {
  float b0lo[3], b0hi[3];  // child 0 box
  float b1lo[3], b1hi[3];  // child 1 box
  int32_t c0, c1;          // child: node index (n == 0) or first prim (n > 0)
  uint32_t n0, n1;         // prim count for leaf children, 0 for internal
};
static_assert(sizeof(DevNode) == 64, "DevNode must be 64 B");

// 4-wide BVH node used by the kernel (collapsed from the SAH BVH2), numbered breadth-first.  Planes are stored per axis
// as [lo x4][hi x4] so a lane loads its ray's near and far planes with one dwordx4 each, picking
// lo or hi by the sign of its direction: no min/max sort in the slab test.  Empty slots have an
// inverted box (lo = +inf, hi = -inf), which that formulation always misses.
struct alignas(16) DevNode4 {
  float lo_x[4], hi_x[4], lo_y[4], hi_y[4], lo_z[4], hi_z[4];
  int32_t child[4];  // >= 0: node4 index; < 0: leaf word ~(first_prim << 3 | count)
  // the same children as 16-bit codes for the sorted-push walk of the LDS-node kernels: internal
  // node4 index (< 2^15), leaf 0x8000 | first_prim << 2 | (count - 1) (first < 2^13, count <= 4),
  // 0 = empty slot; valid when Flat::codes16
  uint32_t code[4];
};
static_assert(sizeof(DevNode4) == 128, "DevNode4 must be 128 B");

// The same node in half precision (112 B, built when Flat::codes16): every plane is an f16 OFFSET from the
// node's f16 origin (<= every child's lo), rounded outward (lo down, hi up: the box only grows, culling
// stays conservative), so the precision follows the node's size, not its distance from the world origin.
// Per axis the four children's planes are stored in both orders, [lo x4 | hi x4] and [hi x4 | lo x4], so a
// lane loads its (near, far) planes with ONE 16-B load picked by its direction sign: a visit is 4 loads and
// 64 B (3 plane loads + codes / origin) instead of 7 loads and 112 B.  The kernel evaluates
// t = off * inv + (origin * inv - o * inv) with v_fma_mix_f32 (f16 operands, f32 arithmetic): no conversions.
// Empty slots: lo = +inf, hi = -inf, as in DevNode4.
struct alignas(16) DevNode4h {
  uint16_t x[2][8], y[2][8], z[2][8];  // [0] = lo0..3, hi0..3; [1] = hi0..3, lo0..3 (f16 offsets)
  uint16_t code[4];                    // DevNode4::code (16-bit child codes)
  uint16_t origin[3];                  // f16, normal or zero
  uint16_t pad;
};
static_assert(sizeof(DevNode4h) == 112, "DevNode4h must be 112 B");

struct alignas(16) DevTriShade {
  float n[9];   // vertex normals after defaults (triangular.rs:55)
  float uv[6];  // vertex uvs after defaults (triangular.rs:57-66)
  uint32_t pad;
};
static_assert(sizeof(DevTriShade) == 64, "DevTriShade must be 64 B");

enum InstOp : uint32_t { IO_TRANSLATE = 1, IO_ROTY = 2 };
constexpr int MAX_INST_OPS = 6;
struct alignas(16) DevInst {
  uint32_t nops, pad[3];
  float op[MAX_INST_OPS][4];  // (type, x, y, z) translate  |  (type, sin, cos, 0) rotate_y
};

enum MatType : uint32_t { MT_LAMBERT = 0, MT_METAL = 1, MT_DIELECTRIC = 2, MT_LIGHT = 3, MT_ISOTROPIC = 4 };
struct alignas(16) DevMat {
  uint32_t type, tex, needs_uv, pad;
  float albedo[3];
  float param;  // metal fuzz | dielectric ir
};

enum TexType : uint32_t { TT_SOLID = 0, TT_CHECKER = 1, TT_IMAGE = 2, TT_UVDEBUG = 3, TT_NOISE = 4 };
struct alignas(16) DevTex {
  uint32_t type, odd, even, pad;
  float c[3], freq;          // freq: checker frequency | noise scale
  uint32_t off, w, h, pad2;  // image: texels[off .. off + 3*w*h) | noise: perlins[off]
};

// perlin.rs:8-12 Perlin: 256 gradients (xyz, w unused) and the three permutations of 0..255.
struct alignas(16) DevPerlin {
  float g[256][4];
  uint8_t perm[3][256];
};

// Per leaf primitive (same index as prims[]): its material and, for the common textures, the texture
// values themselves, so that shading needs ONE load once the closest hit is known instead of the
// prim -> material -> texture -> checker-child chain of dependent loads.  32 B.
enum ShadeMode : uint32_t {
  SM_GENERIC = 0,  // read mats[prim.mat] / texs[] (image, noise, uv-debug, nested checkers)
  SM_SOLID = 1,    // SolidColor: a = colour (texture.rs:56-60); Metal: a = albedo
  SM_CHECKER = 2,  // Checker(SolidColor odd, SolidColor even, freq): a = odd, b = even (texture.rs:69-81)
  SM_IMAGE = 3,    // ImageTexture: a = (texel offset, width, height) as bits (image_texture.rs:34-52)
};
struct alignas(16) DevShade {
  uint32_t kind;  // bits 0..7 MatType, bits 8..11 ShadeMode, bit 12 the material reads uv
  float param;    // metal fuzz | dielectric ir | checker frequency (Lambertian / light / isotropic)
  float a[3];     // colour | Metal albedo | Dielectric (1 / ir, r0 at ratio 1 / ir, r0 at ratio ir)
  float b[3];
};
static_assert(sizeof(DevShade) == 32, "DevShade must be 32 B");

// Scene features: the path kernel is instantiated per feature set so a scene only pays (in code
// size and register pressure) for the primitive / wrapper / material / texture kinds it uses.
enum Feature : uint32_t {
  F_SPHERE = 1u << 0,
  F_MSPHERE = 1u << 1,
  F_RECT = 1u << 2,
  F_TRI = 1u << 3,
  F_INST = 1u << 4,     // Translation / YRotation wrappers
  F_UV = 1u << 5,       // a sphere material reads uv (acos / atan2)
  F_IMAGE = 1u << 6,
  F_CHECKER = 1u << 7,
  F_UVDEBUG = 1u << 8,
  F_LAMBERT = 1u << 9,
  F_METAL = 1u << 10,
  F_DIEL = 1u << 11,
  F_LIGHT = 1u << 12,
  F_MEDIUM = 1u << 13,  // ConstantMedium primitives
  F_NOISE = 1u << 14,   // Perlin noise textures
  F_ISO = 1u << 15,     // Isotropic materials
};
// Not a primitive / material kind: some material's texture needs the generic texture walk
// (image, noise, uv-debug, nested checkers; DevShade SM_GENERIC).  Scenes with only solid and
// checker(solid, solid) textures get kernels without it.
constexpr uint32_t F_TEXGEN = 1u << 17;
constexpr uint32_t F_ALL = ((1u << 16) - 1) | F_TEXGEN;
// Kernel-only flag (not a scene feature): the world has no BVH (list mode, rtw_flatten.cpp), so
// the variant compiles without the BVH walk and its registers (higher occupancy).
constexpr uint32_t F_LIST = 1u << 16;
// Kernel variants (the smallest superset of a scene's features is launched): sphere worlds
// (jumpy-balls), rect/instance worlds with solid colours (cornell-box), the same with media
// (smokey-cornell-box), diffuse meshes (cow, monument), and everything.
constexpr uint32_t F_SPHERES = F_SPHERE | F_MSPHERE | F_CHECKER | F_LAMBERT | F_METAL | F_DIEL | F_LIGHT;
constexpr uint32_t F_BOXES = F_RECT | F_INST | F_LAMBERT | F_METAL | F_DIEL | F_LIGHT;
constexpr uint32_t F_SMOKE = F_BOXES | F_MEDIUM | F_ISO;  // smokey-cornell-box
constexpr uint32_t F_MESHES = F_SPHERE | F_RECT | F_TRI | F_INST | F_CHECKER | F_IMAGE | F_LAMBERT | F_LIGHT | F_TEXGEN;

struct DevScene {
  const DevNode4* nodes;
  const DevNode4h* hnodes;  // the half-precision copy (nullptr unless Flat::codes16)
  const DevPrim* prims;
  const uint32_t* always;
  const DevTriShade* tshade;
  const DevInst* insts;
  const DevMat* mats;
  const DevTex* texs;
  const uint8_t* texels;
  const DevPerlin* perlins;
  const DevShade* shade;
  const DevGroup* lgroups;  // the always list as runs of prims of one wrapper chain and one kind, in list order
  uint32_t n_nodes, n_prims, n_always, n_insts;
  uint32_t n_lgroups;
  uint32_t msphere_unit;  // every moving sphere's shutter is [+0, 1]: center_at needs no q2 / division
  uint32_t uni_inst;      // != 0: the scene's only instance, one Translation by uni_off
  float uni_off[3];
  uint32_t rect_fast;     // every rect has |k| < 2^62 and ordered bounds (a0 <= a1, b0 <= b1): the list-mode rect
                          // loop's fast path may divide by reciprocals and test bounds with med3 (trace_rect_list)
  uint32_t bvh_tri;       // every BVH leaf primitive is a triangle of instance tri_inst (the leaf fast path)
  uint32_t tri_inst;
  // 1: the BVH holds sphere tests, and rays from far origins take the far-origin path (DevFar, trace_begin)
  uint32_t far_check;
};

// The far-origin bound (rtw_flatten.cpp far_bound): the BVH's sphere leaves are padded for origins whose farthest
// corner of the BVH box B is within D0 (D(o)² = sum over axes of (|o - mid| + half)² <= d2); a ray from farther
// away first tests B grown by delta(D) = min(q D² + q0, s D + s0) + l D + l0 and, on a hit, walks the tree with
// every box grown by delta(D) (trace_far).  Stored 256 B before the prim table (the kernel derives its address from
// DevScene::prims at each use, so none of it occupies registers across the path loop).
struct alignas(16) DevFar {
  float mid[3], d2;
  float half[3], q;
  float lo[3], q0;
  float hi[3], s;
  float s0, l, l0;
  uint32_t n_bvh;        // BVH primitives (prims[0 .. n_bvh)): the flat pass of trace_far
  uint32_t nodes_back;   // bytes from the node table to the prim table (both in the scene block)
  uint32_t pad[2];
};
static_assert(sizeof(DevFar) == 96, "DevFar must be 96 B");

constexpr uint32_t DEVFAR_BACK = 256;  // prims - DEVFAR_BACK bytes = the DevFar record

// The render counters (DeviceCopy::counters): [0, 32) statistics, then DISP path-id dispensers DISP_STRIDE words
// (128 B) apart (RenderArgs::queue, path_kernel)
constexpr uint32_t DISP = 8;
constexpr uint32_t DISP_STRIDE = 16;
constexpr uint32_t COUNTER_WORDS = 32 + DISP * DISP_STRIDE;

struct DevCamera {
  float origin[3], llc[3], horizontal[3], vertical[3], u[3], v[3];
  float lens_radius, time0, time1;
};

struct RenderArgs {
  DevScene scene;
  DevCamera cam;
  float bg[3];
  uint32_t w, h, spp, max_depth;
  uint32_t tiles_x;           // ceil(w / 8)
  uint32_t slot_base;         // first tile slot of this pass
  uint32_t quota16;           // trace_run returns once quota16/16 of the wave's lanes are done
  uint32_t leaf16;            // postponed leaves are tested once leaf16/16 of the wave's lanes hold one and are stuck
  uint32_t regen_min;         // regenerate once this many lanes are idle (or every lane is)
  uint32_t batch;             // path ids a wave takes from the global queue per atomic
  uint64_t spp_magic;         // UINT64_MAX / spp + 1 (dev::fastdiv; spp >= 2)
  float fw1, fh1;             // (float)(w - 1), (float)(h - 1) (lib.rs:84-85 divisors)
  float rw1, rh1;             // RN(1 / fw1), RN(1 / fh1): the camera divisions by Markstein's correction
  float time_span;            // cam.time1 - cam.time0 in f32 (UniformFloat scale, camera.rs:72)
  uint64_t tiles_x_magic;     // UINT64_MAX / tiles_x + 1 (tiles_x >= 2)
  const uint32_t* tile_ids;   // device array, or nullptr: slot s renders tile tile_first + s * tile_stride
  uint32_t tile_first, tile_stride;  // (a device's round-robin share of the frame without an id table)
  uint32_t packed_out;        // output [slot][64][3] (always with tile_ids); else the full w x h image
  uint64_t seed_hash;         // splitmix64(seed)
  uint64_t n_paths;           // paths in this pass = slots * 64 * spp
  float* sbuf;                // ordered sample buffer: n_paths x (r, g, b) floats, path-major
  float* out;
  unsigned long long* counters;  // [0] rays, [1] node visits, [2] prim tests, [3..8] per type
  unsigned long long* queue;     // the pass's DISP path-id dispensers (DISP_STRIDE words apart)
  uint32_t* err;                 // host-mapped sticky error word: 1 = a traversal guard tripped (DeviceCopy::err_host)
  int32_t* spill;                // traversal stack entries beyond the LDS stack: [depth][lane]
  uint32_t spill_depth;          // entries per lane (0 = the LDS stack covers the tree's bound)
  uint32_t spill_lanes;          // resident lanes of the launch (stride between levels)
};

}  // namespace rtw
