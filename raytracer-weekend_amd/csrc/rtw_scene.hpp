// rtw_scene.hpp — host-side scene graph behind the rtw_* builder calls.
//
// The graph keeps the reference's Hittable tree shape (raytracer_weekend_lib/src/hittable/,
// bvh.rs) so that rtw_scene_dump() can hand the exact hierarchy to the test oracle; the
// flattener (rtw_flatten.cpp) turns it into the device layout of rtw_device.hpp.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_device.hpp"

struct rtw_scene;  // opaque in the C-ABI; defined below as rtw::Scene's holder

namespace rtw {

enum NodeKind : uint32_t {
  NK_LIST,       // Vec<Box<dyn Hittable>>              hittable/mod.rs:57-69
  NK_BVH,        // BvhNode::new(objects, t0, t1)       bvh.rs:19-74 (set semantics)
  NK_TRANSLATE,  // Translation                         transformations.rs:16-47
  NK_ROTY,       // YRotation                           transformations.rs:50-148
  NK_SPHERE,     // Sphere                              spherical.rs:79-104
  NK_MSPHERE,    // MovingSphere                        spherical.rs:106-151
  NK_RECT,       // XY/XZ/YZRectangle                   rectangular.rs:16-166
  NK_CUBOID,     // Cuboid (six rects)                  rectangular.rs:170-245
  NK_TRI,        // Triangle                            triangular.rs:33-149
  NK_MEDIUM,     // ConstantMedium(boundary, density)   volumes.rs:17-83 (f[0] density, mat = Isotropic)
};

struct Node {
  NodeKind kind;
  std::vector<uint32_t> ch;  // children (groups / wrappers)
  float f[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t axis = 0, mat = 0, tri = 0;
  float sin_t = 0.f, cos_t = 1.f;  // YRotation, computed as transformations.rs:60-63
};

struct TexH {
  uint32_t type = TT_SOLID, odd = 0, even = 0;
  float c[3] = {0, 0, 0};
  float freq = 0.f;
  uint32_t w = 0, h = 0;
  std::vector<uint8_t> img;
  std::vector<float> grad;     // noise: 256 x 3 gradients (perlin.rs:16-19)
  std::vector<uint32_t> perm;  // noise: 3 x 256 permutations (perlin.rs:21-23)
};

struct MatH {
  uint32_t type = MT_LAMBERT, tex = 0;
  float albedo[3] = {0, 0, 0};
  float param = 0.f;
};

// Flattened host copy of what goes to every device.
struct Flat {
  std::vector<DevNode> nodes;    // SAH BVH2 (build + self-check)
  std::vector<DevNode4> nodes4;  // what the kernel walks
  uint32_t stack_need = 0;       // worst-case traversal stack entries of nodes4
  bool codes16 = false;          // DevNode4::code holds valid 16-bit child codes (LDS-node kernels)
  uint32_t stack_need4 = 0;      // the same for the sorted-push walk of the LDS-node kernels (window of 4)
  std::vector<DevNode4h> nodes4h;  // nodes4 in half precision (when codes16; rtw_device.hpp)
  std::vector<DevPrim> prims;
  std::vector<DevShade> shade;  // per prim: material + common texture values (rtw_device.hpp)
  std::vector<uint32_t> always;
  std::vector<DevTriShade> tshade;
  std::vector<DevInst> insts;
  std::vector<DevMat> mats;
  std::vector<DevTex> texs;
  std::vector<uint8_t> texels;
  std::vector<DevPerlin> perlins;
  uint32_t depth = 0;
  uint32_t features = 0;  // Feature bits actually used
  uint32_t msphere_unit = 1;  // every moving sphere has the shutter [+0, 1] (DevPrim::aux)
  uint32_t uni_inst = 0;      // the only instance, a single Translation (0 = none such)
  uint32_t rect_fast = 0;     // DevScene::rect_fast
  std::vector<DevGroup> lgroups;  // DevScene::lgroups
  uint32_t bvh_tri = 0;       // every BVH leaf is a triangle of wrapper chain tri_inst (DevScene::bvh_tri)
  uint32_t tri_inst = 0;
  float uni_off[3] = {0, 0, 0};
  float time_lo = 0.f, time_hi = 1.f;  // shutter interval the moving-sphere boxes cover
  // the far-origin bound of the BVH's sphere tests (rtw_flatten.cpp far_bound; DevScene::far_*)
  uint32_t far_check = 0;
  DevFar far{};
  float far_d0 = 0.f;
};

struct DevBuf {  // a grow-only device allocation
  void* p = nullptr;
  size_t cap = 0;
};

struct DeviceCopy {
  int device = -1;  // the logical device the caller names (rtw_render_device, rtw_render_multi's device d)
  int phys = -1;    // the HIP device it lives on: = device, except under rtw_diag_alias_devices (all on 0)
  void* block = nullptr;  // one hipMalloc holding every table
  size_t bytes = 0;
  DevScene scene{};
  unsigned long long* counters = nullptr;  // COUNTER_WORDS x u64: [0..31] stats, then the path-id dispensers
  // host-mapped sticky error word (hipHostMalloc): a path kernel whose traversal guard trips writes 1;
  // the host reads it at the next render call, rtw_render_status, rtw_path_kernel_times and with stats
  uint32_t* err_host = nullptr;
  float* sbuf = nullptr;                   // ordered per-sample radiance (rgb per path)
  uint64_t sbuf_paths = 0;
  int32_t* spill = nullptr;                // traversal-stack overflow (trees deeper than the LDS stack)
  size_t spill_bytes = 0;
  void* kev[64][2] = {};                   // hipEvent_t pairs around path-kernel launches (ring,
                                           // rtw_path_kernel_times)
  uint32_t kev_head = 0, kev_count = 0;
  int grid[2] = {0, 0};                    // resident path_kernel grid (plain, counting) of the
  void* grid_fn[2] = {nullptr, nullptr};   // variant it was computed for (knobs may switch variants)
  // device buffers kept across render calls (grown, never shrunk; freed by release()): a
  // 30-camera animation through rtw_render does no hipMalloc after the first frame
  DevBuf image, tiles, packed, gathered, gather_ids;
  void* ev[2] = {nullptr, nullptr};        // hipEvent_t pair timing rtw_render / multi calls
  void* stream = nullptr;                  // hipStream_t of rtw_render_multi on this device
  void* gev[2] = {nullptr, nullptr};       // hipEvent_t pair around rtw_render_multi's gather (device 0)
};

struct Scene {
  std::vector<TexH> tex;
  std::vector<MatH> mat;
  std::vector<Node> nodes;        // nodes[0] = world list
  std::vector<uint32_t> open{0};  // open-group stack
  std::vector<float> tri_v, tri_n, tri_uv;  // per triangle: 9, 9, 6 floats (raw inputs)
  std::vector<uint8_t> tri_nm, tri_uvm;     // per triangle: normal / uv presence masks
  bool committed = false;
  Flat flat;
  std::vector<DeviceCopy> dev;
  // the last rtw_render_multi call: per-device render ms (path kernel + in-order reduction) and device 0's
  // gather ms (rtw_render_multi_times)
  std::vector<float> multi_ms;
  float multi_gather_ms = 0.0f;
  // rtw_diag_alias_devices: > 0 = the scene's devices are this many logical devices on physical device 0
  int alias_n = 0;
  Scene() { nodes.push_back(Node{NK_LIST, {}}); }
};

// rtw_flatten.cpp
int flatten(Scene& s);
// rtw_scene.cpp
std::string dump_scene(const Scene& s);
// rtw_kernel.hip
int upload(Scene& s, int device);
void release(Scene& s);
DeviceCopy* find_copy(Scene& s, int device);  // device < 0: the first copy
int grow(DevBuf& b, size_t bytes);            // current device; contents not kept
// Which 8x8 tiles a render covers and where they go: slot k renders tile ids[k] (a device array), or
// tile first + k * stride without one; the output is packed [slot][64][3] when `packed` (always with
// ids), else the full w x h image.
struct TileSet {
  const uint32_t* ids = nullptr;
  uint32_t first = 0, stride = 1, n = 0;
  bool packed = false;
};
// enqueue one render (path kernel passes + in-order reductions) on `stream` (hipStream_t) of
// c.device, which must be current
int enqueue_render(Scene& s, DeviceCopy& c, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h,
                   uint32_t spp, uint32_t max_depth, uint64_t seed, const TileSet& tiles, float* d_out,
                   void* stream, uint32_t flags, void* ev0, void* ev1);
// wait for `stream`, read the launch counters and the ev0 -> ev1 time into st
int collect_stats(DeviceCopy& c, void* stream, void* ev0, void* ev1, uint64_t paths, rtw_stats* st);
// RTW_EINVAL (and clears it) if a path kernel on c's device tripped its traversal guard since the last check
int check_guard(DeviceCopy& c);
int enqueue_unpack(uint32_t w, uint32_t h, const uint32_t* d_tiles, uint32_t n_tiles, const float* d_packed,
                   float* d_image, void* stream);

// thread-local error reporting (rtw_capi.cpp)
int fail(int code, const char* fmt, ...);
// A tuning knob's value (RTW_OCC, RTW_BATCH, RTW_LIST_MAX, ...: DESIGN.md §4), or NULL.  The knobs select
// kernel variants and scheduling parameters for A/B measurements; they are read only when RTW_TUNING=1, so a
// process that inherits a stray variable still runs the default (measured-best) kernels.  A knob set without
// the gate is ignored with one warning on stderr (rtw_capi.cpp).
const char* tuning_env(const char* name);

}  // namespace rtw

struct rtw_scene {
  rtw::Scene s;
};
