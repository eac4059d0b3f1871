// rtw_multi.cpp — Raytracer::render() over the GPUs of one node from ONE host thread.
//
// The reference's only parallelism is Rayon over the pixels of a frame (raytracer_weekend_lib/src/
// lib.rs:57-76).  Here the frame's 8x8 pixel tiles are dealt round-robin to n_gpus devices (tile k ->
// device k mod n; rtw_tile_partition), every device renders its tiles into a packed buffer on its
// own stream with its own copy of the scene (rtw_scene_commit uploads one per device), and one RCCL
// gather over xGMI — a grouped ncclSend from every device to device 0 / ncclRecv on device 0 (RCCL
// has no Gather collective) — brings the packed tiles to device 0, which scatters them into the
// frame and copies it to the host.  Pixels depend only on (seed, j, i, sample), so the frame is
// bit-identical to rtw_render's for every n_gpus.
//
// RCCL is opened at the first render over more than one device (dlopen of librccl.so.1, or the file
// named by RTW_RCCL_LIB), so the rest of the library -- rtw_render_multi(n_gpus = 1) included -- does
// not depend on it.  Under rtw_diag_alias_devices (a test hook) the n devices are logical devices on
// physical device 0, so that this n > 1 path -- per-device streams, sample and packed buffers, the grouped
// send/recv, the gather offsets, the unpack -- runs on a one-GPU box with the loopback RCCL stand-in of
// tests/loopback_rccl (real RCCL refuses a clique whose ranks share a GPU).  The loader and the communicator cache are guarded by one mutex, and every use of a
// clique's communicators (ncclGroupStart .. ncclGroupEnd) by that clique's own mutex, so host threads may
// call rtw_render_multi concurrently on different scenes: RCCL communicators are not thread-safe, and two
// interleaved grouped send/recv sequences on the same communicators could deadlock.
#include <dlfcn.h>
#include <stdlib.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rtw.h"
#include "rtw_scene.hpp"

namespace rtw {
namespace {

struct Rccl {
  std::string path;  // what was opened ("" = the default search)
  void* h = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

std::mutex& rccl_mutex() {
  static std::mutex m;
  return m;
}

// The RCCL library to use: librccl.so.1, or the file RTW_RCCL_LIB names (another RCCL build; a missing file in
// tests; the loopback stand-in of tests/loopback_rccl for the one-GPU rehearsal).  Each library is opened once
// and kept (communicators made by it stay valid); callers hold rccl_mutex().  NULL if it cannot be loaded.
Rccl* rccl() {
  static std::vector<std::unique_ptr<Rccl>> libs;
  const char* want = getenv("RTW_RCCL_LIB");
  const std::string path = want ? want : "";
  for (auto& r : libs)
    if (r->path == path) return r->h ? r.get() : nullptr;
  auto r = std::make_unique<Rccl>();
  r->path = path;
  if (want) {
    r->h = dlopen(want, RTLD_NOW | RTLD_LOCAL);
  } else {
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      r->h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r->h) break;
    }
  }
  if (r->h) {
    auto sym = [&](auto& fn, const char* n) { fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(r->h, n)); };
    sym(r->comm_init_all, "ncclCommInitAll");
    sym(r->comm_destroy, "ncclCommDestroy");
    sym(r->send, "ncclSend");
    sym(r->recv, "ncclRecv");
    sym(r->group_start, "ncclGroupStart");
    sym(r->group_end, "ncclGroupEnd");
    sym(r->error_string, "ncclGetErrorString");
    if (!r->comm_init_all || !r->comm_destroy || !r->send || !r->recv || !r->group_start || !r->group_end ||
        !r->error_string) {
      dlclose(r->h);
      r->h = nullptr;
    }
  }
  libs.push_back(std::move(r));
  return libs.back()->h ? libs.back().get() : nullptr;
}

// one communicator clique per (library, HIP device list), kept for the process (ncclCommInitAll is slow); each
// behind its own allocation, so a pointer handed out stays valid when the cache grows
struct Clique {
  const Rccl* lib = nullptr;
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  std::mutex mu;  // held from ncclGroupStart through ncclGroupEnd of one gather
};
std::vector<std::unique_ptr<Clique>>& cliques() {  // callers hold rccl_mutex()
  static std::vector<std::unique_ptr<Clique>> c;
  return c;
}

#define HIPOK(x, what)                                                              \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail(RTW_ENODEV, "%s: %s", what, hipGetErrorString(e_)); \
  } while (0)

// rank d of the clique is the communicator of the HIP device devs[d] (logical device d of the render)
int get_clique(const std::vector<int>& devs, Clique** out) {
  std::lock_guard<std::mutex> lock(rccl_mutex());
  const Rccl* r = rccl();
  if (!r) return fail(RTW_ENODEV, "%s not loadable (a gather over %zu devices needs RCCL)",
                      getenv("RTW_RCCL_LIB") ? getenv("RTW_RCCL_LIB") : "librccl.so.1", devs.size());
  for (auto& c : cliques())
    if (c->lib == r && c->devs == devs) {
      *out = c.get();
      return RTW_OK;
    }
  auto c = std::make_unique<Clique>();
  c->lib = r;
  c->devs = devs;
  c->comms.resize(devs.size());
  const ncclResult_t e = r->comm_init_all(c->comms.data(), (int)devs.size(), devs.data());
  if (e != ncclSuccess) return fail(RTW_ENODEV, "ncclCommInitAll: %s", r->error_string(e));
  *out = c.get();
  cliques().push_back(std::move(c));
  return RTW_OK;
}

}  // namespace
}  // namespace rtw

using namespace rtw;

extern "C" {

int rtw_tile_partition(uint32_t w, uint32_t h, uint32_t n_parts, uint32_t part, uint32_t* ids, uint32_t cap,
                       uint32_t* n_ids) {
  if (!n_ids || n_parts == 0 || part >= n_parts || (cap && !ids)) return fail(RTW_EINVAL, "bad arguments");
  const uint32_t nt = ((w + 7u) / 8u) * ((h + 7u) / 8u), per = (nt + n_parts - 1) / n_parts;
  uint32_t k = 0;
  for (uint32_t t = part; t < nt; t += n_parts, ++k)
    if (k < cap) ids[k] = t;
  for (uint32_t q = k; q < per && q < cap; ++q) ids[q] = nt;  // padding up to the common size
  *n_ids = k;
  return RTW_OK;
}

int rtw_render_multi(rtw_scene* s, int n_gpus, const rtw_camera* cam, const float bg[3], uint32_t w, uint32_t h,
                     uint32_t spp, uint32_t max_depth, uint64_t seed, float* out, rtw_stats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  if (!s || !cam || !bg || !out) return fail(RTW_EINVAL, "NULL argument");
  if (!s->s.committed) return fail(RTW_ESTATE, "scene not committed");
  if (w < 2 || h < 2) return fail(RTW_EINVAL, "image must be at least 2x2 (lib.rs:84-85 divides by w-1, h-1)");
  s->s.multi_ms.clear();  //  a failed call leaves no stale timings behind
  s->s.multi_gather_ms = 0.0f;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RTW_ENODEV, "no HIP device visible");
  if (s->s.alias_n > 0) ndev = s->s.alias_n;  // logical devices on physical device 0 (rtw_diag_alias_devices)
  const int n = n_gpus <= 0 ? ndev : n_gpus;
  if (n > ndev) return fail(RTW_EINVAL, "n_gpus %d > visible devices %d", n_gpus, ndev);
  std::vector<DeviceCopy*> cp(n);
  for (int d = 0; d < n; ++d) {
    cp[d] = nullptr;
    for (DeviceCopy& c : s->s.dev)
      if (c.device == d) cp[d] = &c;
    if (!cp[d]) return fail(RTW_ENODEV, "scene was not committed to device %d (commit with device = -1)", d);
  }
  int prev = 0;
  hipGetDevice(&prev);
  struct Restore {
    int d;
    ~Restore() { hipSetDevice(d); }
  } restore{prev};
  std::vector<hipEvent_t> e0(n), e1(n);
  for (int d = 0; d < n; ++d) {
    DeviceCopy& c = *cp[d];
    HIPOK(hipSetDevice(c.phys), "hipSetDevice");
    if (!c.stream) {
      hipStream_t st;
      HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
      c.stream = st;
    }
    for (void*& e : c.ev)
      if (!e) {
        hipEvent_t x;
        HIPOK(hipEventCreate(&x), "hipEventCreate");
        e = x;
      }
    e0[d] = static_cast<hipEvent_t>(c.ev[0]);
    e1[d] = static_cast<hipEvent_t>(c.ev[1]);
  }
  const uint32_t tiles_x = (w + 7u) / 8u, nt = tiles_x * ((h + 7u) / 8u);
  const size_t frame_bytes = (size_t)w * h * 3 * sizeof(float);

  if (n == 1) {  // one device: rtw_render's path (the whole frame straight into the image), no RCCL
    DeviceCopy& c = *cp[0];
    HIPOK(hipSetDevice(c.phys), "hipSetDevice");
    hipStream_t st = static_cast<hipStream_t>(c.stream);
    if (int e = grow(c.image, frame_bytes)) return e;
    TileSet all;
    all.n = nt;
    if (int e = enqueue_render(s->s, c, cam, bg, w, h, spp, max_depth, seed, all, static_cast<float*>(c.image.p), st, 0,
                               e0[0], e1[0]))
      return e;
    rtw_stats st1;
    memset(&st1, 0, sizeof st1);
    if (int e = collect_stats(c, st, e0[0], e1[0], (uint64_t)w * h * spp, &st1)) return e;
    HIPOK(hipMemcpy(out, c.image.p, frame_bytes, hipMemcpyDeviceToHost), "hipMemcpy(image)");
    s->s.multi_ms.assign(1, (float)st1.kernel_ms);
    s->s.multi_gather_ms = 0.0f;
    st1.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = st1;
    return RTW_OK;
  }

  Clique* clique = nullptr;
  {
    std::vector<int> devs(n);
    for (int d = 0; d < n; ++d) devs[d] = cp[d]->phys;
    if (int e = get_clique(devs, &clique)) return e;
  }
  const std::vector<ncclComm_t>* comms = &clique->comms;
  const Rccl& r = *clique->lib;  // loaded for good (rccl())
  const uint32_t per = (nt + (uint32_t)n - 1) / (uint32_t)n;  // padded tiles per device
  const size_t slot_floats = (size_t)per * 64 * 3;
  std::vector<uint32_t> all((size_t)n * per);
  std::vector<uint32_t> mine(n);
  for (int d = 0; d < n; ++d) rtw_tile_partition(w, h, (uint32_t)n, (uint32_t)d, all.data() + (size_t)d * per, per, &mine[d]);

  // 1. every device renders its tiles d, d + n, d + 2n, ... (no id table: the kernel computes them) into its
  // packed buffer on its own stream, all enqueued before any wait
  for (int d = 0; d < n; ++d) {
    DeviceCopy& c = *cp[d];
    HIPOK(hipSetDevice(c.phys), "hipSetDevice");
    hipStream_t st = static_cast<hipStream_t>(c.stream);
    if (int e = grow(c.packed, slot_floats * sizeof(float))) return e;
    TileSet mt;
    mt.first = (uint32_t)d;
    mt.stride = (uint32_t)n;
    mt.n = mine[d];
    mt.packed = true;
    if (int e = enqueue_render(s->s, c, cam, bg, w, h, spp, max_depth, seed, mt, static_cast<float*>(c.packed.p), st, 0,
                               e0[d], e1[d]))
      return e;
  }
  // 2. one RCCL gather to device 0 (each device's send waits for its render on the same stream)
  DeviceCopy& c0 = *cp[0];
  HIPOK(hipSetDevice(c0.phys), "hipSetDevice");
  hipStream_t st0 = static_cast<hipStream_t>(c0.stream);
  if (int e = grow(c0.gathered, (size_t)n * slot_floats * sizeof(float))) return e;
  if (int e = grow(c0.gather_ids, all.size() * sizeof(uint32_t))) return e;
  if (int e = grow(c0.image, (size_t)w * h * 3 * sizeof(float))) return e;
  HIPOK(hipMemcpyAsync(c0.gather_ids.p, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st0),
        "hipMemcpyAsync(gather ids)");
  float* gathered = static_cast<float*>(c0.gathered.p);
  // device 0's gather time: its stream from the end of its own render to the last tile's arrival (so it
  // includes waiting for the slowest device), rtw_render_multi_times
  for (void*& e : c0.gev)
    if (!e) {
      hipEvent_t x;
      HIPOK(hipEventCreate(&x), "hipEventCreate");
      e = x;
    }
  HIPOK(hipEventRecord(static_cast<hipEvent_t>(c0.gev[0]), st0), "hipEventRecord");
  {
    std::lock_guard<std::mutex> lock(clique->mu);  // one grouped send/recv on these communicators at a time
    const ncclResult_t g0 = r.group_start();
    if (g0 != ncclSuccess) return fail(RTW_ENODEV, "ncclGroupStart: %s", r.error_string(g0));
    for (int d = 0; d < n; ++d) {
      hipStream_t st = static_cast<hipStream_t>(cp[d]->stream);
      const ncclResult_t a = r.send(cp[d]->packed.p, slot_floats, ncclFloat32, 0, (*comms)[d], st);
      if (a != ncclSuccess) {
        r.group_end();
        return fail(RTW_ENODEV, "ncclSend: %s", r.error_string(a));
      }
    }
    for (int d = 0; d < n; ++d) {
      const ncclResult_t a = r.recv(gathered + (size_t)d * slot_floats, slot_floats, ncclFloat32, d, (*comms)[0], st0);
      if (a != ncclSuccess) {
        r.group_end();
        return fail(RTW_ENODEV, "ncclRecv: %s", r.error_string(a));
      }
    }
    const ncclResult_t g1 = r.group_end();
    if (g1 != ncclSuccess) return fail(RTW_ENODEV, "ncclGroupEnd: %s", r.error_string(g1));
  }
  HIPOK(hipSetDevice(c0.phys), "hipSetDevice");
  HIPOK(hipEventRecord(static_cast<hipEvent_t>(c0.gev[1]), st0), "hipEventRecord");
  // 3. device 0 scatters the gathered tiles into the frame and copies it out
  HIPOK(hipSetDevice(c0.phys), "hipSetDevice");
  if (int e = enqueue_unpack(w, h, static_cast<uint32_t*>(c0.gather_ids.p), (uint32_t)all.size(), gathered,
                             static_cast<float*>(c0.image.p), st0))
    return e;
  HIPOK(hipMemcpyAsync(out, c0.image.p, (size_t)w * h * 3 * sizeof(float), hipMemcpyDeviceToHost, st0),
        "hipMemcpyAsync(image)");
  rtw_stats tot;
  memset(&tot, 0, sizeof tot);
  std::vector<float> dev_ms(n);
  for (int d = 0; d < n; ++d) {
    HIPOK(hipSetDevice(cp[d]->phys), "hipSetDevice");
    rtw_stats st;
    memset(&st, 0, sizeof st);
    if (int e = collect_stats(*cp[d], cp[d]->stream, e0[d], e1[d], 0, &st)) return e;
    tot.rays += st.rays;
    tot.kernel_ms = std::max(tot.kernel_ms, st.kernel_ms);  // the devices run concurrently
    dev_ms[d] = (float)st.kernel_ms;
  }
  float gms = 0.0f;
  HIPOK(hipSetDevice(c0.phys), "hipSetDevice");
  HIPOK(hipEventElapsedTime(&gms, static_cast<hipEvent_t>(c0.gev[0]), static_cast<hipEvent_t>(c0.gev[1])),
        "hipEventElapsedTime(gather)");
  s->s.multi_ms = dev_ms;
  s->s.multi_gather_ms = gms;
  tot.paths = (uint64_t)w * h * spp;
  tot.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = tot;
  return RTW_OK;
}

// Test hook: n logical devices on physical device 0 (upload in rtw_kernel.hip; include/rtw.h)
int rtw_diag_alias_devices(rtw_scene* s, int n) {
  if (!s) return fail(RTW_EINVAL, "NULL argument");
  if (s->s.committed) return fail(RTW_ESTATE, "scene already committed (alias the devices before the commit)");
  if (n < 1 || n > 64) return fail(RTW_EINVAL, "n = %d logical devices (1..64)", n);
  s->s.alias_n = n;
  return RTW_OK;
}

int rtw_render_multi_times(const rtw_scene* s, float* device_ms, uint32_t cap, float* gather_ms) {
  if (!s || (cap && !device_ms)) return fail(RTW_EINVAL, "NULL argument");
  const std::vector<float>& v = s->s.multi_ms;
  for (size_t d = 0; d < v.size() && d < cap; ++d) device_ms[d] = v[d];
  if (gather_ms) *gather_ms = s->s.multi_gather_ms;
  return (int)v.size();
}

}  // extern "C"
