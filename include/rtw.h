/*
 * rtw.h — C-ABI of the MI355X-native render core (librtw_amd.so).
 *
 * Drop-in boundary for raytracer_weekend_lib's render hot path
 * (reference: /root/reference, paths below relative to raytracer_weekend_lib/src/).
 * The reference boundary is
 *     Raytracer::new(world: &[Box<dyn Hittable>], cam: &Camera, background: Color,
 *                    image_width: u32, image_height: u32, samples_per_pixel: u32)   lib.rs:40-48
 *     Raytracer::render(&self) -> impl RenderIterator<Item = Pixel>                  lib.rs:57-76
 * with the scene built through the Hittable/Material/Texture constructors listed per
 * function below.  Because `dyn Hittable` has no introspection, the world crosses this
 * boundary as a builder call stream (one call per reference constructor), is flattened
 * once by rtw_scene_commit(), and rendered by rtw_render*().  INTEGRATION.md shows the
 * Rust `extern "C"` block and the per-type `flatten` method a maintainer would add.
 *
 * Conventions: every int-returning function returns 0 on success or a negative
 * errno-style code (RTW_E*), with a thread-local message in rtw_last_error().  The
 * reference panics in the same situations (bvh.rs:57, material.rs:71, triangular.rs:178).
 * Input arrays are copied; the caller keeps ownership.  A scene is immutable after
 * rtw_scene_commit(); rendering is blocking on the given (or default) HIP stream.
 * There is no CPU fallback: without a usable gfx950 device rtw_scene_commit() and the
 * render calls fail with RTW_ENODEV.
 */
#ifndef RTW_H
#define RTW_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 6

enum {
  RTW_OK = 0,
  RTW_EINVAL = -22,  /* bad argument (reference: panic / assert) */
  RTW_ENOMEM = -12,
  RTW_ENODEV = -19,  /* no HIP device / kernel launch failed */
  RTW_ESTATE = -71,  /* call not valid in the scene's state (e.g. add after commit) */
  RTW_EIO = -5       /* file / parse error (reference: unwrap on io / parse errors) */
};

typedef struct rtw_scene rtw_scene;

/* camera.rs:9-20 Camera — filled by rtw_camera_new (camera.rs:25-64). */
typedef struct {
  float origin[3], lower_left_corner[3], horizontal[3], vertical[3];
  float u[3], v[3], w[3];
  float lens_radius, time0, time1;
} rtw_camera;

/* Render statistics. rays = number of world.hit queries (lib.rs:102). */
typedef struct {
  uint64_t rays;
  uint64_t paths;          /* W*H*spp actually rendered */
  double kernel_ms;        /* device time of the render kernel(s), HIP events */
  double total_ms;         /* host wall time of the call (incl. D2H for rtw_render) */
  uint64_t node_visits;    /* only when RTW_FLAG_COUNT_TRAVERSAL */
  uint64_t prim_tests;     /* only when RTW_FLAG_COUNT_TRAVERSAL */
  uint64_t prim_tests_by_type[6]; /* sphere, moving sphere, rect xy, xz, yz, triangle */
  /* RTW_FLAG_COUNT_TRAVERSAL: SIMD utilisation, pairs of (wave executions, active lanes) for
   * the BVH node loop, primitive tests and path segments */
  uint64_t simd[6];
  /* RTW_FLAG_COUNT_TRAVERSAL: wave-cycles (s_memtime) spent in path regeneration, closest-hit
   * traversal and shading, and in the whole path kernel, summed over waves */
  uint64_t phase_cycles[4];
  /* RTW_FLAG_COUNT_TRAVERSAL: child boxes slab-tested (the non-empty slots of the visited 4-wide
   * nodes), and sub-phase wave-cycles: [0] shading's random_in_unit_sphere (counted apart from
   * phase_cycles[2]), [1] traversal's node loop and [2] leaf tests (parts of phase_cycles[1]),
   * [3] regeneration's per-lane path start (part of phase_cycles[0]) */
  uint64_t boxes_tested;
  uint64_t sub_cycles[4];
} rtw_stats;

enum { RTW_FLAG_COUNT_TRAVERSAL = 1 };

const char* rtw_last_error(void);
int rtw_abi_version(void);
/* Number of visible HIP devices (0 in a GPU-less container; never initialises a context). */
int rtw_device_count(void);

/* ---- scene lifetime */
int rtw_scene_create(rtw_scene** out);
void rtw_scene_destroy(rtw_scene* scene);

/* ---- textures: texture.rs:45-60 SolidColor::new/new_rgb, :62-81 Checker::new(odd, even, freq),
 *      image_texture.rs:23-30 ImageTexture (decoded RGB8 pixels, row-major, top row first),
 *      texture.rs:97-104 UVDebug */
int rtw_texture_solid(rtw_scene* s, float r, float g, float b, uint32_t* id);
int rtw_texture_checker(rtw_scene* s, uint32_t odd, uint32_t even, float frequency, uint32_t* id);
int rtw_texture_image(rtw_scene* s, const uint8_t* rgb8, uint32_t width, uint32_t height, uint32_t* id);
int rtw_texture_uvdebug(rtw_scene* s, uint32_t* id);
/* texture.rs:83-95 Noise::new(Perlin, scale): value = 0.5 (1 + sin(scale p.z + 10 turbulence(p, 7))).
 * The Perlin tables (perlin.rs:8-48) cross as data: gradients 256x3 floats (unit vectors),
 * permutations 3x256 (x, y, z; each a permutation of 0..255, else RTW_EINVAL).  Perlin::new(rng)
 * with this build's seeded stream is rtw_perlin_generate(). */
int rtw_texture_noise(rtw_scene* s, const float* gradients, const uint32_t* permutations, float scale,
                      uint32_t* id);
int rtw_perlin_generate(uint64_t seed, float* gradients, uint32_t* permutations);

/* ---- materials: material.rs:30-39 Lambertian::new, :63-73 Metal::new (fuzz <= 1 else
 *      RTW_EINVAL, as the assert at :71), :102-105 Dielectric::new, light_source.rs:12-15
 *      DiffuseLight::new */
int rtw_material_lambertian(rtw_scene* s, uint32_t texture, uint32_t* id);
int rtw_material_metal(rtw_scene* s, float r, float g, float b, float fuzz, uint32_t* id);
int rtw_material_dielectric(rtw_scene* s, float index_of_refraction, uint32_t* id);
int rtw_material_diffuse_light(rtw_scene* s, uint32_t texture, uint32_t* id);
/* material.rs:148-165 Isotropic::new(albedo texture): scatters into random_in_unit_sphere */
int rtw_material_isotropic(rtw_scene* s, uint32_t texture, uint32_t* id);

/* ---- hierarchy.  Objects are appended to the innermost open group (the world list at the
 *      top).  Groups nest; each must be closed with rtw_end().
 *      rtw_begin_list:      Vec<Box<dyn Hittable>>            hittable/mod.rs:57-69, 90-98
 *      rtw_begin_bvh:       BvhNode::new(objects, t0, t1, rng)  bvh.rs:19-74
 *      rtw_begin_translate: Translation::new(inner, offset)    transformations.rs:16-47
 *      rtw_begin_rotate_y:  YRotation::new(inner, degrees)     transformations.rs:50-75
 *      rtw_begin_constant_medium: ConstantMedium::new(boundary, density, texture) volumes.rs:17-35;
 *        the group holds the boundary: exactly one object, a Sphere or a Cuboid (optionally under
 *        Translation / YRotation) in this build, else RTW_EINVAL at rtw_end / commit.  Creates the
 *        medium's Isotropic(texture) phase function, whose id goes to *material (may be NULL).
 *        The medium's free-path draw comes from a sub-stream keyed by (path segment, medium),
 *        not the path's shared stream (order-independent form).
 *      A wrapper applies to everything added inside it (= the wrapper of a list). */
int rtw_begin_list(rtw_scene* s);
int rtw_begin_bvh(rtw_scene* s, float time0, float time1);
int rtw_begin_translate(rtw_scene* s, float x, float y, float z);
int rtw_begin_rotate_y(rtw_scene* s, float degrees);
int rtw_begin_constant_medium(rtw_scene* s, float density, uint32_t texture, uint32_t* material);
int rtw_end(rtw_scene* s);

/* ---- primitives (SoA arrays of length n; copied)
 *      Sphere::new(center, radius, material)                spherical.rs:79-104
 *      MovingSphere::new(c0, t0, c1, t1, radius, material)  spherical.rs:106-151
 *      XY/XZ/YZRectangle::new(a0, a1, b0, b1, k, material)  rectangular.rs:16-166
 *        axis: 0 = XY (k on z), 1 = XZ (k on y), 2 = YZ (k on x)
 *      Cuboid::new(p0, p1, material)                        rectangular.rs:170-245
 *      Triangle::new(vertices, [Option<normal>;3], [Option<uv>;3], material)  triangular.rs:33-73
 *        verts: 9n floats; normals: 9n floats or NULL; normal_mask: n bytes (bit k = vertex k
 *        has a normal) or NULL; uvs: 6n floats or NULL; uv_mask likewise. */
int rtw_add_spheres(rtw_scene* s, uint32_t n, const float* cx, const float* cy, const float* cz,
                    const float* radius, const uint32_t* material);
int rtw_add_moving_spheres(rtw_scene* s, uint32_t n, const float* c0x, const float* c0y,
                           const float* c0z, const float* t0, const float* c1x, const float* c1y,
                           const float* c1z, const float* t1, const float* radius,
                           const uint32_t* material);
int rtw_add_rects(rtw_scene* s, uint32_t n, const uint32_t* axis, const float* a0, const float* a1,
                  const float* b0, const float* b1, const float* k, const uint32_t* material);
int rtw_add_cuboid(rtw_scene* s, const float p0[3], const float p1[3], uint32_t material);
int rtw_add_triangles(rtw_scene* s, uint32_t n, const float* verts, const float* normals,
                      const uint8_t* normal_mask, const float* uvs, const uint8_t* uv_mask,
                      uint32_t material);

/* load_wavefront_obj(path, rng) triangular.rs:241-260: adds BvhNode(triangles) to the open
 * group.  Faces without a material get DiffuseLight(1,0,1) (:177-182); map_Kd images are
 * decoded only if image_loader != NULL (the build ships no JPEG/PNG decoder; a missing
 * loader or file is RTW_EIO as the reference's unwrap at :308).  `.rtwm` files (this
 * build's binary mesh dump) are accepted too; their material is taken
 * from `fallback_material` when != UINT32_MAX. */
typedef int (*rtw_image_loader)(const char* path, uint8_t** rgb8, uint32_t* w, uint32_t* h);
int rtw_load_wavefront_obj(rtw_scene* s, const char* path, rtw_image_loader image_loader,
                           uint32_t fallback_material, uint32_t* n_triangles);

/* Flatten the hierarchy, build the BVH and upload to every visible device (or only to
 * `device` when >= 0).  After this the scene is immutable. */
int rtw_scene_commit(rtw_scene* s, int device);

/* Camera::new(look_from, look_at, vup, vfov, aspect, aperture, focus_dist, t0, t1) camera.rs:25-64 */
int rtw_camera_new(const float look_from[3], const float look_at[3], const float vup[3],
                   float vfov_degrees, float aspect_ratio, float aperture, float focus_dist,
                   float time0, float time1, rtw_camera* out);

/* Raytracer::new(world, cam, background, w, h, spp).render().collect() — lib.rs:40-95.
 * out_rgb_sum (host, w*h*3 floats) receives the un-normalised Σ over spp per pixel in the
 * reference's emission order (lib.rs:58: row j = h-1 .. 0, column i = 0 .. w-1), i.e.
 * out[((h-1-j)*w + i)*3 + c].  max_depth is MAX_DEPTH (lib.rs:32, 50).  The per-sample
 * random stream is keyed by (seed, j, i, sample) so the image is independent of tiling
 * and device count. */
int rtw_render(rtw_scene* s, const rtw_camera* cam, const float background[3], uint32_t w,
               uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, float* out_rgb_sum,
               rtw_stats* stats);

/* lib.rs:120-126 Pixel: row j (0 = bottom), column i, un-normalised Σ over spp. */
typedef struct {
  uint32_t row, column;
  float color[3];
} rtw_pixel;
/* Receives the next n pixels of the stream; a non-zero return stops the render (returned as is). */
typedef int (*rtw_pixel_sink)(const rtw_pixel* pixels, uint32_t n, void* user);

/* Raytracer::render() as a progressive stream (lib.rs:50-76 RenderIterator): the frame is rendered
 * in bands of `band_rows` output rows (rounded up to whole 8-row tile rows; 0 = 64) and each band's
 * pixels are handed to `sink` in the reference's emission order (row j = h-1 .. 0, column 0 .. w-1)
 * as soon as the band is done.  Same pixels as rtw_render. */
int rtw_render_stream(rtw_scene* s, const rtw_camera* cam, const float background[3], uint32_t w,
                      uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, uint32_t band_rows,
                      rtw_pixel_sink sink, void* user, rtw_stats* stats);

/* lib.rs:128-138 ProgressMessage on the wire (discovery_app/src/bin/raytracer.rs:62-113 ->
 * discovery_host_receiver/src/main.rs:22-110): postcard 0.7.3 (Cargo.lock:2533-2541; enum tag and
 * u32 as varints, f32 little-endian, Color as its 3-float array) framed by COBS (postcard-cobs
 * 0.1.5-pre) with a trailing 0x00, exactly as postcard::to_vec_cobs. */
enum { RTW_MSG_IMAGE_START = 0, RTW_MSG_PIXEL = 1, RTW_MSG_IMAGE_END = 2 };
typedef struct {
  uint32_t kind;
  uint32_t width, height, samples_per_pixel; /* RTW_MSG_IMAGE_START */
  rtw_pixel pixel;                           /* RTW_MSG_PIXEL */
} rtw_progress_msg;
/* Encodes one message (<= 32 bytes incl. the 0x00 delimiter) into out; *len = bytes written. */
int rtw_progress_encode(const rtw_progress_msg* msg, uint8_t* out, size_t cap, size_t* len);
/* Decodes one COBS frame (with or without its trailing 0x00), as postcard::from_bytes_cobs. */
int rtw_progress_decode(const uint8_t* frame, size_t len, rtw_progress_msg* msg);

/* Render a subset of 8x8 pixel tiles into device memory (multi-GPU / framework path).
 * Tile t covers columns [8*tx, 8*tx+8) and output rows [8*ty, 8*ty+8) (row r <-> j = h-1-r),
 * tile id = ty * ceil(w/8) + tx.  If d_tile_ids == NULL all tiles are rendered and d_out is a
 * full w*h*3 image in reference order; otherwise d_tile_ids is a DEVICE array of n_tiles ids
 * and d_out is packed [n_tiles][64][3] (pixels outside the image, and ids beyond the last tile,
 * are left untouched).  `stream` is a hipStream_t (NULL = default).  The call only enqueues unless
 * stats != NULL, in which case it synchronises and fills stats.  Each (scene, device) pair owns one
 * path queue and one sample buffer: renders of a scene on one device must be serialised on one
 * stream (two renders in flight on different streams would share them).  The first render of a
 * given size allocates the sample buffer (hipMalloc: not stream-capturable); later renders of the
 * same or a smaller size only enqueue.  Without stats, a traversal fault of this render surfaces at
 * the first rtw_render* call that starts after this render has COMPLETED (the check reads the device's
 * host-mapped error word without waiting), or at rtw_render_status, which waits. */
int rtw_render_device(rtw_scene* s, int device, const rtw_camera* cam, const float background[3],
                      uint32_t w, uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed,
                      const uint32_t* d_tile_ids, uint32_t n_tiles, float* d_out, void* stream,
                      uint32_t flags, rtw_stats* stats);
/* rtw_render_device over the tiles first_tile + k * tile_stride (k < n_tiles) without an id table
 * (the kernel computes them): a device's round-robin share of the frame (rtw_tile_partition part p of
 * n: first_tile = p, tile_stride = n).  d_out is packed [n_tiles][64][3].  RTW_EINVAL if a tile
 * leaves the frame or tile_stride == 0. */
int rtw_render_device_strided(rtw_scene* s, int device, const rtw_camera* cam, const float background[3],
                              uint32_t w, uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed,
                              uint32_t first_tile, uint32_t tile_stride, uint32_t n_tiles, float* d_out,
                              void* stream, uint32_t flags, rtw_stats* stats);
/* Errors of renders the caller did not wait for.  A path kernel whose BVH walk trips its guard (a
 * corrupt tree: the walk is bounded, and the first trip closes the path queue, so the grid drains after
 * about one trip per wave) sets the device's host-mapped error word.  It is reported, and cleared, as
 * RTW_EINVAL by the first rtw_render* call on that device that starts after the faulting render has
 * completed (checked before it enqueues, without waiting: a call made while the faulting kernel still
 * runs passes, and a later one reports it), by rtw_path_kernel_times and any call with stats (both wait
 * first), and by this function, which first waits for all work on the device (hipDeviceSynchronize).
 * RTW_OK = every frame rendered so far on `device` (-1: the first copy) is valid. */
int rtw_render_status(rtw_scene* s, int device);
/* Test hook: overwrite the device copy's first two BVH nodes with a cycle, so that every render of it
 * trips the traversal guard (tests/test_gpu_parity.py).  The scene stays unusable on that device. */
int rtw_diag_corrupt_bvh(rtw_scene* s, int device);
/* Test hook (the multi-device path on a one-GPU node): before rtw_scene_commit, make the scene's devices n
 * LOGICAL devices 0..n-1 that all live on physical device 0.  rtw_scene_commit(s, -1) then uploads n copies,
 * each with its own stream, path queue, sample and packed buffers, so rtw_render_multi(s, n) runs its n > 1
 * path (per-device renders, the grouped send/recv gather to logical device 0, the unpack) on one GPU.  Real
 * RCCL refuses a clique whose ranks share a GPU: pair it with a loopback RCCL through RTW_RCCL_LIB
 * (tests/loopback_rccl).  1 <= n <= 64, else RTW_EINVAL; RTW_ESTATE after the commit. */
int rtw_diag_alias_devices(rtw_scene* s, int n);

/* Raytracer::new(..).render().collect() (lib.rs:40-95) over n_gpus devices of this node, driven from
 * the calling host thread (the reference's Rayon pixel parallelism, lib.rs:57-76, becomes tiles
 * across GPUs).  Tile k goes to device k mod n (rtw_tile_partition); each device renders its tiles
 * on its own stream with its own copy of the scene (commit with device = -1 first); one RCCL gather
 * over xGMI (grouped ncclSend to device 0 / ncclRecv on device 0; librccl.so.1 is opened on first
 * use) brings the tiles to device 0, which assembles the frame and copies it into out_rgb_sum in the
 * same layout as rtw_render.  n_gpus <= 0 = every visible device.  The frame is bit-identical to
 * rtw_render's for every n_gpus (per-pixel random streams).  stats->rays sums the devices,
 * stats->kernel_ms is the slowest device's.  Blocking.  With one device (n_gpus = 1, or 0 on a one-GPU
 * node) it is rtw_render's path on device 0 and never opens RCCL; RTW_RCCL_LIB names another RCCL
 * library to open. */
int rtw_render_multi(rtw_scene* s, int n_gpus, const rtw_camera* cam, const float background[3], uint32_t w,
                     uint32_t h, uint32_t spp, uint32_t max_depth, uint64_t seed, float* out_rgb_sum,
                     rtw_stats* stats);
/* Timing of the scene's last rtw_render_multi call (a scaling run's diagnosis: load imbalance against
 * gather cost): device_ms[d] = device d's render (path kernel + in-order reduction, HIP events on its
 * stream) for d < min(cap, n); *gather_ms (may be NULL) = device 0's stream time from the end of its own
 * render to the arrival of every device's tiles (the RCCL send/recv group, so it includes waiting for the
 * slowest device; 0 for one device).  Returns n (0 before the first call).  Host only, no wait.
 * (No reference counterpart: a benchmark hook beside rtw_render_multi.) */
int rtw_render_multi_times(const rtw_scene* s, float* device_ms, uint32_t cap, float* gather_ms);

/* The frame partition rtw_render_multi (and bench.py's one-process-per-GPU path) uses: the 8x8 tiles
 * of a w x h frame dealt round-robin to n_parts parts; part p gets tiles p, p + n, p + 2n, ...
 * Writes min(cap, ceil(nt / n)) ids (the part's tiles, then padding ids equal to nt, which
 * rtw_unpack_tiles_device skips) and the part's real tile count to *n_ids.  Host only. */
int rtw_tile_partition(uint32_t w, uint32_t h, uint32_t n_parts, uint32_t part, uint32_t* ids, uint32_t cap,
                       uint32_t* n_ids);

/* Scatter packed tiles (as written by rtw_render_device) into a full device image. */
int rtw_unpack_tiles_device(int device, uint32_t w, uint32_t h, const uint32_t* d_tile_ids,
                            uint32_t n_tiles, const float* d_packed, float* d_image, void* stream);

/* Device time (ms, HIP events on the render stream) of the most recent path-kernel launches of
 * rtw_render / rtw_render_device on `device`, oldest first: at most max_n of the last 64, written
 * to ms[]; returns how many (>= 0) or an error, and forgets them.  Waits for those launches, and
 * returns RTW_EINVAL if one of them tripped the traversal guard (rtw_render_status).
 * (Benchmark hook: the render call itself also enqueues the in-order sample reduction.) */
int rtw_path_kernel_times(rtw_scene* s, int device, float* ms, uint32_t max_n);

/* Diagnostics: evaluate the render path's f32 transcendentals on the device over n host values
 * (fn 0 log10f(a), 1 sinf(a), 2 acosf(a), 3 atan2f(a, b); DESIGN.md §Parity: correctly rounded;
 * fn 4 a / b by the camera's Markstein division from the reciprocal RN(1 / b), fn 5 the sphere
 * test's sqrt(a)).
 * Used by the parity tests to pin the device functions against the oracle's. */
int rtw_diag_libm(int fn, uint32_t n, const float* a, const float* b, float* out);
/* Diagnostics: every 32-bit pattern b in [lo, hi] (as a float) through a device fast path, compared bit
 * for bit with the IEEE operation on the device.  fn 0: the render path's reciprocal rcp_rn (v_rcp_f32 +
 * one Newton step) vs 1.0f / b, over |b| in [2^-126, 2^126].  counts[0] = mismatches, counts[1] = patterns
 * outside the fast path's range (skipped); the first min(cap, counts[0]) mismatching patterns go to bad. */
int rtw_diag_sweep(int fn, uint32_t lo, uint32_t hi, uint64_t* counts, uint32_t* bad, uint32_t cap);
/* Diagnostics (host only, no device): the host's RN(1 / b) that the camera's u, v divisions use
 * (rtw_render*: b = w - 1, h - 1), over n values; exact for integer-valued b in [1, 2^24). */
int rtw_diag_recip(uint32_t n, const float* b, float* out);

/* console_app/src/main.rs:68-90 tonemap: sqrt(sum/spp), clamp [0, 0.999], u8(255.999*c). */
int rtw_tonemap(const float* rgb_sum, uint32_t n_pixels, uint32_t spp, uint8_t* rgb8);

/* ---- scene presets: console_app/src/scenes.rs restated (jumpy-balls :63-162, two-spheres
 *      :164-209, two-perlin-spheres :211-252, earth :254-288, simple-light :290-348, cornell-box
 *      :350-414, smokey-cornell-box :416-483, book2-final-scene :485-620,
 *      animated-book2-final-scene :622-667, simple-triangle :669-717, wavefront-cow-obj :719-771,
 *      textured-monument :816-858).  `seed` replaces thread_rng() for the random placement;
 *      models_dir holds the meshes and images.  Fills cam (the first camera) and background. */
int rtw_scene_preset(rtw_scene* s, const char* name, float aspect_ratio, uint64_t seed,
                     const char* models_dir, rtw_camera* cam, float background[3]);
/* All cameras of a preset (World = (objects, Vec<Camera>, background), scenes.rs:42-58):
 * 30 for animated-book2-final-scene, 1 otherwise.  *n = the count; min(cap, *n) written. */
int rtw_preset_cameras(const char* name, float aspect_ratio, const char* models_dir, rtw_camera* cams,
                       uint32_t cap, uint32_t* n);

/* Introspection for the test harness: the committed hierarchy as text (DESIGN.md
 * §Scene text).  Returns the required size (incl. NUL) in *needed; writes when cap
 * suffices.  rtw_scene_image(k) returns the k-th image texture's pixels. */
int rtw_scene_dump(const rtw_scene* s, char* buf, size_t cap, size_t* needed);
int rtw_scene_image(const rtw_scene* s, uint32_t k, const uint8_t** rgb8, uint32_t* w, uint32_t* h);
/* 0 leaf primitives, 1 materials, 2 textures, 3 BVH nodes, 4 BVH depth, 5 always-tested
 * primitives, 6 instances, 7 BVH2 nodes, 8 traversal-stack bound, 9 feature mask (rtw_device.hpp
 * Feature; selects the path-kernel variant), 10 Perlin tables, 11 stack bound of the sorted-push
 * walk (LDS-node kernels), 12 runs of the always list (one wrapper chain and one prim kind each: the
 * list-mode rect loop's program), 13 1 if every rect admits the list loop's fast path (|k| < 2^62,
 * ordered bounds), 14 1 if the BVH holds sphere tests (their leaves are padded for origins within D0
 * and farther origins take the far-origin walk), 15 that D0 in thousandths.  3-15 are
 * valid once rtw_scene_commit has flattened the scene (also when its upload failed for lack of a device). */
int64_t rtw_scene_info(const rtw_scene* s, int what);
/* Introspection for the test harness: the flattened 4-wide BVH (DevNode4, 128 B each, breadth-first
 * numbered; csrc/rtw_device.hpp), valid once rtw_scene_commit has flattened the scene (also when its
 * upload failed for lack of a device).  *nodes points into the scene (read-only, lives as long as it). */
int rtw_scene_nodes(const rtw_scene* s, const void** nodes, uint32_t* n_nodes);
/* The same tree in half precision (DevNode4h, 112 B each: f16 plane offsets from an f16 origin, rounded
 * outward; built when the 16-bit child codes fit, else *n_nodes = 0), as the kernels read it. */
int rtw_scene_nodes_half(const rtw_scene* s, const void** nodes, uint32_t* n_nodes);

#ifdef __cplusplus
}
#endif
#endif
