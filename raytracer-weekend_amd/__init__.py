"""rtw_amd — Python host mirror of raytracer_weekend_lib's render API over the C-ABI.

The product is ``lib/librtw_amd.so`` (HIP kernels for gfx950 + C++ host, include/rtw.h).
This module is plumbing: ctypes bindings whose names and argument meaning follow the
reference crate (raytracer_weekend_lib/src/), so tests read like the reference's API:

    scene = Scene()
    ground = scene.lambertian(scene.checker(scene.solid_rgb(.2, .3, .1), scene.solid_rgb(.9, .9, .9), 10))
    scene.sphere((0, -1000, 0), 1000, ground)                  # Sphere::new        spherical.rs:79
    with scene.translate((265, 0, 295)), scene.rotate_y(15):   # .rotate_y().translate()
        scene.cuboid((0, 0, 0), (165, 330, 165), white)        # Cuboid::new        rectangular.rs:177
    scene.commit()
    cam = Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 16 / 9, 0.1, 10, 0, 1)   # camera.rs:25
    img, stats = Raytracer(scene, cam, (0.7, 0.8, 1.0), 400, 225, 50).render()       # lib.rs:40-76

There is no CPU fallback: if the shared library is missing this module raises on load,
and without a GPU ``Scene.commit`` raises ``RtwError(-19)``.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
REPO_ROOT = PKG_DIR.parent
LIB_PATH = Path(os.environ.get("RTW_LIB_PATH") or PKG_DIR / "lib" / "librtw_amd.so")  # override: tuning builds
MODELS_DIR = REPO_ROOT / "models"

RTW_EINVAL, RTW_ENOMEM, RTW_ENODEV, RTW_ESTATE, RTW_EIO = -22, -12, -19, -71, -5
FLAG_COUNT_TRAVERSAL = 1
NO_MATERIAL = 0xFFFFFFFF


class RtwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rtw error {code}: {msg}")
        self.code = code


class rtw_camera(C.Structure):  # include/rtw.h, camera.rs:9-20
    _fields_ = [("origin", C.c_float * 3), ("lower_left_corner", C.c_float * 3),
                ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3),
                ("u", C.c_float * 3), ("v", C.c_float * 3), ("w", C.c_float * 3),
                ("lens_radius", C.c_float), ("time0", C.c_float), ("time1", C.c_float)]


class rtw_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("paths", C.c_uint64), ("kernel_ms", C.c_double),
                ("total_ms", C.c_double), ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64),
                ("prim_tests_by_type", C.c_uint64 * 6), ("simd", C.c_uint64 * 6),
                ("phase_cycles", C.c_uint64 * 4), ("boxes_tested", C.c_uint64), ("sub_cycles", C.c_uint64 * 4)]

    def as_dict(self) -> dict:
        return {"rays": int(self.rays), "paths": int(self.paths), "kernel_ms": float(self.kernel_ms),
                "total_ms": float(self.total_ms), "node_visits": int(self.node_visits),
                "prim_tests": int(self.prim_tests),
                "prim_tests_by_type": [int(x) for x in self.prim_tests_by_type],
                "simd_util": {k: (self.simd[2 * q + 1] / (64.0 * self.simd[2 * q]) if self.simd[2 * q] else None)
                              for q, k in enumerate(("node_loop", "prim_tests", "segments"))},
                "boxes_tested": int(self.boxes_tested),
                "phase_share": dict({k: (self.phase_cycles[q] / self.phase_cycles[3] if self.phase_cycles[3] else None)
                                     for q, k in enumerate(("regen", "trace", "shade"))},
                                    **{k: (self.sub_cycles[q] / self.phase_cycles[3] if self.phase_cycles[3] else None)
                                       for q, k in enumerate(("sample", "node_loop", "leaf_tests", "path_start"))})}


class rtw_pixel(C.Structure):  # lib.rs:120-126 Pixel
    _fields_ = [("row", C.c_uint32), ("column", C.c_uint32), ("color", C.c_float * 3)]


class rtw_progress_msg(C.Structure):  # lib.rs:128-138 ProgressMessage
    _fields_ = [("kind", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("pixel", rtw_pixel)]


MSG_IMAGE_START, MSG_PIXEL, MSG_IMAGE_END = 0, 1, 2
PIXEL_SINK = C.CFUNCTYPE(C.c_int, C.POINTER(rtw_pixel), C.c_uint32, C.c_void_p)
PIXEL_DTYPE = np.dtype([("row", np.uint32), ("column", np.uint32), ("color", np.float32, 3)])

_F = C.POINTER(C.c_float)
_U32 = C.POINTER(C.c_uint32)
_U8 = C.POINTER(C.c_uint8)
_SIGS = {
    "rtw_last_error": (C.c_char_p, []),
    "rtw_abi_version": (C.c_int, []),
    "rtw_device_count": (C.c_int, []),
    "rtw_scene_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "rtw_scene_destroy": (None, [C.c_void_p]),
    "rtw_texture_solid": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_float, _U32]),
    "rtw_texture_checker": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, _U32]),
    "rtw_texture_image": (C.c_int, [C.c_void_p, _U8, C.c_uint32, C.c_uint32, _U32]),
    "rtw_texture_uvdebug": (C.c_int, [C.c_void_p, _U32]),
    "rtw_texture_noise": (C.c_int, [C.c_void_p, _F, _U32, C.c_float, _U32]),
    "rtw_perlin_generate": (C.c_int, [C.c_uint64, _F, _U32]),
    "rtw_material_isotropic": (C.c_int, [C.c_void_p, C.c_uint32, _U32]),
    "rtw_material_lambertian": (C.c_int, [C.c_void_p, C.c_uint32, _U32]),
    "rtw_material_metal": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_float, _U32]),
    "rtw_material_dielectric": (C.c_int, [C.c_void_p, C.c_float, _U32]),
    "rtw_material_diffuse_light": (C.c_int, [C.c_void_p, C.c_uint32, _U32]),
    "rtw_begin_list": (C.c_int, [C.c_void_p]),
    "rtw_begin_bvh": (C.c_int, [C.c_void_p, C.c_float, C.c_float]),
    "rtw_begin_translate": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_float]),
    "rtw_begin_rotate_y": (C.c_int, [C.c_void_p, C.c_float]),
    "rtw_begin_constant_medium": (C.c_int, [C.c_void_p, C.c_float, C.c_uint32, _U32]),
    "rtw_end": (C.c_int, [C.c_void_p]),
    "rtw_add_spheres": (C.c_int, [C.c_void_p, C.c_uint32, _F, _F, _F, _F, _U32]),
    "rtw_add_moving_spheres": (C.c_int, [C.c_void_p, C.c_uint32] + [_F] * 9 + [_U32]),
    "rtw_add_rects": (C.c_int, [C.c_void_p, C.c_uint32, _U32, _F, _F, _F, _F, _F, _U32]),
    "rtw_add_cuboid": (C.c_int, [C.c_void_p, _F, _F, C.c_uint32]),
    "rtw_add_triangles": (C.c_int, [C.c_void_p, C.c_uint32, _F, _F, _U8, _F, _U8, C.c_uint32]),
    "rtw_load_wavefront_obj": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, _U32]),
    "rtw_scene_commit": (C.c_int, [C.c_void_p, C.c_int]),
    "rtw_camera_new": (C.c_int, [_F, _F, _F, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                 C.c_float, C.POINTER(rtw_camera)]),
    "rtw_render": (C.c_int, [C.c_void_p, C.POINTER(rtw_camera), _F, C.c_uint32, C.c_uint32, C.c_uint32,
                             C.c_uint32, C.c_uint64, _F, C.POINTER(rtw_stats)]),
    "rtw_render_device": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(rtw_camera), _F, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint32, C.c_uint64, _U32, C.c_uint32, C.c_void_p,
                                    C.c_void_p, C.c_uint32, C.POINTER(rtw_stats)]),
    "rtw_render_device_strided": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(rtw_camera), _F, C.c_uint32,
                                            C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(rtw_stats)]),
    "rtw_render_status": (C.c_int, [C.c_void_p, C.c_int]),
    "rtw_diag_corrupt_bvh": (C.c_int, [C.c_void_p, C.c_int]),
    "rtw_diag_alias_devices": (C.c_int, [C.c_void_p, C.c_int]),
    "rtw_path_kernel_times": (C.c_int, [C.c_void_p, C.c_int, _F, C.c_uint32]),
    "rtw_render_multi": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(rtw_camera), _F, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.c_uint32, C.c_uint64, _F, C.POINTER(rtw_stats)]),
    "rtw_render_multi_times": (C.c_int, [C.c_void_p, _F, C.c_uint32, _F]),
    "rtw_tile_partition": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _U32, C.c_uint32, _U32]),
    "rtw_render_stream": (C.c_int, [C.c_void_p, C.POINTER(rtw_camera), _F, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint64, C.c_uint32, PIXEL_SINK, C.c_void_p,
                                    C.POINTER(rtw_stats)]),
    "rtw_progress_encode": (C.c_int, [C.POINTER(rtw_progress_msg), _U8, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rtw_progress_decode": (C.c_int, [_U8, C.c_size_t, C.POINTER(rtw_progress_msg)]),
    "rtw_unpack_tiles_device": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32,
                                          C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtw_tonemap": (C.c_int, [_F, C.c_uint32, C.c_uint32, _U8]),
    "rtw_diag_libm": (C.c_int, [C.c_int, C.c_uint32, _F, _F, _F]),
    "rtw_diag_recip": (C.c_int, [C.c_uint32, _F, _F]),
    "rtw_diag_sweep": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), _U32, C.c_uint32]),
    "rtw_scene_preset": (C.c_int, [C.c_void_p, C.c_char_p, C.c_float, C.c_uint64, C.c_char_p,
                                   C.POINTER(rtw_camera), _F]),
    "rtw_preset_cameras": (C.c_int, [C.c_char_p, C.c_float, C.c_char_p, C.POINTER(rtw_camera), C.c_uint32,
                                     _U32]),
    "rtw_scene_dump": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rtw_scene_image": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(_U8), _U32, _U32]),
    "rtw_scene_nodes": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), _U32]),
    "rtw_scene_nodes_half": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), _U32]),
    "rtw_scene_info": (C.c_int64, [C.c_void_p, C.c_int]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


ABI_VERSION = 6  # include/rtw.h RTW_ABI_VERSION


def lib_sha() -> str:
    """First 16 hex digits of the SHA-256 of the library file this process loads (LIB_PATH): ties profiler
    evidence under profiles/ to the build it was measured on (bench.py attaches it only on a match)."""
    import hashlib
    return hashlib.sha256(LIB_PATH.read_bytes()).hexdigest()[:16] if LIB_PATH.exists() else ""


def lib() -> C.CDLL:
    """Load librtw_amd.so (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RtwError(RTW_ENODEV, f"{LIB_PATH} not built (run __graft_entry__.build())")
        # torch-ROCm bundles its own libamdhip64.so.7 + libhsa-runtime64 under the same SONAME as
        # /opt/rocm's; whichever loads first serves the whole process.  Load torch's first so the
        # render core and torch's streams / RCCL share ONE HIP runtime (the other order leaves torch
        # with "No HIP GPUs are available").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.rtw_abi_version() != ABI_VERSION:  # rtw_stats layout etc. must match this mirror
            raise RtwError(RTW_ESTATE, f"{LIB_PATH} has ABI {L.rtw_abi_version()}, this mirror {ABI_VERSION}")
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        raise RtwError(rc, lib().rtw_last_error().decode())


def _fa(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(-1))


def _ua(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint32).reshape(-1))


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_F)


def _up(a: np.ndarray):
    return a.ctypes.data_as(_U32)


def device_count() -> int:
    return int(lib().rtw_device_count())


class Camera:
    """Camera::new (camera.rs:25-64)."""

    def __init__(self, c: rtw_camera):
        self.c = c

    @classmethod
    def new(cls, look_from, look_at, vup, vfov, aspect, aperture, focus_dist, time0=0.0, time1=1.0):
        c = rtw_camera()
        _check(lib().rtw_camera_new(_fp(_fa(look_from)), _fp(_fa(look_at)), _fp(_fa(vup)), vfov, aspect,
                                    aperture, focus_dist, time0, time1, C.byref(c)))
        return cls(c)

    def as_dict(self) -> dict:
        return {k: (list(getattr(self.c, k)) if k not in ("lens_radius", "time0", "time1")
                    else float(getattr(self.c, k))) for k, _ in rtw_camera._fields_}


class Scene:
    """The world: Vec<Box<dyn Hittable>> plus its materials/textures, built by reference
    constructor names (include/rtw.h documents the file:line each one replaces)."""

    def __init__(self):
        p = C.c_void_p()
        _check(lib().rtw_scene_create(C.byref(p)))
        self._p = p
        self._keep = []

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.rtw_scene_destroy(self._p)
            self._p = None

    # textures ------------------------------------------------------------
    def _id(self, fn, *args) -> int:
        out = C.c_uint32()
        _check(fn(self._p, *args, C.byref(out)))
        return int(out.value)

    def solid_rgb(self, r, g, b) -> int:
        return self._id(lib().rtw_texture_solid, r, g, b)

    def checker(self, odd: int, even: int, frequency: float) -> int:
        return self._id(lib().rtw_texture_checker, odd, even, frequency)

    def image(self, rgb8: np.ndarray) -> int:
        a = np.ascontiguousarray(rgb8, dtype=np.uint8)
        h, w, _ = a.shape
        return self._id(lib().rtw_texture_image, a.ctypes.data_as(_U8), w, h)

    def uv_debug(self) -> int:
        return self._id(lib().rtw_texture_uvdebug)

    def noise(self, scale: float, perlin=None, seed: int = 0) -> int:
        """Noise::new(Perlin, scale) (texture.rs:83-95).  perlin = (gradients[256, 3],
        permutations[3, 256]); default Perlin::new with the build's seeded stream."""
        g, p = perlin if perlin is not None else perlin_generate(seed)
        g, p = _fa(g), _ua(p)
        return self._id(lib().rtw_texture_noise, _fp(g), _up(p), float(scale))

    # materials -----------------------------------------------------------
    def lambertian(self, tex: int) -> int:
        return self._id(lib().rtw_material_lambertian, tex)

    def lambertian_solid(self, rgb) -> int:
        return self.lambertian(self.solid_rgb(*rgb))

    def metal(self, albedo, fuzz) -> int:
        return self._id(lib().rtw_material_metal, albedo[0], albedo[1], albedo[2], fuzz)

    def dielectric(self, ir) -> int:
        return self._id(lib().rtw_material_dielectric, ir)

    def diffuse_light(self, tex: int) -> int:
        return self._id(lib().rtw_material_diffuse_light, tex)

    def isotropic(self, tex: int) -> int:
        return self._id(lib().rtw_material_isotropic, tex)

    # hierarchy -----------------------------------------------------------
    @contextlib.contextmanager
    def _group(self, rc):
        _check(rc)
        yield self
        _check(lib().rtw_end(self._p))

    def list(self):
        return self._group(lib().rtw_begin_list(self._p))

    def bvh(self, t0=0.0, t1=1.0):
        return self._group(lib().rtw_begin_bvh(self._p, t0, t1))

    def translate(self, offset):
        return self._group(lib().rtw_begin_translate(self._p, *[float(x) for x in offset]))

    def rotate_y(self, degrees):
        return self._group(lib().rtw_begin_rotate_y(self._p, float(degrees)))

    def constant_medium(self, density: float, tex: int):
        """ConstantMedium::new(boundary, density, texture) (volumes.rs:24-35): add the boundary
        (one Sphere or Cuboid, optionally translated / rotated) inside the `with` block."""
        return self._group(lib().rtw_begin_constant_medium(self._p, float(density), tex, None))

    # primitives ----------------------------------------------------------
    def spheres(self, centers, radii, mats) -> None:
        c = np.asarray(centers, np.float32).reshape(-1, 3)
        cx, cy, cz = (_fa(c[:, k]) for k in range(3))
        r, m = _fa(radii), _ua(mats)
        _check(lib().rtw_add_spheres(self._p, len(r), _fp(cx), _fp(cy), _fp(cz), _fp(r), _up(m)))

    def sphere(self, center, radius, mat) -> None:
        self.spheres([center], [radius], [mat])

    def moving_spheres(self, c0, t0, c1, t1, radii, mats) -> None:
        c0 = np.asarray(c0, np.float32).reshape(-1, 3)
        c1 = np.asarray(c1, np.float32).reshape(-1, 3)
        arrs = [_fa(c0[:, 0]), _fa(c0[:, 1]), _fa(c0[:, 2]), _fa(t0), _fa(c1[:, 0]), _fa(c1[:, 1]),
                _fa(c1[:, 2]), _fa(t1), _fa(radii)]
        m = _ua(mats)
        _check(lib().rtw_add_moving_spheres(self._p, len(m), *[_fp(a) for a in arrs], _up(m)))

    def moving_sphere(self, c0, t0, c1, t1, radius, mat) -> None:
        self.moving_spheres([c0], [t0], [c1], [t1], [radius], [mat])

    def rects(self, axis, a0, a1, b0, b1, k, mats) -> None:
        ax = _ua(axis)
        arrs = [_fa(a0), _fa(a1), _fa(b0), _fa(b1), _fa(k)]
        m = _ua(mats)
        _check(lib().rtw_add_rects(self._p, len(m), _up(ax), *[_fp(a) for a in arrs], _up(m)))

    def xy_rect(self, x0, x1, y0, y1, k, mat):
        self.rects([0], [x0], [x1], [y0], [y1], [k], [mat])

    def xz_rect(self, x0, x1, z0, z1, k, mat):
        self.rects([1], [x0], [x1], [z0], [z1], [k], [mat])

    def yz_rect(self, y0, y1, z0, z1, k, mat):
        self.rects([2], [y0], [y1], [z0], [z1], [k], [mat])

    def cuboid(self, p0, p1, mat) -> None:
        _check(lib().rtw_add_cuboid(self._p, _fp(_fa(p0)), _fp(_fa(p1)), mat))

    def triangles(self, verts, mat, normals=None, normal_mask=None, uvs=None, uv_mask=None) -> None:
        v = _fa(verts)
        n = len(v) // 9
        nn = _fa(normals) if normals is not None else None
        uu = _fa(uvs) if uvs is not None else None
        nm = np.ascontiguousarray(normal_mask, np.uint8) if normal_mask is not None else None
        um = np.ascontiguousarray(uv_mask, np.uint8) if uv_mask is not None else None
        _check(lib().rtw_add_triangles(
            self._p, n, _fp(v), _fp(nn) if nn is not None else None,
            nm.ctypes.data_as(_U8) if nm is not None else None, _fp(uu) if uu is not None else None,
            um.ctypes.data_as(_U8) if um is not None else None, mat))

    def load_wavefront_obj(self, path, material_override: int = NO_MATERIAL) -> int:
        n = C.c_uint32()
        _check(lib().rtw_load_wavefront_obj(self._p, str(path).encode(), None, material_override, C.byref(n)))
        return int(n.value)

    def preset(self, name: str, aspect: float, seed: int = 0, models_dir=None):
        """console_app/src/scenes.rs scene by subcommand name -> (Camera, background)."""
        cam = rtw_camera()
        bg = np.zeros(3, np.float32)
        md = str(models_dir or MODELS_DIR).encode()
        _check(lib().rtw_scene_preset(self._p, name.encode(), aspect, seed, md, C.byref(cam), _fp(bg)))
        return Camera(cam), tuple(float(x) for x in bg)

    def commit(self, device: int = -1) -> "Scene":
        _check(lib().rtw_scene_commit(self._p, device))
        return self

    # introspection -------------------------------------------------------
    def dump(self) -> str:
        need = C.c_size_t()
        _check(lib().rtw_scene_dump(self._p, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        _check(lib().rtw_scene_dump(self._p, buf, need.value, C.byref(need)))
        return buf.value.decode()

    def images(self) -> list:
        out, k = [], 0
        while True:
            px, w, h = _U8(), C.c_uint32(), C.c_uint32()
            if lib().rtw_scene_image(self._p, k, C.byref(px), C.byref(w), C.byref(h)) != 0:
                return out
            out.append(np.ctypeslib.as_array(px, shape=(h.value * w.value * 3,)).copy())
            k += 1

    def path_kernel_times(self, device: int = -1, max_n: int = 64) -> list:
        """Device ms of the recent path-kernel launches on `device` (oldest first; waits for them)."""
        buf = (C.c_float * max_n)()
        n = lib().rtw_path_kernel_times(self._p, device, buf, max_n)
        if n < 0:
            _check(n)
        return [float(buf[q]) for q in range(n)]

    def multi_times(self, max_n: int = 64):
        """(per-device render ms, device 0's gather ms) of the last rtw_render_multi call on this scene."""
        buf, g = (C.c_float * max_n)(), C.c_float()
        n = lib().rtw_render_multi_times(self._p, buf, max_n, C.byref(g))
        if n < 0:
            _check(n)
        return [float(buf[q]) for q in range(min(n, max_n))], float(g.value)

    def render_status(self, device: int = -1) -> None:
        """Wait for the device and raise if a render since the last check tripped the traversal guard."""
        _check(lib().rtw_render_status(self._p, device))

    def diag_corrupt_bvh(self, device: int = -1) -> None:
        """Test hook: a cyclic BVH on the device copy (every render of it trips the guard)."""
        _check(lib().rtw_diag_corrupt_bvh(self._p, device))

    def diag_alias_devices(self, n: int) -> "Scene":
        """Test hook (before commit): n logical devices on physical device 0, so rtw_render_multi's n > 1
        path runs on one GPU (with the loopback RCCL of tests/loopback_rccl via RTW_RCCL_LIB)."""
        _check(lib().rtw_diag_alias_devices(self._p, int(n)))
        return self

    def info(self, what: int) -> int:
        return int(lib().rtw_scene_info(self._p, what))

    def nodes(self) -> np.ndarray:
        """The flattened BVH4 (DevNode4 records, rtw_device.hpp) as a structured array (a copy)."""
        p, n = C.c_void_p(), C.c_uint32()
        _check(lib().rtw_scene_nodes(self._p, C.byref(p), C.byref(n)))
        dt = np.dtype([("lo_x", "<f4", 4), ("hi_x", "<f4", 4), ("lo_y", "<f4", 4), ("hi_y", "<f4", 4),
                       ("lo_z", "<f4", 4), ("hi_z", "<f4", 4), ("child", "<i4", 4), ("code", "<u4", 4)])
        if not n.value:
            return np.zeros(0, dt)
        buf = (C.c_uint8 * (128 * n.value)).from_address(p.value)
        return np.frombuffer(bytes(buf), dtype=dt).copy()


    def nodes_half(self) -> np.ndarray:
        """The half-precision BVH4 (DevNode4h, rtw_device.hpp) as a structured array (a copy; empty when
        the 16-bit codes do not fit).  Planes are f16 offsets from `origin`: x[0] = lo x4, hi x4 and x[1] =
        hi x4, lo x4 (likewise y, z)."""
        p, n = C.c_void_p(), C.c_uint32()
        _check(lib().rtw_scene_nodes_half(self._p, C.byref(p), C.byref(n)))
        dt = np.dtype([("x", "<f2", (2, 8)), ("y", "<f2", (2, 8)), ("z", "<f2", (2, 8)), ("code", "<u2", 4),
                       ("origin", "<f2", 3), ("pad", "<u2")])
        assert dt.itemsize == 112
        if not n.value:
            return np.zeros(0, dt)
        buf = (C.c_uint8 * (112 * n.value)).from_address(p.value)
        return np.frombuffer(bytes(buf), dtype=dt).copy()


class Raytracer:
    """Raytracer::new(world, cam, background, w, h, spp) (lib.rs:40-48) + render() (:57-95)."""

    def __init__(self, scene: Scene, cam: Camera, background, image_width: int, image_height: int,
                 samples_per_pixel: int, seed: int = 0, max_depth: int = 50):
        self.scene, self.cam = scene, cam
        self.bg = _fa(background)
        self.w, self.h, self.spp = int(image_width), int(image_height), int(samples_per_pixel)
        self.seed, self.max_depth = int(seed), int(max_depth)

    def render(self):
        """-> (sums[h, w, 3] float32 in reference emission order: row r is j = h-1-r, stats)."""
        out = np.empty((self.h, self.w, 3), np.float32)
        st = rtw_stats()
        _check(lib().rtw_render(self.scene._p, C.byref(self.cam.c), _fp(self.bg), self.w, self.h, self.spp,
                                self.max_depth, self.seed, out.ctypes.data_as(_F), C.byref(st)))
        return out, st.as_dict()

    def render_multi(self, n_gpus: int = 0):
        """The same frame over n_gpus devices from this thread (rtw_render_multi: interleaved tiles,
        one RCCL gather to device 0); n_gpus <= 0 = every visible device.  -> (sums, stats)."""
        out = np.empty((self.h, self.w, 3), np.float32)
        st = rtw_stats()
        _check(lib().rtw_render_multi(self.scene._p, int(n_gpus), C.byref(self.cam.c), _fp(self.bg), self.w, self.h,
                                      self.spp, self.max_depth, self.seed, out.ctypes.data_as(_F), C.byref(st)))
        return out, st.as_dict()

    def render_stream(self, on_pixels, band_rows: int = 64):
        """Raytracer::render() as a progressive Pixel stream (lib.rs:50-76): on_pixels(array of
        PIXEL_DTYPE records) per finished band, in emission order (row j = h-1 .. 0).  -> stats."""
        err = []

        def sink(px, n, _user):
            try:
                buf = C.string_at(px, n * C.sizeof(rtw_pixel))
                on_pixels(np.frombuffer(buf, PIXEL_DTYPE).copy())
                return 0
            except Exception as e:  # stop the render, re-raise below
                err.append(e)
                return RTW_ESTATE

        cb = PIXEL_SINK(sink)
        st = rtw_stats()
        rc = lib().rtw_render_stream(self.scene._p, C.byref(self.cam.c), _fp(self.bg), self.w, self.h, self.spp,
                                     self.max_depth, self.seed, band_rows, cb, None, C.byref(st))
        if err:
            raise err[0]
        _check(rc)
        return st.as_dict()

    def render_device(self, d_out_ptr: int, device: int = 0, d_tiles_ptr: int = 0, n_tiles: int = 0,
                      stream_ptr: int = 0, flags: int = 0, want_stats: bool = False):
        """Enqueue into device memory.  d_tiles_ptr: device uint32 tile ids (0 = whole image,
        full-layout output); with tiles the output is packed [n_tiles][64][3]."""
        st = rtw_stats()
        _check(lib().rtw_render_device(
            self.scene._p, device, C.byref(self.cam.c), _fp(self.bg), self.w, self.h, self.spp, self.max_depth,
            self.seed, C.cast(C.c_void_p(d_tiles_ptr), _U32) if d_tiles_ptr else None, n_tiles,
            C.c_void_p(d_out_ptr), C.c_void_p(stream_ptr), flags, C.byref(st) if want_stats else None))
        return st.as_dict() if want_stats else None

    def render_device_strided(self, d_out_ptr: int, device: int, first_tile: int, tile_stride: int, n_tiles: int,
                              stream_ptr: int = 0, flags: int = 0, want_stats: bool = False):
        """Enqueue tiles first_tile + k * tile_stride (k < n_tiles) into packed device memory
        [n_tiles][64][3] (a device's round-robin share of the frame, no id table)."""
        st = rtw_stats()
        _check(lib().rtw_render_device_strided(
            self.scene._p, device, C.byref(self.cam.c), _fp(self.bg), self.w, self.h, self.spp, self.max_depth,
            self.seed, first_tile, tile_stride, n_tiles, C.c_void_p(d_out_ptr), C.c_void_p(stream_ptr), flags,
            C.byref(st) if want_stats else None))
        return st.as_dict() if want_stats else None


def progress_encode(kind: int, width=0, height=0, spp=0, pixel=None) -> bytes:
    """postcard::to_vec_cobs(&ProgressMessage) (lib.rs:128-138): COBS frame incl. its 0x00."""
    m = rtw_progress_msg(kind=kind, width=width, height=height, samples_per_pixel=spp)
    if pixel is not None:
        m.pixel.row, m.pixel.column = int(pixel[0]), int(pixel[1])
        m.pixel.color[:] = [float(x) for x in pixel[2]]
    out = (C.c_uint8 * 64)()
    n = C.c_size_t()
    _check(lib().rtw_progress_encode(C.byref(m), out, 64, C.byref(n)))
    return bytes(out[:n.value])


def progress_decode(frame: bytes) -> dict:
    """postcard::from_bytes_cobs::<ProgressMessage> (discovery_host_receiver/src/main.rs:37)."""
    buf = (C.c_uint8 * max(1, len(frame))).from_buffer_copy(frame or b"\0")
    m = rtw_progress_msg()
    _check(lib().rtw_progress_decode(buf, len(frame), C.byref(m)))
    d = {"kind": int(m.kind)}
    if m.kind == MSG_IMAGE_START:
        d.update(width=int(m.width), height=int(m.height), samples_per_pixel=int(m.samples_per_pixel))
    elif m.kind == MSG_PIXEL:
        d.update(row=int(m.pixel.row), column=int(m.pixel.column), color=[float(x) for x in m.pixel.color])
    return d


def perlin_generate(seed: int = 0):
    """Perlin::new(rng) (perlin.rs:14-48) with the build's seeded stream -> (grad[256, 3], perm[3, 256])."""
    g = np.zeros(768, np.float32)
    p = np.zeros(768, np.uint32)
    _check(lib().rtw_perlin_generate(seed, _fp(g), _up(p)))
    return g.reshape(256, 3), p.reshape(3, 256)


def preset_cameras(name: str, aspect: float, models_dir=None) -> list:
    """Every camera of a preset (scenes.rs World's Vec<Camera>): 30 for animated-book2-final-scene."""
    n = C.c_uint32()
    md = str(models_dir or MODELS_DIR).encode()
    _check(lib().rtw_preset_cameras(name.encode(), aspect, md, None, 0, C.byref(n)))
    cams = (rtw_camera * max(1, n.value))()
    _check(lib().rtw_preset_cameras(name.encode(), aspect, md, cams, n.value, C.byref(n)))
    return [Camera(cams[k]) for k in range(n.value)]


def unpack_tiles_device(w, h, d_tiles_ptr, n_tiles, d_packed_ptr, d_image_ptr, device=-1, stream_ptr=0):
    _check(lib().rtw_unpack_tiles_device(device, w, h, C.c_void_p(d_tiles_ptr), n_tiles, C.c_void_p(d_packed_ptr),
                                         C.c_void_p(d_image_ptr), C.c_void_p(stream_ptr)))


def diag_libm(fn: int, a, b=None) -> np.ndarray:
    """Device f32 transcendentals (0 log10f, 1 sinf, 2 acosf, 3 atan2f(a, b)) and the camera's
    division (4: a / b by Markstein's correction from RN(1 / b)) and the sphere test's sqrt (5) over
    host arrays."""
    a = _fa(a)
    bb = _fa(b) if b is not None else None
    out = np.empty_like(a)
    _check(lib().rtw_diag_libm(fn, len(a), _fp(a), _fp(bb) if bb is not None else None, _fp(out)))
    return out


def diag_sweep(fn: int, lo: int = 0, hi: int = 0xFFFFFFFF, cap: int = 64):
    """Device fast path vs the IEEE operation over every bit pattern in [lo, hi] (fn 0: reciprocal)
    -> (mismatches, skipped, first mismatching patterns)."""
    counts = (C.c_uint64 * 2)()
    bad = np.zeros(max(1, cap), np.uint32)
    _check(lib().rtw_diag_sweep(fn, lo, hi, counts, _up(bad), cap))
    return int(counts[0]), int(counts[1]), bad[:min(cap, int(counts[0]))]


def diag_recip(b) -> np.ndarray:
    """The host's RN(1 / b) behind the camera divisions (no device needed)."""
    b = _fa(b)
    out = np.empty_like(b)
    _check(lib().rtw_diag_recip(len(b), _fp(b), _fp(out)))
    return out


def tile_partition(w: int, h: int, n_parts: int, part: int):
    """rtw_tile_partition -> (padded ids of the part [ceil(nt / n_parts)], number of real ids)."""
    nt = n_tiles(w, h)
    per = (nt + n_parts - 1) // n_parts if n_parts > 0 else 0
    ids = np.zeros(max(1, per), np.uint32)
    n = C.c_uint32()
    _check(lib().rtw_tile_partition(w, h, n_parts, part, _up(ids), per, C.byref(n)))
    return ids[:per], int(n.value)


def n_tiles(w: int, h: int) -> int:
    return ((w + 7) // 8) * ((h + 7) // 8)


def tonemap(sums: np.ndarray, spp: int) -> np.ndarray:
    """console_app/src/main.rs:68-90 -> uint8 image of the same shape."""
    s = np.ascontiguousarray(sums, np.float32)
    out = np.empty(s.shape, np.uint8)
    _check(lib().rtw_tonemap(_fp(s.reshape(-1)), s.size // 3, spp, out.ctypes.data_as(_U8)))
    return out


def image_height(width: int, aspect: float = 1.7777778) -> int:
    """console_app/src/main.rs:33: (width as f64 / aspect).round() as u32 (ties away from zero)."""
    import math
    x = width / aspect
    return int(math.floor(x + 0.5))


def camera_aspect(width: int, height: int) -> float:
    """console_app/src/main.rs:39: (w as f32) / (h as f32)."""
    return float(np.float32(width) / np.float32(height))
