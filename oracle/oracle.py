"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline, never by the product.
See rtw_oracle.c's header for what it restates and its parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "_build" / "liboracle.so"

ITERATIVE, RECURSIVE = 0, 1
BVH_AS_LIST, BVH_REFERENCE = 0, 1


class oracle_camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("lower_left_corner", C.c_float * 3),
                ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3),
                ("u", C.c_float * 3), ("v", C.c_float * 3), ("w", C.c_float * 3),
                ("lens_radius", C.c_float), ("time0", C.c_float), ("time1", C.c_float)]


_F = C.POINTER(C.c_float)
_U32 = C.POINTER(C.c_uint32)
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        sig = {
            "oracle_scene_parse": (C.c_void_p, [C.c_char_p, C.POINTER(C.c_void_p), C.c_int]),
            "oracle_scene_free": (None, [C.c_void_p]),
            "oracle_last_error": (C.c_char_p, []),
            "oracle_scene_count": (C.c_int, [C.c_void_p, C.c_int]),
            "oracle_camera_new": (None, [_F, _F, _F, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                         C.c_float, C.POINTER(oracle_camera)]),
            "oracle_render": (C.c_int, [C.c_void_p, C.POINTER(oracle_camera), _F, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_int, _U32,
                                        C.c_uint32, _F, C.POINTER(C.c_uint64)]),
            "oracle_render_counts": (C.c_int, [C.c_void_p, C.POINTER(oracle_camera), _F, C.c_uint32, C.c_uint32,
                                               C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_int, _U32,
                                               C.c_uint32, _F, C.POINTER(C.c_uint64), _U32]),
            "oracle_render_pixels": (C.c_int, [C.c_void_p, C.POINTER(oracle_camera), _F, C.c_uint32, C.c_uint32,
                                               C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_int, _U32,
                                               C.c_uint32, _F, C.POINTER(C.c_uint64)]),
            "oracle_pcg32_stream": (C.c_uint32, [C.c_uint64, C.c_uint32, _U32, C.POINTER(C.c_uint64)]),
            "oracle_rng_stream": (C.c_uint32, [C.c_uint64, C.c_uint32, _U32, C.POINTER(C.c_uint64)]),
            "oracle_splitmix64": (C.c_uint64, [C.c_uint64]),
            "oracle_path_state": (C.c_uint64, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]),
            "oracle_u32_to_f32": (C.c_float, [C.c_uint32]),
            "oracle_u32_to_range": (C.c_float, [C.c_uint32, C.c_float, C.c_float]),
            "oracle_u64_to_f64": (C.c_double, [C.c_uint64]),
            "oracle_sphere_uv": (None, [_F, _F]),
            "oracle_hit_primitive": (C.c_int, [C.c_int, _F, _F, C.c_float, C.c_float, _F]),
            "oracle_aabb_hit": (C.c_int, [_F, _F, _F, C.c_float, C.c_float]),
            "oracle_scatter": (C.c_int, [C.c_int, _F, _F, _F, _U32, C.c_uint32, _F, _U32]),
            "oracle_get_ray": (None, [C.POINTER(oracle_camera), C.c_float, C.c_float, _U32, C.c_uint32, _F,
                                      _U32]),
            "oracle_tonemap": (C.c_uint8, [C.c_float, C.c_uint32]),
            "oracle_libm": (C.c_int, [C.c_int, C.c_uint32, _F, _F, _F]),
            "oracle_medium_hit": (C.c_int, [C.c_int, _F, C.c_float, _F, C.c_float, C.c_float, C.c_uint64,
                                            C.c_uint32, _F]),
            "oracle_noise": (C.c_float, [_F, C.POINTER(C.c_int32), _F, C.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def f32(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1))


def fp(a: np.ndarray):
    return a.ctypes.data_as(_F)


def camera_new(look_from, look_at, vup, vfov, aspect, aperture, focus, t0=0.0, t1=1.0) -> oracle_camera:
    c = oracle_camera()
    lib().oracle_camera_new(fp(f32(look_from)), fp(f32(look_at)), fp(f32(vup)), vfov, aspect, aperture,
                            focus, t0, t1, C.byref(c))
    return c


def camera_from_fields(d: dict) -> oracle_camera:
    c = oracle_camera()
    for k, _ in oracle_camera._fields_:
        v = d[k]
        if isinstance(v, (list, tuple)):
            getattr(c, k)[:] = [float(x) for x in v]
        else:
            setattr(c, k, float(v))
    return c


class OracleScene:
    """A scene parsed from rtw_scene_dump() text (+ image texture buffers)."""

    def __init__(self, text: str, images=()):
        self._imgs = [np.ascontiguousarray(i, np.uint8) for i in images]
        arr = (C.c_void_p * max(1, len(self._imgs)))(*[i.ctypes.data for i in self._imgs])
        self._p = lib().oracle_scene_parse(text.encode(), arr, len(self._imgs))
        if not self._p:
            raise RuntimeError(lib().oracle_last_error().decode())

    def __del__(self):
        if getattr(self, "_p", None):
            lib().oracle_scene_free(self._p)
            self._p = None

    def count(self, what: int) -> int:
        return lib().oracle_scene_count(self._p, what)

    def render(self, cam: oracle_camera, background, w, h, spp, seed=0, max_depth=50,
               integrator=ITERATIVE, bvh_mode=BVH_AS_LIST, threads=None, rows=None, pixel_rays=False):
        """-> (sums[h, w, 3] in reference order, rays[, per-pixel rays[h, w] when pixel_rays]).
        rows: list of j (bottom-based) to render."""
        out = np.zeros((h, w, 3), np.float32)
        rays = C.c_uint64()
        pr = np.zeros((h, w), np.uint32) if pixel_rays else None
        r = np.ascontiguousarray(rows, np.uint32) if rows is not None else None
        n = threads or min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16
        rc = lib().oracle_render_counts(self._p, C.byref(cam), fp(f32(background)), w, h, spp, max_depth, seed,
                                        integrator, bvh_mode, n, r.ctypes.data_as(_U32) if r is not None else None,
                                        len(r) if r is not None else 0, fp(out), C.byref(rays),
                                        pr.ctypes.data_as(_U32) if pr is not None else None)
        if rc != 0:
            raise RuntimeError(lib().oracle_last_error().decode())
        return (out, int(rays.value), pr) if pixel_rays else (out, int(rays.value))

    def render_pixels(self, cam: oracle_camera, background, w, h, spp, pixels, seed=0, max_depth=50,
                      integrator=ITERATIVE, bvh_mode=BVH_AS_LIST, threads=None):
        """-> (sums[n, 3], rays) of the given (j, i) pixels (j bottom-based), in their order."""
        px = np.ascontiguousarray(np.asarray(pixels, np.uint32).reshape(-1, 2))
        out = np.zeros((len(px), 3), np.float32)
        rays = C.c_uint64()
        n = threads or min(16, os.cpu_count() or 1)
        rc = lib().oracle_render_pixels(self._p, C.byref(cam), fp(f32(background)), w, h, spp, max_depth, seed,
                                        integrator, bvh_mode, n, px.ctypes.data_as(_U32), len(px), fp(out),
                                        C.byref(rays))
        if rc != 0:
            raise RuntimeError(lib().oracle_last_error().decode())
        return out, int(rays.value)


def libm(fn: int, a, b=None) -> np.ndarray:
    """The oracle's f32 transcendentals (0 log10f, 1 sinf, 2 acosf, 3 atan2f(a, b))."""
    a = f32(a)
    bb = f32(b) if b is not None else None
    out = np.empty_like(a)
    if lib().oracle_libm(fn, len(a), fp(a), fp(bb) if bb is not None else None, fp(out)) != 0:
        raise ValueError(fn)
    return out


def noise(grad, perm, p, depth: int = 7) -> float:
    """perlin.rs noise (depth 0) / turbulence(p, depth) over explicit tables."""
    g = f32(grad)
    pm = np.ascontiguousarray(np.asarray(perm, np.int32).reshape(-1))
    return float(lib().oracle_noise(fp(g), pm.ctypes.data_as(C.POINTER(C.c_int32)), fp(f32(p)), depth))
