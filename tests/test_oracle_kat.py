"""Analytic known-answer tests of the oracle, each derived from a cited reference line."""
import ctypes as C
import math

import numpy as np


def hit(orc, kind, par, ray, tmin=0.001, tmax=np.inf):
    out = np.zeros(10, np.float32)
    h = orc.lib().oracle_hit_primitive(kind, orc.fp(orc.f32(par)), orc.fp(orc.f32(ray)), tmin, tmax, orc.fp(out))
    return h, out


def scatter(orc, kind, params, ray, rec, draws):
    out = np.zeros(6, np.float32)
    used = C.c_uint32()
    dr = np.ascontiguousarray(draws, np.uint32)
    ok = orc.lib().oracle_scatter(kind, orc.fp(orc.f32(params)), orc.fp(orc.f32(ray)), orc.fp(orc.f32(rec)),
                                  dr.ctypes.data_as(C.POINTER(C.c_uint32)), len(dr), orc.fp(out), C.byref(used))
    return ok, out, used.value


def test_camera_center_ray_aperture0(orc):
    """camera.rs:41-48,66-71: with aperture 0 the centre ray points from look_from to look_at."""
    c = orc.camera_new((278, 278, -800), (278, 278, 0), (0, 1, 0), 40, 1.0, 0.0, 10.0)
    out = np.zeros(7, np.float32)
    used = C.c_uint32()
    draws = np.array([0x80000000, 0x80000000, 0x80000000], np.uint32)  # disk (0,0); time 0.5
    orc.lib().oracle_get_ray(C.byref(c), 0.5, 0.5, draws.ctypes.data_as(C.POINTER(C.c_uint32)), 3, orc.fp(out),
                             C.byref(used))
    d = out[3:6]
    assert abs(d[0]) < 1e-4 and abs(d[1]) < 1e-4 and d[2] > 0
    assert used.value == 3 and abs(out[6] - 0.5) < 1e-6  # disk drawn although aperture == 0


def test_sphere_near_and_far_root(orc):
    """spherical.rs:37-44: nearer root first, else the farther one (origin inside)."""
    h, o = hit(orc, 0, (0, 0, 5, 1), (0, 0, 0, 0, 0, 1, 0))
    assert h and o[0] == 4.0 and o[9] == 1.0  # front face, t = 4
    h, o = hit(orc, 0, (0, 0, 0, 1), (0, 0, 0, 0, 0, 1, 0))
    assert h and o[0] == 1.0 and o[9] == 0.0 and o[6] == -1.0  # inside: back face, normal flipped
    h, o = hit(orc, 0, (0, 0, 5, 1), (0, 0, 0, 0, 0, 1, 0), tmax=3.9)
    assert not h  # both roots beyond t_max


def test_negative_radius_flips_normal(orc):
    """spherical.rs:49 divides by radius: r < 0 makes the outward normal point inwards."""
    h, o = hit(orc, 0, (0, 0, 5, -1), (0, 0, 0, 0, 0, 1, 0))
    assert h and o[0] == 4.0 and o[9] == 0.0 and o[6] == -1.0


def test_rect_closed_bounds(orc):
    """rectangular.rs:40: x < x0 || x > x1 rejects, so the edges themselves hit."""
    for x in (-1.0, 1.0):
        h, o = hit(orc, 2, (0, -1, 1, -1, 1, 0), (x, 0, -2, 0, 0, 1, 0))
        assert h and o[0] == 2.0
    h, _ = hit(orc, 2, (0, -1, 1, -1, 1, 0), (1.0001, 0, -2, 0, 0, 1, 0))
    assert not h


def test_triangle_edge_and_default_uv(orc):
    """triangular.rs:118 u + v <= 1 accepts the hypotenuse; :57-61 default uvs (0,0),(1,0),(0,1)."""
    tri = (0, 0, 0, 1, 0, 0, 0, 1, 0)
    h, o = hit(orc, 3, tri, (0.5, 0.5, 1, 0, 0, -1, 0))
    assert h and o[0] == 1.0
    assert abs(o[7] - 0.5) < 1e-7 and abs(o[8] - 0.5) < 1e-7  # uv = barycentric (u, v)
    h, _ = hit(orc, 3, tri, (0.51, 0.5, 1, 0, 0, -1, 0))
    assert not h


def test_schlick_normal_incidence(orc):
    """material.rs:108-112: reflectance(cos=1, 1.5) = r0 = 0.04 -> a draw < 0.04 reflects."""
    rec = (0, 0, 0, 0, 0, 1, 1)  # p, n, front
    ray = (0, 0, 1, 0, 0, -1, 0)
    params = (1, 1, 1, 1.5)
    # draw 0.03 * 2^32 -> gen_f32 ~ 0.03 < 0.0400 -> reflect
    ok, out, used = scatter(orc, 2, params, ray, rec, [int(0.03 * 2 ** 32)])
    assert ok and used == 1 and out[2] > 0
    ok, out, used = scatter(orc, 2, params, ray, rec, [int(0.05 * 2 ** 32)])
    assert ok and used == 1 and out[2] < 0  # refracted straight through


def test_total_internal_reflection_draws_nothing(orc):
    """material.rs:126-130: cannot_refract short-circuits, so no uniform is drawn."""
    s = math.sin(math.radians(60))
    ray = (0, 0, 0, s, 0, -math.cos(math.radians(60)), 0)
    rec = (0, 0, 0, 0, 0, 1, 0)  # back face: ratio = ir = 1.5, 1.5 * sin60 > 1
    ok, out, used = scatter(orc, 2, (1, 1, 1, 1.5), ray, rec, [0])
    assert ok and used == 0 and out[2] > 0


def test_metal_absorbs_below_surface(orc):
    """material.rs:87: scattered . n <= 0 -> None; the sphere sample is drawn even for fuzz 0."""
    ray = (0, 0, 1, 0, 0, -1, 0)
    rec = (0, 0, 0, 0, 0, 1, 1)
    ok, out, used = scatter(orc, 1, (0.5, 0.5, 0.5, 0.0), ray, rec, [0x80000000] * 3)
    assert ok and used == 3 and out[2] > 0
    ok, out, used = scatter(orc, 1, (0.5, 0.5, 0.5, 1.0), (0, 0, 1, 1, 0, -1e-3, 0), rec,
                            [0x80000000, 0x80000000, 0x40000000])  # fuzz (0,0,-0.5) pulls below
    assert not ok


def test_lambertian_rejection_draw_counts(orc):
    """vec3.rs:101-108: rejection in the cube; a point outside the sphere costs 3 more draws."""
    ray = (0, 0, 1, 0, 0, -1, 0)
    rec = (0, 0, 0, 0, 0, 1, 1)
    big = 0xFFFFFFFF  # -> ~ +1 on every axis: |p|^2 ~ 3 > 1, rejected
    ok, out, used = scatter(orc, 0, (0.5, 0.5, 0.5, 0), ray, rec, [big, big, big, 0x80000000, 0x80000000,
                                                                   0xC0000000])
    assert ok and used == 6


def test_aabb_parallel_ray_nan_semantics(orc):
    """aabb.rs:29-44 with Rust max/min (NaN ignored): a ray parallel to a slab and exactly on
    its face does not by itself reject the box."""
    L = orc.lib()
    inside = L.oracle_aabb_hit(orc.fp(orc.f32((0, 0, 0))), orc.fp(orc.f32((1, 1, 1))),
                               orc.fp(orc.f32((0, 0.5, -1, 0, 0, 1, 0))), 0.001, np.inf)
    outside = L.oracle_aabb_hit(orc.fp(orc.f32((0, 0, 0))), orc.fp(orc.f32((1, 1, 1))),
                                orc.fp(orc.f32((-0.5, 0.5, -1, 0, 0, 1, 0))), 0.001, np.inf)
    assert inside == 1 and outside == 0


def test_tonemap_edges(orc):
    """console_app/src/main.rs:78-88: NaN -> 0 (as u8 saturates), clamp at 0.999 -> 255."""
    L = orc.lib()
    assert L.oracle_tonemap(float("nan"), 10) == 0
    assert L.oracle_tonemap(-5.0, 10) == 0
    assert L.oracle_tonemap(1e9, 10) == 255
    assert L.oracle_tonemap(10.0, 10) == 255  # sqrt(1) clamps to 0.999 -> 255.74 -> 255
    assert L.oracle_tonemap(2.5, 10) == 127  # sqrt(0.25) * 255.999 = 127.99


def test_checker_sign_fast_path_sample():
    """The kernel decides Checker (texture.rs:69-81) by the parity of floor(x/pi) for
    2^-12 <= |x| < 65536; oracle/tools/sin_sign_check.c proves it exhaustively against libm's
    sinf.  This re-checks a random sample (plus values next to multiples of pi) on every run."""
    libm = C.CDLL("libm.so.6")
    libm.sinf.restype = C.c_float
    libm.sinf.argtypes = [C.c_float]
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-65536, 65536, 100000),
                         np.exp(rng.uniform(np.log(2.0 ** -12), np.log(65536.0), 50000)),
                         np.pi * np.arange(1, 20000)]).astype(np.float32)
    xs = xs[(np.abs(xs) >= 2.0 ** -12) & (np.abs(xs) < 65536)]
    nb = np.nextafter(xs, np.float32(np.inf)).astype(np.float32)
    for arr in (xs, nb):
        par = np.floor(arr.astype(np.float64) * 0.31830988618379067154).astype(np.int64) & 1
        sgn = np.array([libm.sinf(float(x)) < 0 for x in arr])
        assert np.array_equal(par.astype(bool), sgn)


def test_pm1_never_retries():
    """gen_range(-1, 1) (UniformFloat::sample_single) never takes its retry branch: the kernel's
    gen_pm1 relies on it.  Every 23-bit mantissa draw, evaluated in f32 as mul-then-add."""
    m = np.arange(1 << 23, dtype=np.uint32)
    v01 = ((m | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)).astype(np.float32)
    r = (v01 * np.float32(2.0)).astype(np.float32) + np.float32(-1.0)
    assert r.dtype == np.float32
    assert float(r.max()) < 1.0 and float(r.min()) == -1.0
