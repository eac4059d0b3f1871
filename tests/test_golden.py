"""The C oracle vs the independent numpy restatement's golden vectors (tests/golden/).

Everything here is bit-exact: both sides evaluate the reference's f32 expressions in the
same order without FMA, so any difference is a restatement bug on one side.
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

G = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_rng_streams_and_path_keys(orc):
    """The scene stream (PCG32), the per-path stream (xoroshiro64*) and the path keys."""
    L = orc.lib()
    for s, first, stream in zip(G["pcg_state"], G["pcg_out"], G["pcg_stream"]):
        out = (C.c_uint32 * 8)()
        L.oracle_pcg32_stream(int(s), 8, out, None)
        assert list(out) == [int(x) for x in stream]
        assert int(first[0]) == int(stream[0])
    for s, stream in zip(G["xoro_state"], G["xoro_stream"]):
        out = (C.c_uint32 * 8)()
        L.oracle_rng_stream(int(s), 8, out, None)
        assert list(out) == [int(x) for x in stream]
    # xoroshiro64*'s published first outputs for the state s0 = 1, s1 = 0: 0x9E3779BB, then
    # s0' = rotl(1, 26) ^ 1 ^ (1 << 9) -> result s0' * 0x9E3779BB
    out = (C.c_uint32 * 2)()
    L.oracle_rng_stream(1, 2, out, None)
    s0 = ((1 << 26) ^ 1 ^ (1 << 9)) & 0xFFFFFFFF
    assert list(out) == [0x9E3779BB, (s0 * 0x9E3779BB) & 0xFFFFFFFF]
    for key, want in zip(G["path_keys"], G["path_state"]):
        assert L.oracle_path_state(*[int(k) for k in key]) == int(want)


def test_rand_float_conversions(orc):
    """rand 0.9 Standard<f32> and UniformFloat::sample_single (one draw each)."""
    L = orc.lib()
    for u, f, m11, h in zip(G["u32"], G["u32_f32"], G["u32_m11"], G["u32_05"]):
        assert bits(L.oracle_u32_to_f32(int(u))) == bits(f)
        assert bits(L.oracle_u32_to_range(int(u), -1.0, 1.0)) == bits(m11)
        assert bits(L.oracle_u32_to_range(int(u), 0.0, 0.5)) == bits(h)
    assert L.oracle_u32_to_f32(0xFFFFFFFF) < 1.0
    assert L.oracle_u32_to_range(0xFFFFFFFF, -1.0, 1.0) < 1.0


def test_sphere_uv_reference_kat(orc):
    """hittable/spherical.rs:66-68 — the reference's own known-answer table."""
    table = {(1, 0, 0): (0.50, 0.50), (-1, 0, 0): (0.00, 0.50), (0, 1, 0): (0.50, 1.00),
             (0, -1, 0): (0.50, 0.00), (0, 0, 1): (0.25, 0.50), (0, 0, -1): (0.75, 0.50)}
    for p, want in table.items():
        uv = (C.c_float * 2)()
        orc.lib().oracle_sphere_uv(orc.fp(orc.f32(p)), uv)
        assert np.allclose(list(uv), want, atol=1e-6), (p, list(uv))
    for p, want in zip(G["uv_pts"], G["uv_out"]):
        uv = (C.c_float * 2)()
        orc.lib().oracle_sphere_uv(orc.fp(orc.f32(p)), uv)
        assert np.array_equal(bits(list(uv)), bits(want))


@pytest.mark.parametrize("name", ["sphere", "hollow", "msphere", "rect_xy", "rect_xz", "rect_yz", "tri"])
def test_primitive_hits(orc, name):
    kind = int(G[f"prim_{name}_kind"][0])
    par = orc.f32(G[f"prim_{name}_par"])
    want = G[f"prim_{name}_out"]
    n_hit = 0
    for r, w in zip(G["rays"], want):
        out = np.zeros(10, np.float32)
        hit = orc.lib().oracle_hit_primitive(kind, orc.fp(par), orc.fp(orc.f32(r)), 0.001, np.inf, orc.fp(out))
        assert hit == int(w[0])
        if hit:
            n_hit += 1
            assert np.array_equal(bits(out), bits(w[1:])), (name, r, out, w)
    assert n_hit > 10  # the ray set exercises hits, not only misses


def test_aabb_slab(orc):
    for b, r, w in zip(G["aabb_boxes"], G["aabb_rays"], G["aabb_out"]):
        got = orc.lib().oracle_aabb_hit(orc.fp(orc.f32(b[:3])), orc.fp(orc.f32(b[3:])), orc.fp(orc.f32(r)),
                                        0.001, np.inf)
        assert bool(got) == bool(w)


def test_scatter(orc):
    for row, draws, w in zip(G["scatter_in"], G["scatter_draws"], G["scatter_out"]):
        kind, front = int(row[0]), row[1]
        params, d_in, p, n = row[2:6], row[6:9], row[9:12], row[12:15]
        ray = orc.f32(list(p) + list(d_in) + [0.5])
        rec = orc.f32(list(p) + list(n) + [front])
        out = np.zeros(6, np.float32)
        used = C.c_uint32()
        dr = np.ascontiguousarray(draws, np.uint32)
        ok = orc.lib().oracle_scatter(kind, orc.fp(orc.f32(params)), orc.fp(ray), orc.fp(rec),
                                      dr.ctypes.data_as(C.POINTER(C.c_uint32)), len(dr), orc.fp(out),
                                      C.byref(used))
        assert ok == int(w[0]) and used.value == int(w[1])
        assert np.array_equal(bits(out), bits(w[2:8])), (kind, out, w[2:8])


def test_camera_and_get_ray(orc):
    cams = []
    for args, fields in zip(G["cam_args"], G["cam_fields"]):
        c = orc.camera_new(args[0:3], args[3:6], args[6:9], args[9], args[10], args[11], args[12])
        got = np.concatenate([list(getattr(c, k)) for k in ("origin", "lower_left_corner", "horizontal",
                                                             "vertical", "u", "v", "w")]
                             + [[c.lens_radius, c.time0, c.time1]]).astype(np.float32)
        assert np.array_equal(bits(got), bits(fields))
        cams.append(c)
    for row, draws in zip(G["get_ray"], G["get_ray_draws"]):
        ci, s, t = int(row[0]), row[1], row[2]
        out = np.zeros(7, np.float32)
        used = C.c_uint32()
        dr = np.ascontiguousarray(draws, np.uint32)
        orc.lib().oracle_get_ray(C.byref(cams[ci]), s, t, dr.ctypes.data_as(C.POINTER(C.c_uint32)), len(dr),
                                 orc.fp(out), C.byref(used))
        assert np.array_equal(bits(out), bits(row[3:10])) and used.value == int(row[10])


def test_tonemap(orc):
    for s, w in zip(G["tm_sum"], G["tm_out"]):
        assert orc.lib().oracle_tonemap(float(s), 50) == int(w), s


def test_whole_image_jumpy(orc, rtw):
    """16x9x2 spp jumpy-balls: oracle (via the product's preset + dump) vs the numpy restatement
    (its own scenes.rs generator and integrator)."""
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", 16 / 9, seed=5)
    o = orc.OracleScene(s.dump(), s.images())
    img, rays = o.render(orc.camera_from_fields(cam.as_dict()), bg, 16, 9, 2, seed=9)
    assert rays == int(G["jumpy_rays"][0])
    assert np.array_equal(bits(img), bits(G["jumpy_img"]))
