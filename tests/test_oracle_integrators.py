"""The oracle's two integrators and two BVH modes agree.

ITERATIVE (L = T * terminal, T = ((a0*a1)*a2)...) is what the GPU computes bit-for-bit;
RECURSIVE is lib.rs:97-117 literally (emitted + a0 * (a1 * (...))).  They draw the same
random numbers and trace the same paths, so they differ only in the rounding of the
throughput product: a few ulp per bounce.  Tolerance: relative 2e-5 per pixel component,
far inside the north_star's RMSE < 1e-4 on the mean image.
BVH_REFERENCE builds bvh.rs:19-74's tree (random axis, median split) and walks it as
bvh.rs:100-120 does; BVH_AS_LIST is the set semantics the GPU reproduces.  They agree
except on exact t ties between triangles, so the images must match to the same tolerance.
"""
import numpy as np
import pytest


def scene(rtw, orc, name, seed=3):
    s = rtw.Scene()
    cam, bg = s.preset(name, 16 / 9, seed=seed)
    return orc.OracleScene(s.dump(), s.images()), orc.camera_from_fields(cam.as_dict()), bg


@pytest.mark.parametrize("name,w,h,spp", [("jumpy-balls", 48, 27, 4), ("cornell-box", 32, 18, 8),
                                          ("wavefront-cow-obj", 32, 18, 2)])
def test_recursive_vs_iterative(rtw, orc, name, w, h, spp):
    o, cam, bg = scene(rtw, orc, name)
    a, ra = o.render(cam, bg, w, h, spp, seed=4, integrator=orc.ITERATIVE)
    b, rb = o.render(cam, bg, w, h, spp, seed=4, integrator=orc.RECURSIVE)
    assert ra == rb
    assert np.allclose(a, b, rtol=2e-5, atol=1e-6)
    rmse = np.sqrt(np.mean((a / spp - b / spp) ** 2))
    assert rmse < 1e-6


def test_reference_bvh_vs_list(rtw, orc):
    o, cam, bg = scene(rtw, orc, "wavefront-cow-obj")
    a, ra = o.render(cam, bg, 40, 22, 2, seed=4, bvh_mode=orc.BVH_AS_LIST)
    b, rb = o.render(cam, bg, 40, 22, 2, seed=4, bvh_mode=orc.BVH_REFERENCE)
    assert ra == rb
    assert np.allclose(a, b, rtol=2e-5, atol=1e-6)


def test_threads_do_not_change_the_image(rtw, orc):
    o, cam, bg = scene(rtw, orc, "jumpy-balls")
    a, _ = o.render(cam, bg, 32, 18, 2, seed=8, threads=1)
    b, _ = o.render(cam, bg, 32, 18, 2, seed=8, threads=7)
    assert np.array_equal(a, b)


def test_row_subset_matches_full(rtw, orc):
    o, cam, bg = scene(rtw, orc, "jumpy-balls")
    full, _ = o.render(cam, bg, 32, 18, 2, seed=8)
    part, _ = o.render(cam, bg, 32, 18, 2, seed=8, rows=[17, 5, 0])
    for j in (17, 5, 0):
        assert np.array_equal(part[18 - 1 - j], full[18 - 1 - j])


def test_pixel_subset_matches_full(rtw, orc):
    """oracle_render_pixels (scripts/fullspp_parity.py re-renders a frame's differing pixels with it) gives each
    pixel's sums of the whole-frame render, in the order asked, for both traversal modes."""
    o, cam, bg = scene(rtw, orc, "wavefront-cow-obj")
    px = [(17, 31), (0, 0), (9, 12), (9, 13), (4, 30)]  # (j bottom-based, i)
    for mode in (orc.BVH_AS_LIST, orc.BVH_REFERENCE):
        full, _ = o.render(cam, bg, 32, 18, 2, seed=8, bvh_mode=mode)
        part, rays = o.render_pixels(cam, bg, 32, 18, 2, px, seed=8, bvh_mode=mode, threads=3)
        assert rays > 0
        for k, (j, i) in enumerate(px):
            assert np.array_equal(part[k].view(np.uint32), full[18 - 1 - j, i].view(np.uint32))
    with pytest.raises(RuntimeError):
        o.render_pixels(cam, bg, 32, 18, 2, [(18, 0)])


def test_estimator_converges(rtw, orc):
    """Different seeds estimate the same mean image: RMSE shrinks ~ 1/sqrt(spp)."""
    o, cam, bg = scene(rtw, orc, "cornell-box")
    errs = []
    for spp in (4, 64):
        a, _ = o.render(cam, bg, 16, 9, spp, seed=1)
        b, _ = o.render(cam, bg, 16, 9, spp, seed=2)
        errs.append(np.sqrt(np.mean((a / spp - b / spp) ** 2)))
    assert errs[1] < errs[0] / 2


def _fuzz_world(rtw, orc, seed, w, h):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import test_gpu_fuzz as F  # the GPU fuzz suite's world builder (building needs no GPU)
    rng = np.random.default_rng(1000 + seed)
    s = rtw.Scene()
    F._build(rtw, s, rng)
    eye = rng.uniform(-1, 1, 3) * np.array([8, 2, 8]) + np.array([0, 3, 0])
    cam = rtw.Camera.new(tuple(eye), tuple(rng.uniform(-1, 1, 3)), (0, 1, 0), float(rng.uniform(30, 70)), w / h,
                         float(rng.choice([0.0, 0.1])), float(np.linalg.norm(eye)))
    bg = tuple(rng.uniform(0, 0.8, 3))
    return orc.OracleScene(s.dump(), s.images()), orc.camera_from_fields(cam.as_dict()), bg


def test_nan_throughput_terminals_match_the_recursion(rtw, orc):
    """Round 6: fuzz world 329 at 96x54x8 has paths whose throughput turns NaN (a UVDebug ground whose sphere uv
    takes acos of -1.0000001, spherical.rs:70-71).  The recursion multiplies every terminal -- an absorbed Metal's
    black, the black at depth 0 -- by the attenuations above it (lib.rs:109-116), so the NaN reaches the pixel; the
    iterative form must return T * 0 there too, not a constant 0 (the GPU follows it: test_gpu_fuzz's regression)."""
    o, cam, bg = _fuzz_world(rtw, orc, 329, 96, 54)
    a, ra = o.render(cam, bg, 96, 54, 8, seed=329, integrator=orc.ITERATIVE)
    b, rb = o.render(cam, bg, 96, 54, 8, seed=329, integrator=orc.RECURSIVE)
    assert ra == rb
    assert np.isnan(b).sum() > 0
    assert np.array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(b)
    assert np.allclose(a[ok], b[ok], rtol=2e-5, atol=1e-6)
    # 20 paths deep at most: the depth-0 terminal of a NaN throughput too
    a, _ = o.render(cam, bg, 96, 54, 8, seed=329, max_depth=3, integrator=orc.ITERATIVE)
    b, _ = o.render(cam, bg, 96, 54, 8, seed=329, max_depth=3, integrator=orc.RECURSIVE)
    assert np.array_equal(np.isnan(a), np.isnan(b))
