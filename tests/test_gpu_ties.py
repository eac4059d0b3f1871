"""Exact-t ties: the later object wins (hittable/mod.rs:61-65 tests every object against the closest t so far, and
the primitives reject only t > t_max: spherical.rs:40-43, rectangular.rs:40, triangular.rs:118).

Worlds of coincident primitives with different materials make every hit on them an exact tie, so the colour of the
image depends on the tie rule alone.  Each kernel family must pick the later object in the hierarchy's depth-first
order -- the sphere worlds' LDS-node BVH4 walk with its 32-B branch-free test, the rect list loop (`t <= best`), the
rect BVH kernel, the triangle-leaf fast path (key read only on a candidate at or below the best t), instanced
cuboids -- bit for bit against the oracle's flat list.  Each world is also rendered with the two copies swapped:
the image must change, or the ties decided nothing."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, SPP = 48, 27, 2


def _render(rtw, orc, build, cam, bg):
    s = rtw.Scene()
    build(s, False)
    text, imgs = s.dump(), s.images()
    s.commit()
    g, st = rtw.Raytracer(s, cam, bg, W, H, SPP, seed=13).render()
    r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, W, H, SPP, seed=13)
    assert st["rays"] == rays
    bad = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} mismatching components, first {bad[:4].tolist()}"
    s2 = rtw.Scene()
    build(s2, True)
    s2.commit()
    g2, _ = rtw.Raytracer(s2, cam, bg, W, H, SPP, seed=13).render()
    assert not np.array_equal(g, g2), "swapping the coincident copies left the image unchanged: no tie was decided"
    return s


def _mats(s):
    return s.lambertian_solid((0.9, 0.15, 0.1)), s.lambertian_solid((0.1, 0.8, 0.2))


def test_coincident_spheres_lds_node_walk(gpu, orc):
    """80 spheres added twice (static, then as moving spheres that do not move) over a ground sphere: a BVH'd
    sphere world, so the LDS-node kernel's walk and its 32-B test decide the ties."""
    rtw = gpu
    rng = np.random.default_rng(5)
    c = np.stack([rng.uniform(-6, 6, 80), rng.uniform(0.2, 1.5, 80), rng.uniform(-6, 6, 80)], 1).astype(np.float32)
    r = rng.uniform(0.2, 0.6, 80).astype(np.float32)

    def build(s, swap):
        a, b = _mats(s)
        first, second = (b, a) if swap else (a, b)
        ground = s.lambertian_solid((0.5, 0.5, 0.5))
        s.sphere((0, -1000, 0), 1000, ground)
        s.spheres(c, r, [first] * len(r))
        s.moving_spheres(c, np.zeros(len(r)), c, np.ones(len(r)), r, [second] * len(r))

    cam = rtw.Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 30.0, W / H, 0.0, 10.0)
    s = _render(rtw, orc, build, cam, (0.7, 0.8, 1.0))
    assert s.info(3) > 0  # a BVH, not the list


def test_coincident_rects_list_loop_and_instances(gpu, orc):
    """A box of walls, each wall twice, and two rotated + translated cuboids, each twice: a list-mode world of 24
    rects (the rect list loop and its per-chain reciprocals)."""
    rtw = gpu

    def build(s, swap):
        a, b = _mats(s)
        first, second = (b, a) if swap else (a, b)
        light = s.diffuse_light(s.solid_rgb(8, 8, 8))
        for m in (first, second):
            s.yz_rect(0, 555, 0, 555, 555, m)
            s.yz_rect(0, 555, 0, 555, 0, m)
            s.xz_rect(0, 555, 0, 555, 0, m)
            s.xy_rect(0, 555, 0, 555, 555, m)
        s.xz_rect(113, 443, 127, 432, 554, light)
        for m in (first, second):
            with s.translate((265, 0, 295)):
                with s.rotate_y(15):
                    s.cuboid((0, 0, 0), (165, 330, 165), m)
        s.xz_rect(0, 555, 0, 555, 555, first)

    cam = rtw.Camera.new((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, W / H, 0.0, 10.0)
    s = _render(rtw, orc, build, cam, (0.0, 0.0, 0.0))
    assert s.info(3) == 0  # list mode


def test_coincident_rects_bvh(gpu, orc):
    """40 small rects, each twice (80 > the 32-prim list limit): the rect BVH kernel's leaves decide the ties."""
    rtw = gpu
    rng = np.random.default_rng(9)
    x0 = rng.uniform(-5, 4, 40).astype(np.float32)
    y0 = rng.uniform(-3, 2, 40).astype(np.float32)
    k = rng.uniform(-4, 0, 40).astype(np.float32)

    def build(s, swap):
        a, b = _mats(s)
        first, second = (b, a) if swap else (a, b)
        for m in (first, second):
            s.rects([0] * 40, x0, x0 + 1.5, y0, y0 + 1.5, k, [m] * 40)

    cam = rtw.Camera.new((0, 0, 8), (0, 0, 0), (0, 1, 0), 60.0, W / H, 0.0, 8.0)
    s = _render(rtw, orc, build, cam, (0.7, 0.8, 1.0))
    assert s.info(3) > 0


def test_coincident_triangles_mesh_leaves(gpu, orc):
    """A 12 x 12 grid of 288 triangles, added twice: every BVH leaf is a triangle of one chain, so the triangle
    leaf fast path decides the ties (its key load only for candidates at or below the best t)."""
    rtw = gpu
    n = 12
    g = np.linspace(-4, 4, n + 1, dtype=np.float32)
    tris = []
    for i in range(n):
        for j in range(n):
            p00 = (g[i], g[j], -0.3 * g[i])
            p10 = (g[i + 1], g[j], -0.3 * g[i + 1])
            p01 = (g[i], g[j + 1], -0.3 * g[i])
            p11 = (g[i + 1], g[j + 1], -0.3 * g[i + 1])
            tris += [p00, p10, p11, p00, p11, p01]
    verts = np.asarray(tris, np.float32).reshape(-1)

    def build(s, swap):
        a, b = _mats(s)
        first, second = (b, a) if swap else (a, b)
        with s.translate((0.0, 0.5, 0.0)):
            s.triangles(verts, first)
            s.triangles(verts, second)
        s.xz_rect(-20, 20, -20, 20, 30, s.diffuse_light(s.solid_rgb(2, 2, 2)))

    cam = rtw.Camera.new((2, 1, 9), (0, 0, 0), (0, 1, 0), 50.0, W / H, 0.0, 9.0)
    s = _render(rtw, orc, build, cam, (0.3, 0.3, 0.35))
    assert s.info(3) > 0


def test_degenerate_primitives(gpu, orc):
    """Degenerate inputs the reference accepts without complaint render as the oracle does: zero-area triangles (a
    repeated vertex, collinear vertices: det = 0, t = NaN fails `t >= 0`), slivers (|det| tiny, 1 / det huge), a
    zero-radius sphere, a hollow (negative-radius) glass sphere, zero-width and inverted-bounds rects (never hit:
    rectangular.rs:40 cannot pass with a0 > a1), next to ordinary geometry."""
    rtw = gpu
    rng = np.random.default_rng(21)
    tris = []
    for _ in range(40):  # ordinary triangles
        p = rng.uniform(-3, 3, 3).astype(np.float32)
        tris += [p, p + rng.uniform(-1, 1, 3), p + rng.uniform(-1, 1, 3)]
    for _ in range(20):  # repeated vertex / collinear / sliver
        p = rng.uniform(-3, 3, 3).astype(np.float32)
        q = p + rng.uniform(-1, 1, 3).astype(np.float32)
        tris += [p, p, q]
        tris += [p, q, p + np.float32(2.0) * (q - p)]
        tris += [p, q, q + np.float32(1e-6) * rng.uniform(-1, 1, 3).astype(np.float32)]
    verts = np.asarray(tris, np.float32).reshape(-1)
    s = rtw.Scene()
    a, b = _mats(s)
    glass = s.dielectric(1.5)
    s.triangles(verts, a)
    s.sphere((0, 0, 0), 0.0, b)
    s.sphere((1, 0.5, 1), 0.8, glass)
    s.sphere((1, 0.5, 1), -0.7, glass)
    s.xy_rect(-2, -2, -2, 2, -3, b)   # zero width
    s.xz_rect(2, -2, -2, 2, -2.5, b)  # inverted bounds
    s.xz_rect(-50, 50, -50, 50, -4, s.lambertian_solid((0.5, 0.5, 0.5)))
    cam = rtw.Camera.new((3, 2, 8), (0, 0, 0), (0, 1, 0), 50.0, W / H, 0.0, 8.0)
    bg = (0.7, 0.8, 1.0)
    text, imgs = s.dump(), s.images()
    s.commit()
    g, st = rtw.Raytracer(s, cam, bg, W, H, 4, seed=3).render()
    r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, W, H, 4, seed=3)
    assert st["rays"] == rays
    bad = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} mismatching components, first {bad[:4].tolist()}"


def test_infinite_rect_bounds_list_mode(gpu, orc):
    """Rects with infinite bounds: an endless floor, a wall unbounded on one side, a ceiling strip.  Their
    hit points can overflow to +-inf, so the flattener leaves such a world off the rect loop's fast path (rect_fast 0,
    rtw_scene_info 13) and the IEEE path decides `x < a0 || x > a1` as rectangular.rs:40 does; grazing rays along the
    floor (the camera a hair above it) included."""
    rtw = gpu
    inf = float("inf")
    s = rtw.Scene()
    a, b = _mats(s)
    s.xz_rect(-inf, inf, -inf, inf, 0.0, s.lambertian_solid((0.5, 0.5, 0.5)))  # floor
    s.xy_rect(-inf, 3.0, 0.0, 4.0, -6.0, a)                                    # wall, unbounded to -x
    s.yz_rect(0.5, 2.5, -inf, inf, 4.0, b)                                     # strip, unbounded in z
    s.xz_rect(-1.0, 1.0, -1.0, 1.0, 5.0, s.diffuse_light(s.solid_rgb(4, 4, 4)))
    cam = rtw.Camera.new((0.0, 1e-3, 6.0), (0.0, 0.5, 0.0), (0, 1, 0), 70.0, W / H, 0.0, 6.0)
    bg = (0.6, 0.7, 0.9)
    text, imgs = s.dump(), s.images()
    s.commit()
    assert s.info(3) == 0 and s.info(13) == 0  # list mode, off the fast path
    g, st = rtw.Raytracer(s, cam, bg, W, H, 4, seed=3).render()
    r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, W, H, 4, seed=3)
    assert st["rays"] == rays
    bad = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} mismatching components, first {bad[:4].tolist()}"


@pytest.mark.parametrize("kernel", ["rect_list", "all_features_list", "generic"])
@pytest.mark.parametrize("tile,spp", [(2149, 20), (2347, 16)])
def test_in_plane_bounce_list_mode(gpu, orc, knobs, kernel, tile, spp):
    """A Lambertian bounce off cornell's floor whose direction lost its normal component exactly (d.y = 0, the
    origin on the plane y = 0) meets the floor at t = 0 / 0 = NaN, and the reference's rejections (rectangular.rs:
    33-41: `t < t_min || t > t_max`, then the bounds) all let a NaN through: it is a hit, best becomes NaN, every later
    rect whose own test passes wins, and the path continues from a NaN origin to the depth limit.  The rect list
    loop reproduces this on its IEEE path.  These two tiles of the 800 x 800 bench frame (scene seed 42, render seed
    2024) hold the only two such events of its first 32 samples (scripts/count_bisect.py): their last sample is the
    one with the in-plane bounce.  Packed tile render against the oracle's rows, bit for bit, with ray counts; through
    the rect list loop and through the all-features list kernel (knob RTW_LIST_ALL: test_prim's list fold; and
    RTW_GENERIC, which on a list world selects that same kernel: ADVICE r5)."""
    torch = pytest.importorskip("torch")
    rtw = gpu
    if kernel == "all_features_list":
        knobs.setenv("RTW_LIST_ALL", "1")
    if kernel == "generic":
        knobs.setenv("RTW_GENERIC", "1")
    w = h = 800
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0, seed=42)
    text, imgs = s.dump(), s.images()
    s.commit()
    rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=2024)
    ids = torch.tensor([tile], dtype=torch.int32, device="cuda:0")
    packed = torch.zeros((1, 64, 3), dtype=torch.float32, device="cuda:0")
    st = rt.render_device(packed.data_ptr(), 0, ids.data_ptr(), 1, torch.cuda.current_stream().cuda_stream,
                          want_stats=True)
    torch.cuda.synchronize()
    r, c = divmod(tile, (w + 7) // 8)
    rows = [h - 1 - (r * 8 + k) for k in range(8)]  # j of the tile's rows (output row 0 = j = h - 1)
    ref, _, pr = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=2024,
                                                    rows=rows, pixel_rays=True)
    assert int(st["rays"]) == int(pr[r * 8:(r + 1) * 8, c * 8:(c + 1) * 8].sum())
    want = ref[r * 8:(r + 1) * 8, c * 8:(c + 1) * 8].reshape(64, 3)
    got = packed.cpu().numpy()[0]
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} mismatching components, first {bad[:4].tolist()}"
