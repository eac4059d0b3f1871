"""GPU parity: the HIP render core vs the CPU oracle on the same seeded inputs.

Bar: bit-exact against the oracle's iterative integrator (same draws, same IEEE f32
operation order; the reference's own association differs only in the throughput product,
covered by test_oracle_integrators.py).  Sizes are chosen so the oracle (flat-list
closest hit, as hittable/mod.rs:57-69) finishes in about a second.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCENES = [
    # name, aspect, w, h, spp
    ("jumpy-balls", 16 / 9, 64, 36, 4),
    ("cornell-box", 1.0, 40, 40, 8),
    ("wavefront-cow-obj", 16 / 9, 48, 27, 3),
    ("textured-monument", 16 / 9, 48, 27, 3),
    ("two-spheres", 16 / 9, 48, 27, 4),
    ("simple-triangle", 16 / 9, 48, 27, 4),
    # Perlin noise, image-textured spheres (uv), media, the book-2 scenes
    ("two-perlin-spheres", 16 / 9, 48, 27, 3),
    ("earth", 16 / 9, 48, 27, 3),
    ("simple-light", 16 / 9, 48, 27, 4),
    ("smokey-cornell-box", 1.0, 32, 32, 6),
    ("book2-final-scene", 1.0, 32, 32, 3),
    ("animated-book2-final-scene", 1.0, 24, 24, 2),
]


def _both(rtw, orc, name, aspect, w, h, spp, seed=11, max_depth=50):
    s = rtw.Scene()
    cam, bg = s.preset(name, aspect, seed=3)
    text, imgs = s.dump(), s.images()
    s.commit()
    gpu_img, st = rtw.Raytracer(s, cam, bg, w, h, spp, seed=seed, max_depth=max_depth).render()
    o = orc.OracleScene(text, imgs)
    ref_img, rays = o.render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=seed,
                             max_depth=max_depth)
    return gpu_img, ref_img, st, rays


@pytest.mark.parametrize("name,aspect,w,h,spp", SCENES)
def test_scene_bit_exact(gpu, orc, name, aspect, w, h, spp):
    g, r, st, rays = _both(gpu, orc, name, aspect, w, h, spp)
    assert st["rays"] == rays, f"ray count {st['rays']} vs oracle {rays}"
    bad = np.argwhere(g.view(np.uint32) != r.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} mismatching components, first {bad[:4].tolist()}: " \
                          f"gpu {g[tuple(bad[0][:2])]} oracle {r[tuple(bad[0][:2])]}"
    rmse = float(np.sqrt(np.mean((g / spp - r / spp) ** 2)))
    assert rmse < 1e-4  # north_star tolerance (implied by bit-exactness, stated for the record)


def test_depth_limits(gpu, orc):
    for depth in (0, 1, 2, 7):
        g, r, st, rays = _both(gpu, orc, "cornell-box", 1.0, 16, 16, 2, max_depth=depth)
        assert st["rays"] == rays
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), depth


def test_seed_changes_image_not_stats(gpu, orc):
    g1, _, st1, _ = _both(gpu, orc, "jumpy-balls", 16 / 9, 32, 18, 2, seed=1)
    g2, _, st2, _ = _both(gpu, orc, "jumpy-balls", 16 / 9, 32, 18, 2, seed=2)
    assert not np.array_equal(g1, g2)
    assert abs(g1.mean() - g2.mean()) < 0.1 * g1.mean()


def test_tiles_match_full_frame(gpu):
    """Packed tile rendering (multi-GPU path) == full-frame rendering, any tile split."""
    torch = pytest.importorskip("torch")
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", 16 / 9, seed=3)
    s.commit(device=0)
    w, h, spp = 72, 40, 2  # ragged: 9 x 5 tiles, last tile row half outside
    rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=5)
    full, _ = rt.render()
    nt = rtw.n_tiles(w, h)
    img = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    for world in (1, 2, 3):
        for rank in range(world):
            ids = torch.arange(rank, nt, world, dtype=torch.int32, device="cuda:0")
            packed = torch.zeros((len(ids), 64, 3), dtype=torch.float32, device="cuda:0")
            rt.render_device(packed.data_ptr(), 0, ids.data_ptr(), len(ids),
                             torch.cuda.current_stream().cuda_stream)
            rtw.unpack_tiles_device(w, h, ids.data_ptr(), len(ids), packed.data_ptr(), img.data_ptr(), 0,
                                    torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(img.cpu().numpy().view(np.uint32), full.view(np.uint32)), world


@pytest.mark.parametrize("scene,w,h,spp", [(None, 16, 8, 3), ("jumpy-balls", 2, 2, 1), ("cornell-box", 9, 3, 1),
                                            ("wavefront-cow-obj", 2, 2, 5), ("jumpy-balls", 65536, 2, 1)])
def test_empty_world_and_smallest_frames(gpu, orc, scene, w, h, spp):
    """Edge cases of lib.rs:57-117: a world with no objects (every ray misses: the background, one ray per path,
    the F_LIST kernel with an empty list), the smallest frame the reference can divide by (2 x 2: w - 1 = h - 1 = 1),
    a single-row-of-tiles ragged frame, the widest frame the 16-bit pixel coordinates of the path key allow
    (65536 columns), and one sample per pixel (the path id decode without the spp division).
    These frames also take the small-frame batches."""
    rtw = gpu
    s = rtw.Scene()
    if scene is None:
        cam, bg = rtw.Camera.new((0, 0, 5), (0, 0, 0), (0, 1, 0), 40.0, w / h, 0.1, 5.0), (0.7, 0.8, 1.0)
    else:
        cam, bg = s.preset(scene, w / h, seed=3)
    text, imgs = s.dump(), s.images()
    s.commit()
    g, st = rtw.Raytracer(s, cam, bg, w, h, spp, seed=7).render()
    r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=7)
    assert st["rays"] == rays
    if scene is None:
        assert rays == w * h * spp
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


def test_error_paths(gpu):
    rtw = gpu
    s = rtw.Scene()
    m = s.lambertian_solid((0.5, 0.5, 0.5))
    s.sphere((0, 0, 0), 1, m)
    s.commit()
    cam = rtw.Camera.new((0, 0, 5), (0, 0, 0), (0, 1, 0), 40, 1.0, 0.0, 1.0)
    with pytest.raises(rtw.RtwError):
        rtw.Raytracer(s, cam, (0, 0, 0), 1, 1, 1).render()  # lib.rs:84-85 divides by w-1
    with pytest.raises(rtw.RtwError):
        rtw.Raytracer(s, cam, (0, 0, 0), 65537, 2, 1).render()  # beyond the path key's 16-bit column
    with pytest.raises(rtw.RtwError):
        s.sphere((0, 0, 0), 1, m)  # scene immutable after commit


@pytest.mark.parametrize("name,aspect,w,h,spp", [SCENES[0], SCENES[2], SCENES[3]])
def test_stack_spill_bit_exact(gpu, orc, knobs, name, aspect, w, h, spp):
    """A 4-entry LDS stack pushes every deeper entry through the HBM spill area
    (RenderArgs::spill); the image must not change."""
    knobs.setenv("RTW_STACK_LDS", "4")
    g, r, st, rays = _both(gpu, orc, name, aspect, w, h, spp)
    assert st["rays"] == rays
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


@pytest.mark.parametrize("knob", ["RTW_REGEN_MIN=1", "RTW_REGEN_MIN=64", "RTW_QUOTA16=1", "RTW_QUOTA16=16",
                                  "RTW_LIST_MAX=0", "RTW_LIST_MAX=64", "RTW_LIST_OCC=6", "RTW_LEAF16=1",
                                  "RTW_LEAF16=16", "RTW_LDS_NODES=0", "RTW_OCC=5", "RTW_HALF_NODES=1",
                                  "RTW_HALF_NODES=0", "RTW_TRI_LEAF=0", "RTW_LDSN_WAVES=6", "RTW_LDSN_WAVES=7",
                                  "RTW_LDSN_BLK=512", "RTW_MESH_S16=0", "RTW_MESH_S16=6",
                                  "RTW_MESH_S16=7", "RTW_BVH_PAIR=1", "RTW_BVH_BINS=64", "RTW_BATCH=64",
                                  "RTW_BATCH=65536"])
def test_scheduling_knobs_bit_exact(gpu, orc, knobs, knob):
    """When a wave regenerates paths (RenderArgs::regen_min) and when a suspended traversal
    yields (quota16) change only which lanes run which path when; every path's draws and
    operations are keyed by its (pixel, sample) id, so the image and the ray count must not move.
    Same for the node table in LDS vs global memory (RTW_LDS_NODES) and the occupancy variants
    (RTW_OCC).  Same for list mode vs BVH (RTW_LIST_MAX) and for other trees over the same prims (RTW_BVH_PAIR,
    RTW_BVH_BINS): closest hit with ties to the later object is a commutative reduction over the leaves,
    whatever culls them -- with one documented exemption: RTW_LIST_MAX=0 walks a list world's rects
    through a BVH, whose fold counts a NaN candidate (an in-plane bounce, t = 0/0) as a miss where the reference's
    list order lets it win; these frames hold no in-plane bounce (cornell-800 x 32 holds two, pinned in list mode by
    test_in_plane_bounce_list_mode)."""
    k, v = knob.split("=")
    knobs.setenv(k, v)
    # the half-node knobs matter for BVH worlds: jumpy-balls (LDS nodes) and the cow (global nodes)
    mesh = "HALF" in k or "TRI" in k or "MESH" in k or "BVH" in k
    for name, aspect, w, h, spp in ((SCENES[0], SCENES[2], SCENES[3]) if mesh else (SCENES[0], SCENES[1])):
        g, r, st, rays = _both(gpu, orc, name, aspect, w, h, spp)
        assert st["rays"] == rays
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), name


def test_pass_with_path_ids_above_2_31(gpu, knobs):
    """One pass of more than 2^31 paths (monument-4k's passes hold 2^32): path ids past 2^31 must
    dispense and index correctly.  The same frame split into 2^30-path passes is the reference."""
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("two-spheres", 1.0, seed=3)
    s.commit()
    w = h = 256
    spp = 32800  # 256 * 256 * 32800 = 2.15e9 paths > 2^31
    one, st1 = rtw.Raytracer(s, cam, bg, w, h, spp, seed=7).render()
    knobs.setenv("RTW_PASS_LOG2", "30")
    split, st2 = rtw.Raytracer(s, cam, bg, w, h, spp, seed=7).render()
    assert st1["rays"] == st2["rays"] > w * h * spp
    assert np.array_equal(one.view(np.uint32), split.view(np.uint32))


def test_start_ring_passes_and_tiles(gpu, knobs):
    """The rect list kernel's path starts come from a per-wave ring of 64 made at once from consecutive ids of the
    wave's pool.  A frame split into passes (the pool restarts at each) and packed tile
    renders of a ragged frame (off-image ids inside the ring) must give the one-pass full frame's bits and rays."""
    torch = pytest.importorskip("torch")
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0, seed=3)
    s.commit(device=0)
    w, h, spp = 96, 96, 2048  # 18.9 M paths: two passes of 2^24
    one, st1 = rtw.Raytracer(s, cam, bg, w, h, spp, seed=11).render()
    knobs.setenv("RTW_PASS_LOG2", "24")
    split, st2 = rtw.Raytracer(s, cam, bg, w, h, spp, seed=11).render()
    assert st1["rays"] == st2["rays"]
    assert np.array_equal(one.view(np.uint32), split.view(np.uint32))
    w, h, spp = 44, 21, 3  # ragged: 6 x 3 tiles, the last column and row partly outside
    rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=5)
    full, _ = rt.render()
    nt = rtw.n_tiles(w, h)
    img = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    for world in (1, 2, 5):
        for rank in range(world):
            ids = torch.arange(rank, nt, world, dtype=torch.int32, device="cuda:0")
            packed = torch.zeros((len(ids), 64, 3), dtype=torch.float32, device="cuda:0")
            rt.render_device(packed.data_ptr(), 0, ids.data_ptr(), len(ids),
                             torch.cuda.current_stream().cuda_stream)
            rtw.unpack_tiles_device(w, h, ids.data_ptr(), len(ids), packed.data_ptr(), img.data_ptr(), 0,
                                    torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(img.cpu().numpy().view(np.uint32), full.view(np.uint32)), world


def test_path_kernel_times(gpu):
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0, seed=3)
    s.commit(device=0)
    rt = rtw.Raytracer(s, cam, bg, 16, 16, 2, seed=1)
    rt.render()
    rt.render()
    t = s.path_kernel_times(0)
    assert len(t) == 2 and all(x > 0 for x in t)
    assert s.path_kernel_times(0) == []  # consumed


@pytest.mark.parametrize("name,aspect,w,h,spp", [SCENES[1], SCENES[2], SCENES[3], SCENES[5]])
def test_generic_kernel_bit_exact(gpu, orc, knobs, name, aspect, w, h, spp):
    """Every scene normally runs the smallest specialised kernel variant covering its features
    (F_SPHERES / F_BOXES / F_MESHES, rtw_device.hpp); the all-features kernel must agree too.  A list world
    (cornell-box) takes the all-features LIST kernel, whose fold keeps the reference's NaN semantics."""
    knobs.setenv("RTW_GENERIC", "1")
    g, r, st, rays = _both(gpu, orc, name, aspect, w, h, spp)
    assert st["rays"] == rays
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))


def test_device_libm_equals_oracle(gpu, orc):
    """The kernel's f32 transcendentals (double-evaluated, correctly rounded) are the oracle's,
    bit for bit: every rand Standard<f32> value for log10 (the medium draw), dense strides of the
    float line for acos (sphere uv) and sin (Noise), random pairs and IEEE specials for atan2."""
    rtw = gpu
    u = (np.arange(1, 1 << 24, dtype=np.float64) * 2.0 ** -24).astype(np.float32)
    u = np.concatenate([u, np.array([0.0, -0.0, 1.0, np.inf, -1.0, np.nan, 1e-45, 3e38], np.float32)])
    b = np.arange(0, 0x3F800001, 37, dtype=np.uint32)
    ac = np.concatenate([b, b | np.uint32(0x80000000)]).view(np.float32)
    b = np.arange(0, 0x47000000, 97, dtype=np.uint32)
    sn = np.concatenate([b, b | np.uint32(0x80000000), np.array([0x7F800000, 0xFF800000, 0x7FC00000,
                                                                  0x4F000000, 0x5F000000], np.uint32)]).view(np.float32)
    rng = np.random.default_rng(11)
    e = rng.integers(90, 160, (2, 1 << 20))
    m = rng.integers(0, 1 << 23, (2, 1 << 20))
    sg = rng.integers(0, 2, (2, 1 << 20))
    ab = ((sg << 31) | (e << 23) | m).astype(np.uint32).view(np.float32)
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3e38], np.float32)
    y, x = np.meshgrid(sp, sp)
    ay = np.concatenate([ab[0], y.ravel()])
    ax = np.concatenate([ab[1], x.ravel()])
    for fn, a, bb in ((0, u, None), (1, sn, None), (2, ac, None), (3, ay, ax)):
        dev = rtw.diag_libm(fn, a, bb)
        ref = orc.libm(fn, a, bb)
        same = (dev.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(dev) & np.isnan(ref))
        bad = np.nonzero(~same)[0]
        assert bad.size == 0, (fn, bad.size, a[bad[:4]], dev[bad[:4]], ref[bad[:4]])


def test_camera_division_equals_ieee(gpu):
    """start_path's u = (i + U) / (w - 1), v = (j + U) / (h - 1) (lib.rs:84-85) use Markstein's
    correction from RN(1 / b) instead of an IEEE division: bit-identical to the IEEE f32 quotient for
    every dividend the camera forms (0, or i + U with U = k 2^-24) and every divisor 1..65535."""
    rtw = gpu
    rng = np.random.default_rng(7)
    n = 1 << 22
    i = rng.integers(0, 65536, n).astype(np.float32)
    U = (rng.integers(0, 1 << 24, n).astype(np.float64) * 2.0 ** -24).astype(np.float32)
    U[: n // 8] = (np.arange(n // 8) % 64).astype(np.float32) * np.float32(2.0 ** -24)  # tiny draws
    i[: n // 16] = 0.0
    a = (i + U).astype(np.float32)  # one IEEE f32 addition, as the kernel forms it
    b = rng.integers(1, 65536, n).astype(np.float32)
    b[:1024] = np.arange(1, 1025, dtype=np.float32)
    b[1024:2048] = np.arange(65535 - 1023, 65536, dtype=np.float32)
    a[2048:3072] = b[2048:3072]  # exact quotients
    dev = rtw.diag_libm(4, a, b)
    ref = (a / b).astype(np.float32)
    bad = np.nonzero(dev.view(np.uint32) != ref.view(np.uint32))[0]
    assert bad.size == 0, (bad.size, a[bad[:4]], b[bad[:4]], dev[bad[:4]], ref[bad[:4]])


def test_sphere_root_division_equals_ieee(gpu):
    """cand_sphere_rcp's roots (-hb -+ sq) / a by Markstein's correction from y = RN(1 / a): over the
    range the kernel takes that path for (a in [2^-60, 2^60], |numerator| < 2^64) the quotient is the
    IEEE one bit for bit wherever it is normal, and below 2^-126 both are < TMIN (rejected alike)."""
    rtw = gpu
    rng = np.random.default_rng(13)
    n = 1 << 22

    def rand_f32(lo_e, hi_e, signed):
        e = rng.integers(lo_e, hi_e, n)
        m = rng.random(n) + 1.0
        x = (m * np.exp2(e.astype(np.float64))).astype(np.float32)
        if signed:
            x = np.where(rng.random(n) < 0.5, -x, x).astype(np.float32)
        return x
    num = rand_f32(-70, 64, True)
    a = rand_f32(-60, 60, False)
    num[:4096] = 0.0
    dev = rtw.diag_libm(4, num, a)
    ref = (num / a).astype(np.float32)
    normal = np.abs(ref) >= np.float32(2.0 ** -126)
    bad = np.nonzero(normal & (dev.view(np.uint32) != ref.view(np.uint32)))[0]
    assert bad.size == 0, (bad.size, num[bad[:4]], a[bad[:4]], dev[bad[:4]], ref[bad[:4]])
    tiny = ~normal
    assert np.all(np.abs(dev[tiny]) < 0.001) and np.all(np.abs(ref[tiny]) < 0.001)


def test_sphere_sqrt_equals_ieee(gpu):
    """The sphere test's sqrt (sqrt_rn: the backend's correctly rounded expansion without the scaling
    it only applies below 2^-96) equals IEEE sqrt: every mantissa at an even and an odd exponent, the
    2^-96 boundary, zeros, subnormals, infinities and NaN, and random floats over the whole range."""
    rtw = gpu
    m = np.arange(1 << 23, dtype=np.uint32)
    x = np.concatenate([(m | np.uint32(127 << 23)), (m | np.uint32(128 << 23)),
                        np.arange(0x0F800000 - 4096, 0x0F800000 + 4096, dtype=np.uint32),  # 2^-96
                        np.arange(0, 1 << 16, dtype=np.uint32),                              # subnormals
                        np.array([0x7F7FFFFF, 0x7F800000, 0x7FC00000, 0x80000000, 0xBF800000], np.uint32),
                        np.random.default_rng(17).integers(0, 0x7F800000, 1 << 22, dtype=np.uint32)]).view(np.float32)
    dev = rtw.diag_libm(5, x)
    with np.errstate(invalid="ignore"):
        ref = np.sqrt(x)
    same = (dev.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(dev) & np.isnan(ref))
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, (bad.size, x[bad[:4]], dev[bad[:4]], ref[bad[:4]])


def test_render_stream_pixels(gpu):
    """Raytracer::render() as a Pixel stream (lib.rs:50-76): same sums as rtw_render, emitted
    row j = h-1 .. 0, column 0 .. w-1, band by band; the ProgressMessage frames round-trip."""
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0, seed=3)
    s.commit()
    w, h, spp = 40, 27, 3
    rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=4)
    full, st = rt.render()
    bands = []
    st2 = rt.render_stream(bands.append, band_rows=8)
    assert len(bands) == 4 and st2["rays"] == st["rays"]
    px = np.concatenate(bands)
    assert len(px) == w * h
    assert np.array_equal(px["row"], np.repeat(np.arange(h - 1, -1, -1), w))
    assert np.array_equal(px["column"], np.tile(np.arange(w), h))
    assert np.array_equal(px["color"].reshape(h, w, 3).view(np.uint32), full.view(np.uint32))
    frame = rtw.progress_encode(rtw.MSG_PIXEL, pixel=(px[5]["row"], px[5]["column"], px[5]["color"]))
    d = rtw.progress_decode(frame)
    assert (d["row"], d["column"]) == (h - 1, 5) and np.float32(d["color"]).tolist() == px[5]["color"].tolist()


def test_console_app_frames(gpu, tmp_path):
    """console_app/src/main.rs:28-94: one PNG per camera (30 for animated-book2-final-scene), named
    render/image_{:04}.png (:92-94), each the tonemap (:68-90) of that camera's render over the one
    committed world, rows top-down = the emission order row j = h-1 .. 0 (:66-71).  The PNG pixels
    are decoded and compared byte for byte with rtw_tonemap(rtw_render(...)) for three cameras."""
    import subprocess
    from pathlib import Path
    from PIL import Image
    rtw = gpu
    exe = Path(__file__).resolve().parents[1] / "raytracer-weekend_amd" / "bin" / "rtw_console"
    assert exe.exists(), "rtw_console not built"
    name, width, aspect, spp, seed = "animated-book2-final-scene", 32, 1.7777778, 2, 0
    r = subprocess.run([str(exe), name, "-w", str(width), "-a", str(aspect), "-s", str(spp),
                        "--models", str(gpu.MODELS_DIR), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    pngs = sorted(tmp_path.glob("image_*.png"))
    assert [p.name for p in pngs] == [f"image_{k:04d}.png" for k in range(30)]
    assert len(set(p.read_bytes() for p in pngs)) > 20  # the camera sweeps across the scene
    height = rtw.image_height(width, aspect)            # main.rs:33
    cam_aspect = rtw.camera_aspect(width, height)       # main.rs:38-41
    s = rtw.Scene()
    _, bg = s.preset(name, cam_aspect, seed=seed)
    s.commit()
    cams = rtw.preset_cameras(name, cam_aspect)
    assert len(cams) == 30
    for k in (0, 13, 29):
        sums, _ = rtw.Raytracer(s, cams[k], bg, width, height, spp, seed=seed).render()
        want = rtw.tonemap(sums, spp)
        got = np.asarray(Image.open(pngs[k]).convert("RGB"))
        assert got.shape == (height, width, 3)
        assert np.array_equal(got, want), f"camera {k}: {int((got != want).sum())} bytes differ"


def _sphere_world(rtw, seed, n=120):
    """A random sphere world in a BvhNode (> list_max leaves, so the BVH kernels run): static and
    moving spheres (unit and non-unit shutters), negative radii (hollow glass, spherical.rs:98-103),
    Lambertian / checker / Metal / Dielectric / DiffuseLight materials, a ground sphere."""
    rng = np.random.default_rng(seed)
    s = rtw.Scene()
    mats = [s.lambertian_solid(rng.uniform(0.1, 0.9, 3)) for _ in range(4)]
    mats += [s.lambertian(s.checker(s.solid_rgb(0.2, 0.3, 0.1), s.solid_rgb(0.9, 0.9, 0.9), 10.0))]
    mats += [s.metal(rng.uniform(0.5, 1.0, 3), float(f)) for f in (0.0, 0.3)]
    mats += [s.dielectric(1.5), s.diffuse_light(s.solid_rgb(4.0, 4.0, 4.0))]
    c = np.stack([rng.uniform(-6, 6, n), rng.uniform(0.1, 1.2, n), rng.uniform(-6, 6, n)], 1)
    r = rng.uniform(0.15, 0.4, n)
    r[rng.random(n) < 0.1] *= -1.0  # hollow glass shells
    m = rng.integers(0, len(mats), n)
    mov = rng.random(n) < 0.4
    with s.bvh(0.0, 1.0):
        s.sphere((0.0, -1000.0, 0.0), 1000.0, mats[4])
        s.spheres(c[~mov], r[~mov], m[~mov])
        k = int(mov.sum())
        t0 = np.where(rng.random(k) < 0.5, 0.0, 0.25).astype(np.float32)
        t1 = np.where(rng.random(k) < 0.5, 1.0, 0.75).astype(np.float32)
        s.moving_spheres(c[mov], t0, c[mov] + rng.uniform(-0.3, 0.3, (k, 3)), t1, r[mov], m[mov])
    cam = rtw.Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 16 / 9, 0.1, 10.0, 0.0, 1.0)
    return s, cam, (0.7, 0.8, 1.0)


@pytest.mark.parametrize("knob", ["", "RTW_LDS_NODES=0", "RTW_LDSN_WAVES=6", "RTW_LDSN_WAVES=7", "RTW_HALF_NODES=1",
                                  "RTW_LDSN_BLK=512", "RTW_BVH_PAIR=1"])
@pytest.mark.parametrize("seed,n", [(1, 120), (2, 120), (3, 700)])
def test_random_sphere_world_bit_exact(gpu, orc, knobs, knob, seed, n):
    """Sphere worlds run the LDS-node kernel (node table in LDS, sorted-push walk over 16-bit codes)
    when their tree fits -- the 8-wave variant for trees of <= 144 node4s (the 120-sphere worlds: 1024-lane
    workgroups with the paths' T / depth / id in LDS, or the 512-lane form by knob), the
    6-wave one up to 224 (the 700-sphere world) -- else the global-node one: all bit-exact against the
    oracle, with equal ray counts, on worlds that mix every sphere kind and material the sphere kernels
    specialise for; likewise the 6 / 7-wave and half-precision-node variants by knob."""
    if knob:
        k, v = knob.split("=")
        knobs.setenv(k, v)
    rtw = gpu
    s, cam, bg = _sphere_world(rtw, seed, n)
    text = s.dump()
    s.commit()
    assert s.info(3) > 0 and s.info(11) <= 24  # a BVH, within the LDS-node kernel's 24-row stack
    assert (s.info(3) > 144) == (n > 500)  # the 700-sphere world fills more than the old 144-node table
    w, h, spp = 48, 27, 4
    g, st = rtw.Raytracer(s, cam, bg, w, h, spp, seed=5).render()
    ref, rays = orc.OracleScene(text, []).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=5)
    assert st["rays"] == rays
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))


def test_fast_reciprocal_equals_ieee_for_every_float(gpu):
    """rcp_rn (v_rcp_f32 + one Newton step with an exact fma residual) is the IEEE f32 reciprocal
    1.0f / b for every bit pattern it is used on (|b| in [2^-126, 2^126]): an exhaustive device sweep
    of all 2^32 patterns, so the rect / unit-vector / normal divisions built on it (Markstein's
    correction from RN(1 / b)) are the reference's IEEE divisions (rectangular.rs:33-41, vec3.rs:85-87,
    spherical.rs:49)."""
    rtw = gpu
    bad, skipped, first = rtw.diag_sweep(0, 0, 0xFFFFFFFF)
    assert bad == 0, [hex(int(x)) for x in first[:8]]
    # the skipped patterns are exactly those outside [2^-126, 2^126] in magnitude (and NaNs / infs)
    inside = 2 * ((0x7E800000 - 0x00800000) + 1)
    assert skipped == (1 << 32) - inside


@pytest.mark.parametrize("case", ["far_plane", "far_origin", "near"])
def test_rect_reciprocal_guard_paths_bit_exact(gpu, orc, case):
    """Rect tests at the edges of f32's range (rectangular.rs:27-57, :78-108, :129-159): a sky plane at
    |k| = 1e19, camera rays whose origin is 1e19 away, and near planes, each with a wrapper chain (a rotated,
    translated cuboid) in list mode, must match the oracle bit for bit: the rect test's IEEE divisions
    (k - o) / d and its bounds must round exactly as the reference's at huge and tiny quotients."""
    rtw = gpu
    s = rtw.Scene()
    red = s.lambertian_solid((0.65, 0.05, 0.05))
    white = s.lambertian_solid((0.73, 0.73, 0.73))
    light = s.diffuse_light(s.solid_rgb(7.0, 7.0, 7.0))
    big = 1e25
    far = 1e19 if case == "far_plane" else 300.0  # 1e19 > 2^62
    s.xz_rect(-big, big, -big, big, far, light)                  # sky plane (y = k)
    s.xz_rect(-big, big, -big, big, 0.0, white)                  # floor
    s.yz_rect(0.0, 200.0, -200.0, 200.0, -150.0, red)            # a wall
    with s.translate((40.0, 0.0, 20.0)), s.rotate_y(-18.0):
        s.cuboid((0.0, 0.0, 0.0), (60.0, 120.0, 60.0), white)
    text = s.dump()
    s.commit()
    if case == "far_origin":  # camera rays start at |o.z| >= 2^62: those chains' z guard fails, those lanes divide
        cam = rtw.Camera.new((50.0, 80.0, 1e19), (50.0, 40.0, 0.0), (0, 1, 0), 50.0, 1.0, 0.0, 10.0)
    else:
        cam = rtw.Camera.new((50.0, 80.0, 400.0), (50.0, 40.0, 0.0), (0, 1, 0), 50.0, 1.0, 0.0, 10.0)
    w, h, spp = 32, 32, 4
    g, st = rtw.Raytracer(s, cam, (0.1, 0.1, 0.1), w, h, spp, seed=3).render()
    r, rays = orc.OracleScene(text).render(orc.camera_from_fields(cam.as_dict()), (0.1, 0.1, 0.1), w, h, spp, seed=3)
    assert st["rays"] == rays
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32))
    assert np.isfinite(g).all() and g.max() > 0
