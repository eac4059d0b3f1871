"""C-ABI checks that need no GPU: the library loads, exports every symbol include/rtw.h
declares, builder errors match the reference's panics, host-side pieces (camera, tonemap,
flattener) agree with the oracle.  Nothing here launches a kernel."""
import re
from pathlib import Path

import numpy as np
import pytest

REF_MODELS = Path("/root/reference/models")

ROOT = Path(__file__).resolve().parents[1]


def header_functions():
    text = (ROOT / "include" / "rtw.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rtw_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(rtw):
    lib = rtw.lib()
    declared = header_functions()
    assert len(declared) >= 30
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert set(declared) == set(rtw.EXPORTED_SYMBOLS), set(declared) ^ set(rtw.EXPORTED_SYMBOLS)
    assert lib.rtw_abi_version() == rtw.ABI_VERSION


def test_camera_matches_oracle(rtw, orc):
    """camera.rs:25-64 restated twice (product host C++ vs oracle C): bit-identical."""
    cases = [((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 16 / 9, 0.1, 10.0),
             ((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, 1.0, 0.0, 10.0),
             ((-5, -30, 25), (0, 0, 5), (1, 0, 0), 40.0, 3840 / 2160, 0.0, 10.0),
             ((0.5, 2.5, 0.8), (-0.1, 2.3, 0.15), (0, 1, 0), 40.0, 1.3, 0.5, 3.3)]
    for a in cases:
        p = rtw.Camera.new(*a).as_dict()
        o = orc.camera_new(*a)
        for k, _ in orc.oracle_camera._fields_:
            pv = np.asarray(p[k], np.float32)
            ov = np.asarray(list(getattr(o, k)) if isinstance(p[k], list) else getattr(o, k), np.float32)
            assert np.array_equal(pv.view(np.uint32), ov.view(np.uint32)), (a, k, pv, ov)


def test_camera_rejects_empty_shutter(rtw):
    with pytest.raises(rtw.RtwError) as e:
        rtw.Camera.new((0, 0, 1), (0, 0, 0), (0, 1, 0), 40, 1, 0, 1, 0.5, 0.5)  # gen_range panics on empty
    assert e.value.code == rtw.RTW_EINVAL


def test_tonemap_matches_oracle(rtw, orc):
    rng = np.random.default_rng(1)
    sums = np.concatenate([rng.uniform(-1, 60, 3000), [np.nan, np.inf, -np.inf, 0, 50]]).astype(np.float32)
    sums = sums[: (len(sums) // 3) * 3].reshape(-1, 3)
    got = rtw.tonemap(sums, 50)
    want = np.array([[orc.lib().oracle_tonemap(float(x), 50) for x in row] for row in sums], np.uint8)
    assert np.array_equal(got, want)


def test_metal_fuzz_assert(rtw):
    s = rtw.Scene()
    s.metal((0.5, 0.5, 0.5), 1.0)
    with pytest.raises(rtw.RtwError) as e:
        s.metal((0.5, 0.5, 0.5), 1.01)  # material.rs:71 assert!(fuzz <= 1.0)
    assert e.value.code == rtw.RTW_EINVAL


def test_builder_errors(rtw):
    s = rtw.Scene()
    with pytest.raises(rtw.RtwError):
        s.sphere((0, 0, 0), 1, 7)  # no such material
    with pytest.raises(rtw.RtwError):
        s.checker(0, 1, 10)  # no such textures
    assert rtw.lib().rtw_end(s._p) == rtw.RTW_ESTATE  # no open group
    m = s.lambertian_solid((0.5, 0.5, 0.5))
    assert rtw.lib().rtw_begin_translate(s._p, 1, 2, 3) == 0
    with pytest.raises(rtw.RtwError) as e:  # a group is still open
        s.commit()
    assert e.value.code == rtw.RTW_ESTATE
    assert rtw.lib().rtw_end(s._p) == 0
    assert rtw.lib().rtw_end(s._p) == rtw.RTW_ESTATE  # nothing open
    with pytest.raises(rtw.RtwError) as e:
        rtw.Scene().load_wavefront_obj("/nonexistent.obj")
    assert e.value.code == rtw.RTW_EIO
    del m


@pytest.mark.parametrize("name", ["jumpy-balls", "cornell-box", "wavefront-cow-obj", "textured-monument",
                                  "two-spheres", "simple-triangle"])
def test_flatten_self_check(rtw, name):
    """rtw_scene_commit flattens + builds the BVH (with its structural self-check) before it
    needs a device; on a GPU-less host the only acceptable failure is RTW_ENODEV."""
    s = rtw.Scene()
    s.preset(name, 16 / 9, seed=3)
    leaves = s.info(0)
    if rtw.device_count() > 0:
        s.commit()
    else:
        with pytest.raises(rtw.RtwError) as e:
            s.commit()
        assert e.value.code == rtw.RTW_ENODEV, str(e.value)
    nodes, depth, always = s.info(3), s.info(4), s.info(5)
    assert depth <= 31
    if leaves <= 32:  # list mode (rtw_flatten.cpp list_max): no BVH, every ray tests every leaf
        assert nodes == 0 and always == leaves
    else:
        assert nodes >= 1
    if name == "jumpy-balls":
        assert always == 1  # the r=1000 ground sphere is tested for every ray, not in the BVH
        assert nodes < 2 * leaves


def test_presets_unknown_scene(rtw):
    s = rtw.Scene()
    with pytest.raises(rtw.RtwError) as e:
        s.preset("no-such-scene", 1.0)
    assert "unknown" in str(e.value)


@pytest.mark.skipif(not (REF_MODELS / "Normals_Try3.obj").exists(), reason="reference models not mounted")
def test_suspension_obj_fails_like_the_reference(rtw):
    """scenes.rs:773-814 loads Normals_Try3.obj, whose `usemtl` has no `mtllib`: the reference
    panics at triangular.rs:176 (unwrap); the preset returns RTW_EIO."""
    s = rtw.Scene()
    with pytest.raises(rtw.RtwError) as e:
        s.preset("wavefront-suspension-obj", 16 / 9, models_dir=REF_MODELS)
    assert e.value.code == rtw.RTW_EIO and "usemtl without mtllib" in str(e.value)


def test_image_height_rule(rtw):
    """console_app/src/main.rs:33: round(width / 1.7777778)."""
    assert rtw.image_height(400) == 225
    assert rtw.image_height(1920) == 1080
    assert rtw.image_height(3840) == 2160
    assert rtw.camera_aspect(1920, 1080) == np.float32(1920) / np.float32(1080)


def test_abi_version_matches_header(rtw):
    import pathlib
    text = (pathlib.Path(__file__).resolve().parents[1] / "include" / "rtw.h").read_text()
    assert int(re.search(r"#define RTW_ABI_VERSION (\d+)", text).group(1)) == rtw.ABI_VERSION


def _commit_anywhere(rtw, s):
    if rtw.device_count() > 0:
        s.commit()
    else:
        with pytest.raises(rtw.RtwError):
            s.commit()


@pytest.mark.parametrize("name", ["jumpy-balls", "wavefront-cow-obj", "textured-monument", "book2-final-scene"])
def test_bvh4_breadth_first_codes_and_bounds(rtw, name):
    """rtw_flatten.cpp: node4s are numbered breadth-first (every internal child's index is larger than
    its parent's and children appear in visit order), each child's 16-bit code (DevNode4::code, the
    LDS-node kernels' stack entries) decodes to the same child as its 32-bit child word, and the
    sorted-push walk's stack bound (info 11) covers the 32-bit walk's (info 8) plus its 4-row window
    over a root-to-leaf path (recomputed here from the nodes)."""
    s = rtw.Scene()
    s.preset(name, 16 / 9, seed=3)
    _commit_anywhere(rtw, s)
    nd = s.nodes()
    assert len(nd) == s.info(3) > 0
    empty = nd["lo_x"] > nd["hi_x"]
    nxt = 1
    for i in range(len(nd)):
        for k in range(4):
            if empty[i, k]:
                assert nd["code"][i, k] == 0
                continue
            w, c = int(nd["child"][i, k]), int(nd["code"][i, k])
            if w >= 0:
                assert w == nxt and c == w  # breadth-first: the next unnumbered index
                nxt += 1
            else:
                v = ~w & 0xFFFFFFFF
                first, cnt = v >> 3, v & 7
                assert c & 0x8000 and ((c >> 2) & 0x1FFF) == first and (c & 3) + 1 == cnt
    assert nxt == len(nd)

    def bound4(i):  # max over paths of sum(children - 1) + 4 (rtw_flatten.cpp Collapse::build)
        ch = [k for k in range(4) if not empty[i, k]]
        inner = [int(nd["child"][i, k]) for k in ch if nd["child"][i, k] >= 0]
        return max(4, len(ch) - 1 + max(bound4(j) for j in inner)) if inner else 4
    assert s.info(11) == bound4(0) >= s.info(8)


def test_camera_reciprocal_is_correctly_rounded(rtw):
    """rtw_render's camera divisions (lib.rs:84-85) use Markstein's correction from the host's
    RN(1 / (w - 1)) and RN(1 / (h - 1)) (rtw_kernel.hip recip_rn): it must be the IEEE f32 reciprocal
    for every image size (w, h <= 65536) and beyond, up to 2^24."""
    b = np.concatenate([np.arange(1, 65536), np.arange(65536, 1 << 24, 4099), [(1 << 24) - 1]]).astype(np.float32)
    got = rtw.diag_recip(b)
    want = (np.float32(1.0) / b).astype(np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name", ["jumpy-balls", "wavefront-cow-obj", "textured-monument", "book2-final-scene"])
def test_half_nodes_contain_the_f32_boxes(rtw, name):
    """DevNode4h (rtw_flatten.cpp half_node): every child's f16 box, origin + offsets, contains its padded
    f32 box (lo rounded down, hi up), so the half-precision walk culls conservatively; empty slots stay
    inverted; the two plane orders agree; the codes are DevNode4's; no f16 subnormal reaches the kernel
    (the origin is normal or zero, offsets normal or zero)."""
    s = rtw.Scene()
    s.preset(name, 16 / 9, seed=3)
    _commit_anywhere(rtw, s)
    nd, nh = s.nodes(), s.nodes_half()
    assert len(nh) == len(nd) > 0
    for ax in ("x", "y", "z"):
        lo32, hi32 = nd["lo_" + ax].astype(np.float64), nd["hi_" + ax].astype(np.float64)
        h = nh[ax]
        org = nh["origin"][:, "xyz".index(ax)].astype(np.float64)
        lo16, hi16 = h[:, 0, :4].astype(np.float64), h[:, 0, 4:].astype(np.float64)
        assert np.array_equal(h[:, 1, :4].view(np.uint16), h[:, 0, 4:].view(np.uint16))
        assert np.array_equal(h[:, 1, 4:].view(np.uint16), h[:, 0, :4].view(np.uint16))
        empty = nd["lo_x"] > nd["hi_x"]
        assert np.all(np.isposinf(lo16[empty])) and np.all(np.isneginf(hi16[empty]))
        full = ~empty
        with np.errstate(invalid="ignore"):
            assert np.all((org[:, None] + lo16 <= lo32)[full]), ax
            assert np.all((org[:, None] + hi16 >= hi32)[full]), ax
        bits = h.view(np.uint16)
        sub = ((bits & 0x7C00) == 0) & ((bits & 0x3FF) != 0)
        assert not sub.any()
        ob = nh["origin"].view(np.uint16)
        assert not (((ob & 0x7C00) == 0) & ((ob & 0x3FF) != 0)).any()
    assert np.array_equal(nh["code"].astype(np.uint32), nd["code"])


@pytest.mark.parametrize("offset,built", [(-1.0e5, False), (-6.0e4, True), (1.0e5, True)])
def test_half_nodes_beyond_f16_range(rtw, offset, built):
    """a child box whose lower bound is below -65504 would get an f16 origin of -inf (every offset
    +inf, every plane NaN).  The flattener then builds no half-precision table (the kernels walk the f32
    one); bounds above +65504 round outward to +inf offsets (conservative) and keep it."""
    rng = np.random.default_rng(7)
    s = rtw.Scene()
    m = s.lambertian_solid((0.5, 0.5, 0.5))
    n = 600
    base = rng.uniform(-50, 50, (n, 1, 3)) + np.array([offset, 0.0, 0.0])
    verts = (base + rng.uniform(-1, 1, (n, 3, 3))).astype(np.float32)
    with s.bvh():
        s.triangles(verts.reshape(-1), m)
    _commit_anywhere(rtw, s)
    nd, nh = s.nodes(), s.nodes_half()
    assert len(nd) > 4
    assert (len(nh) == len(nd)) == built
    if built:
        for ax in ("x", "y", "z"):
            org = nh["origin"][:, "xyz".index(ax)].astype(np.float64)
            assert np.all(np.isfinite(org)), ax
            lo16 = nh[ax][:, 0, :4].astype(np.float64)
            full = ~(nd["lo_x"] > nd["hi_x"])
            with np.errstate(invalid="ignore"):
                assert np.all((org[:, None] + lo16 <= nd["lo_" + ax])[full]), ax


@pytest.mark.parametrize("knob", ["RTW_BVH_PAIR=1", "RTW_BVH_PAIR=3", "RTW_BVH_BINS=64", "RTW_BVH_LEAF=2"])
def test_bvh_build_knobs_cover_every_prim(rtw, knobs, knob):
    """The SAH build knobs (RTW_BVH_PAIR / BINS / LEAF) only reshape the tree: the flattener's own
    self-check (every node4 reached once, every BVH prim in exactly one leaf) passes, the leaves' prim ranges
    cover the BVH part once, and the 16-bit codes still hold (leaves of <= 4 prims)."""
    k, v = knob.split("=")
    knobs.setenv(k, v)
    for name in ("jumpy-balls", "wavefront-cow-obj"):
        s = rtw.Scene()
        s.preset(name, 16 / 9, seed=42)
        _commit_anywhere(rtw, s)
        nd = s.nodes()
        assert len(nd) == s.info(3) > 4
        full = ~(nd["lo_x"] > nd["hi_x"])
        leaf = full & ((nd["code"] & 0x8000) != 0)
        first, cnt = (nd["code"][leaf] >> 2) & 0x1FFF, (nd["code"][leaf] & 3) + 1
        cover = np.zeros(int((first + cnt).max()), np.int32)
        for f, c in zip(first, cnt):
            cover[f:f + c] += 1
        assert np.all(cover == 1), name
        assert s.info(11) >= 4


def test_tuning_knobs_need_the_gate(rtw, monkeypatch, capfd):
    """a stray tuning variable must not change the product's kernels.  RTW_LIST_MAX=0 (BVH
    instead of list mode, read by the flattener at commit) takes effect only with RTW_TUNING=1; without the
    gate it is ignored with a warning on stderr, and cornell-box stays a BVH-less list-mode world."""
    monkeypatch.delenv("RTW_TUNING", raising=False)
    monkeypatch.setenv("RTW_LIST_MAX", "0")
    s = rtw.Scene()
    s.preset("cornell-box", 1.0, seed=3)
    _commit_anywhere(rtw, s)
    assert s.info(3) == 0 and s.info(5) > 0  # list mode: no BVH nodes, every prim always tested
    assert "RTW_LIST_MAX=0 ignored" in capfd.readouterr().err
    monkeypatch.setenv("RTW_TUNING", "1")
    s = rtw.Scene()
    s.preset("cornell-box", 1.0, seed=3)
    _commit_anywhere(rtw, s)
    assert s.info(3) > 0  # the knob applies: a BVH over the rects


def test_alias_devices_arguments(rtw):
    """rtw_diag_alias_devices (the one-GPU rehearsal of rtw_render_multi, tests/test_gpu_multi.py): 1..64
    logical devices, before the commit only."""
    s = rtw.Scene()
    for bad in (0, -1, 65):
        with pytest.raises(rtw.RtwError) as e:
            s.diag_alias_devices(bad)
        assert e.value.code == rtw.RTW_EINVAL
    s.diag_alias_devices(8)
    s.diag_alias_devices(2)  # may be changed until the commit


def test_list_runs_and_rect_fast_flag(rtw):
    """The list-mode rect loop's program (DevScene::lgroups, rtw_scene_info 12): cornell-box's 18 always-tested
    rects form 5 runs of one wrapper chain, in list order (the room's yz yz | xz xz xz | xy, then each box's
    xy xy xz xz yz yz as one whole-Cuboid run, GK_BOX6); its fast path (info 13) needs |k| < 2^62 and ordered bounds on every rect,
    which a plane at 1e19, an inverted rect or an infinite bound revokes."""
    s = rtw.Scene()
    s.preset("cornell-box", 1.0, seed=3)
    _commit_anywhere(rtw, s)
    assert (s.info(5), s.info(12), s.info(13)) == (18, 5, 1)
    for k, bounds in ((1e19, (0.0, 1.0, 0.0, 1.0)), (1.0, (1.0, 0.0, 0.0, 1.0)), (1.0, (0.0, float("inf"), 0.0, 1.0)),
                      (1.0, (0.0, 1.0, float("-inf"), 1.0))):  # (infinite bounds: ADVICE r5)
        s = rtw.Scene()
        m = s.lambertian_solid((0.5, 0.5, 0.5))
        s.xy_rect(0.0, 1.0, 0.0, 1.0, 0.0, m)
        s.xy_rect(bounds[0], bounds[1], bounds[2], bounds[3], k, m)
        _commit_anywhere(rtw, s)
        assert s.info(5) == 2 and s.info(12) == 1 and s.info(13) == 0


def _sphere_reach(D, r):
    """rtw_flatten.cpp sphere_reach: how far outside a radius-r sphere the reference's f32 test (spherical.rs:26-44)
    can report a hit for an origin D from its centre (the first-order bound of DESIGN.md §2, 37u -> 40u)."""
    ku = 40.0 * 2.0 ** -24
    x = ku * (D * D + r * r)
    return min(x / (2 * r), np.sqrt(x)) + 2.0 ** -24 * D


def test_far_bound_pads_sphere_leaves(rtw):
    """Round 6, VERDICT r5 item 1: a BVH holding spheres gets the far-origin bound (rtw_scene_info 14), with D0 the
    diagonal of the BVH's box (info 15).  Every sphere leaf of jumpy-balls is padded by at least its reach at D0 (a
    0.2 ball's leaf spans >= 2 (0.2 + reach)), so origins within D0 -- the camera and every bounce among the balls --
    cull nothing the reference's flat list hits.  Worlds without BVH spheres (the cow's triangle-only tree, cornell's
    list mode) need no bound."""
    s = rtw.Scene()
    s.preset("jumpy-balls", 16 / 9, seed=42)
    _commit_anywhere(rtw, s)
    assert s.info(14) == 1
    d0 = s.info(15) / 1000.0
    nd = s.nodes()
    full = ~(nd["lo_x"] > nd["hi_x"])
    lo = np.stack([nd["lo_" + a][0][full[0]].min() for a in "xyz"])
    hi = np.stack([nd["hi_" + a][0][full[0]].max() for a in "xyz"])
    diag = float(np.linalg.norm(hi - lo))
    e = _sphere_reach(d0, 0.2)
    assert 30.0 < d0 <= diag and d0 >= diag - 2 * np.sqrt(3) * (e + 1e-3), (d0, diag)
    leaf = full & ((nd["code"] & 0x8000) != 0)
    ext = np.stack([(nd["hi_" + a] - nd["lo_" + a])[leaf] for a in "xyz"]).min(axis=0)
    assert ext.min() >= 2 * (0.2 + e), (ext.min(), e)
    for name, aspect in (("wavefront-cow-obj", 16 / 9), ("cornell-box", 1.0)):
        s = rtw.Scene()
        s.preset(name, aspect, seed=42)
        _commit_anywhere(rtw, s)
        assert s.info(14) == 0, name
