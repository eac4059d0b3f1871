"""BASELINE.json configs[0] at its own size, and the error / multi-device paths.

configs[0] is console_app's default jumpy-balls run at 400x225, 50 spp (console_app/src/main.rs:15-64,
scenes.rs:63-162).  The whole frame is rendered through rtw_render and compared bit for bit, with
its ray count, against the oracle; rtw_console (the console_app mirror) is run at that config and its
PNG is checked against rtw_tonemap of the GPU sums (main.rs:68-94).
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
SCENE_SEED, RENDER_SEED = 42, 2024  # bench.py's seeds (the jumpy-400 bench line renders this frame)


def test_config0_jumpy_400x225x50_whole_frame_bit_exact(gpu, orc):
    rtw = gpu
    w = 400
    h = rtw.image_height(w)  # main.rs:33: 225
    assert h == 225
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", rtw.camera_aspect(w, h), seed=SCENE_SEED)
    text, imgs = s.dump(), s.images()
    s.commit(device=0)
    img, st = rtw.Raytracer(s, cam, bg, w, h, 50, seed=RENDER_SEED).render()
    ref, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, 50,
                                                   seed=RENDER_SEED, threads=min(256, os.cpu_count() or 1))
    assert st["rays"] == rays, (st["rays"], rays)
    assert st["paths"] == w * h * 50
    bad = img.view(np.uint32) != ref.view(np.uint32)
    assert not bad.any(), f"{int(bad.sum())} of {bad.size} components differ"
    assert rays > w * h * 50  # every path traced its camera ray, most scattered


def test_config0_console_png(gpu, tmp_path):
    """`rtw_console jumpy-balls -w 400 -s 50` (console_app's Opts, main.rs:15-26, 33): one 400x225 PNG
    under --out named image_0000.png, equal byte for byte to rtw_tonemap(rtw_render) of that frame."""
    from PIL import Image
    rtw = gpu
    exe = ROOT / "raytracer-weekend_amd" / "bin" / "rtw_console"
    assert exe.exists(), "rtw_console not built"
    r = subprocess.run([str(exe), "jumpy-balls", "-w", "400", "-s", "50", "--seed", str(SCENE_SEED),
                        "--models", str(rtw.MODELS_DIR), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    pngs = sorted(tmp_path.glob("image_*.png"))
    assert [p.name for p in pngs] == ["image_0000.png"]
    got = np.asarray(Image.open(pngs[0]).convert("RGB"))
    assert got.shape == (225, 400, 3)
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", rtw.camera_aspect(400, 225), seed=SCENE_SEED)
    s.commit()
    sums, _ = rtw.Raytracer(s, cam, bg, 400, 225, 50, seed=SCENE_SEED).render()
    want = rtw.tonemap(sums, 50)
    assert np.array_equal(got, want), f"{int((got != want).sum())} bytes differ"


def _sphere_cloud(rtw, n=200, seed=4):
    """Spheres of one size (no always-tested prim: every ray goes through the BVH walk)."""
    rng = np.random.default_rng(seed)
    s = rtw.Scene()
    m = s.lambertian_solid((0.5, 0.6, 0.7))
    s.spheres(np.stack([rng.uniform(-4, 4, n), rng.uniform(-2, 2, n), rng.uniform(-4, 4, n)], 1),
              rng.uniform(0.1, 0.3, n), np.full(n, m))
    cam = rtw.Camera.new((0, 0, 12), (0, 0, 0), (0, 1, 0), 40.0, 1.0, 0.0, 12.0)
    return s, cam, (0.7, 0.8, 1.0)


@pytest.mark.parametrize("knob", ["", "RTW_LDS_NODES=0"])
def test_corrupt_bvh_fails_every_path(gpu, knobs, knob):
    """A cyclic node table (rtw_diag_corrupt_bvh) trips the traversal guard.  Renders enqueued
    without stats (bench.py's timed frames, the torchrun N>1 path) return RTW_OK, and the fault
    surfaces at rtw_render_status, at the next render call and at rtw_path_kernel_times; a render with
    stats fails itself.  Both walks: the LDS-node kernel (16-bit codes) and the global-node one."""
    torch = pytest.importorskip("torch")
    if knob:
        knobs.setenv(*knob.split("="))
    rtw = gpu
    s, cam, bg = _sphere_cloud(rtw)
    s.commit(device=0)
    assert s.info(3) >= 2 and s.info(5) == 0
    rt = rtw.Raytracer(s, cam, bg, 8, 8, 1, seed=1)  # one wave: each walk runs 2^20 node-loop iterations
    good, _ = rt.render()
    s.render_status(0)  # nothing tripped yet
    s.diag_corrupt_bvh(0)
    out = torch.zeros((8, 8, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    rt.render_device(out.data_ptr(), 0, 0, 0, stream)  # enqueued: no error yet
    with pytest.raises(rtw.RtwError) as e:
        s.render_status(0)
    assert e.value.code == rtw.RTW_EINVAL and "guard" in str(e.value)
    s.render_status(0)  # reported once, then cleared
    rt.render_device(out.data_ptr(), 0, 0, 0, stream)
    torch.cuda.synchronize()
    with pytest.raises(rtw.RtwError) as e:  # the next call reports the previous frame's fault
        rt.render_device(out.data_ptr(), 0, 0, 0, stream)
    assert e.value.code == rtw.RTW_EINVAL
    rt.render_device(out.data_ptr(), 0, 0, 0, stream)
    with pytest.raises(rtw.RtwError):  # bench.py's read of the kernel times after the timed steps
        s.path_kernel_times(0)
    with pytest.raises(rtw.RtwError):
        rt.render()
    del good


@pytest.mark.parametrize("knob", ["", "RTW_LDS_NODES=0"])
def test_corrupt_bvh_frame_drains_after_one_trip_per_wave(gpu, knobs, knob):
    """after a guard trip the kernel closes the path queue and empties the wave's id pool, so a
    large corrupt frame costs about one trip per wave, not one per 64 paths.  A 256x256x16 frame (16 K
    64-path groups, ~1 K waves with work) must take at most 8x the path-kernel time of an 8x8x1 frame (one
    wave, one trip); without the drain every wave runs ~16 trips in a row.  A smoke check on device time (the
    library's HIP events around the launch, rtw_path_kernel_times, read after rtw_render_status has reported and
    cleared the fault), not on host wall clock."""
    torch = pytest.importorskip("torch")
    if knob:
        knobs.setenv(*knob.split("="))
    rtw = gpu
    s, cam, bg = _sphere_cloud(rtw)
    s.commit(device=0)
    s.diag_corrupt_bvh(0)
    stream = torch.cuda.current_stream().cuda_stream

    def timed(w, h, spp):
        out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
        rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=1)
        torch.cuda.synchronize()
        s.path_kernel_times(0)  # forget earlier launches
        rt.render_device(out.data_ptr(), 0, 0, 0, stream)
        torch.cuda.synchronize()
        with pytest.raises(rtw.RtwError):
            s.render_status(0)  # reports the fault and clears it
        t = s.path_kernel_times(0)
        assert len(t) == 1
        return t[0]

    timed(8, 8, 1)  # warm-up (buffers, code objects)
    small = timed(8, 8, 1)
    big = timed(256, 256, 16)
    print(f"corrupt frames, path-kernel ms: 8x8x1 {small:.3f}, 256x256x16 {big:.3f}")
    assert big <= 8.0 * small + 5.0, (small, big)


def test_render_multi_one_gpu_needs_no_rccl(gpu, monkeypatch):
    """rtw_render_multi over one device is rtw_render's path: it never opens RCCL, so it
    works with the RCCL library made unloadable, and equals rtw_render bit for bit."""
    monkeypatch.setenv("RTW_RCCL_LIB", "/nonexistent/librccl.so.1")
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", 16 / 9, seed=3)
    s.commit()
    rt = rtw.Raytracer(s, cam, bg, 72, 40, 3, seed=9)
    ref, st = rt.render()
    got, st2 = rt.render_multi(1)
    assert st2["rays"] == st["rays"] and st2["kernel_ms"] > 0
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_strided_tiles_match_full_frame(gpu):
    """rtw_render_device_strided (a device's round-robin share, tiles computed by the kernel) packs the
    same pixels as the id-table path; unpacked over all parts it rebuilds rtw_render's frame."""
    torch = pytest.importorskip("torch")
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", 16 / 9, seed=3)
    s.commit(device=0)
    w, h, spp = 72, 40, 2  # ragged: 9 x 5 tiles
    rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=5)
    full, st = rt.render()
    stream = torch.cuda.current_stream().cuda_stream
    for world in (1, 2, 3, 7):
        img = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
        rays = 0
        for rank in range(world):
            pad, n = rtw.tile_partition(w, h, world, rank)
            ids = torch.tensor(pad.astype(np.int32), device="cuda:0")
            packed = torch.zeros((len(pad), 64, 3), dtype=torch.float32, device="cuda:0")
            stp = rt.render_device_strided(packed.data_ptr(), 0, rank, world, n, stream, want_stats=True)
            rays += stp["rays"]
            via_ids = torch.zeros_like(packed)
            rt.render_device(via_ids.data_ptr(), 0, ids.data_ptr(), n, stream)
            torch.cuda.synchronize()
            assert torch.equal(packed[:n].view(torch.int32), via_ids[:n].view(torch.int32)), (world, rank)
            rtw.unpack_tiles_device(w, h, ids.data_ptr(), len(pad), packed.data_ptr(), img.data_ptr(), 0, stream)
        torch.cuda.synchronize()
        assert rays == st["rays"], world
        assert np.array_equal(img.cpu().numpy().view(np.uint32), full.view(np.uint32)), world
