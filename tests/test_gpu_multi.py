"""rtw_render_multi's n > 1 path on a one-GPU box (reference: Rayon over the pixels of
Raytracer::render, raytracer_weekend_lib/src/lib.rs:57-67).

rtw_diag_alias_devices(scene, n) makes the scene's devices n logical devices on physical device 0, each with
its own scene copy, stream, path queue, sample buffer and packed buffer; the loopback RCCL stand-in
(tests/loopback_rccl, test infrastructure loaded through the library's RTW_RCCL_LIB knob) carries the grouped
ncclSend / ncclRecv as stream-ordered device copies.  So everything of the n > 1 path but RCCL's own transport
runs here: the round-robin tile split, the per-device strided renders into packed buffers, the send / recv
group and its gather offsets, the padding ids, the unpack on device 0 and the per-device timings.  The frame
must equal rtw_render's bit for bit with the same ray count (pixels depend only on (seed, j, i, sample)).
The real RCCL calls over xGMI stay unmeasured until a multi-GPU node runs them.
"""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOOPBACK = Path(__file__).resolve().parent / "loopback_rccl" / "libloopback_rccl.so"


@pytest.fixture
def loopback(monkeypatch):
    assert LOOPBACK.exists(), "tests/loopback_rccl not built (__graft_entry__.build())"
    monkeypatch.setenv("RTW_RCCL_LIB", str(LOOPBACK))


def _single_and_multi(rtw, name, aspect, n, w, h, spp, seed=5):
    one = rtw.Scene()
    cam, bg = one.preset(name, aspect, seed=3)
    one.commit(device=0)
    ref, st_ref = rtw.Raytracer(one, cam, bg, w, h, spp, seed=seed).render()
    many = rtw.Scene()
    many.preset(name, aspect, seed=3)
    many.diag_alias_devices(n).commit()
    rt = rtw.Raytracer(many, cam, bg, w, h, spp, seed=seed)
    return ref, st_ref, rt, many


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name,aspect,w,h,spp", [
    ("jumpy-balls", 16 / 9, 72, 40, 3),       # ragged: 9 x 5 tiles, the last tile row half outside
    ("cornell-box", 1.0, 40, 40, 4),          # list mode
    ("wavefront-cow-obj", 16 / 9, 48, 27, 2),  # mesh kernel, half-precision nodes
    ("textured-monument", 16 / 9, 64, 36, 1),  # configs[4]'s scene (its 8-way split), image texture
])
def test_render_multi_equals_render(gpu, loopback, name, aspect, w, h, spp, n):
    rtw = gpu
    ref, st_ref, rt, many = _single_and_multi(rtw, name, aspect, n, w, h, spp)
    for rep in range(2):  # the second call reuses the clique, streams and grown buffers
        img, st = rt.render_multi(n)
        bad = np.argwhere(img.view(np.uint32) != ref.view(np.uint32))
        assert bad.size == 0, f"{name} n={n} rep={rep}: {len(bad)} components differ, first {bad[:4].tolist()}"
        assert st["rays"] == st_ref["rays"], (st["rays"], st_ref["rays"])
        assert st["paths"] == w * h * spp
        dev_ms, gather_ms = many.multi_times()
        assert len(dev_ms) == n and all(t >= 0 for t in dev_ms) and max(dev_ms) > 0 and gather_ms >= 0.0


@pytest.mark.parametrize("n", [3, 8])
def test_render_multi_fewer_tiles_than_devices(gpu, loopback, n):
    """A 16 x 8 frame has 2 tiles: devices 2.. render nothing, send only padding, and the unpack skips it."""
    rtw = gpu
    ref, st_ref, rt, many = _single_and_multi(rtw, "jumpy-balls", 16 / 9, n, 16, 8, 4)
    img, st = rt.render_multi(n)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    assert st["rays"] == st_ref["rays"]
    dev_ms, _ = many.multi_times()
    assert len(dev_ms) == n


def test_render_multi_equals_oracle(gpu, orc, loopback):
    """The gathered frame against the CPU oracle directly (4 logical devices, ragged cornell frame)."""
    rtw = gpu
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0, seed=3)
    text = s.dump()
    s.diag_alias_devices(4).commit()
    w, h, spp = 36, 20, 3
    img, st = rtw.Raytracer(s, cam, bg, w, h, spp, seed=9).render_multi(4)
    ref, rays = orc.OracleScene(text).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=9)
    assert st["rays"] == rays
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_aliased_scene_renders_per_logical_device(gpu, loopback):
    """Every logical device holds its own copy: rtw_render_device on device d of an aliased scene (what one
    rank of bench.py's torchrun path does with its strided share) fills its packed tiles like device 0's."""
    torch = pytest.importorskip("torch")
    rtw = gpu
    ref, _, rt, many = _single_and_multi(rtw, "jumpy-balls", 16 / 9, 3, 48, 24, 2)
    w, h = 48, 24
    img = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for d in range(3):
        ids, k = rtw.tile_partition(w, h, 3, d)
        packed = torch.zeros((k, 64, 3), dtype=torch.float32, device="cuda:0")
        rt.render_device_strided(packed.data_ptr(), d, d, 3, k, stream)
        d_ids = torch.from_numpy(ids[:k].astype(np.int32)).to("cuda:0")
        rtw.unpack_tiles_device(w, h, d_ids.data_ptr(), k, packed.data_ptr(), img.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    for d in range(3):
        many.render_status(d)


def test_bench_multi_device_branch_runs(gpu):
    """bench.py's single-process N > 1 branch (rtw_render_multi, the driver's `--gpus 8` without a
    launcher) executed end to end before the first real 8-GPU node runs it: configs[4]'s scene over 8 logical devices
    of this GPU (--diag-alias, the loopback RCCL), 1 spp, as a fresh process.  The line must say n_gpus 8, carry eight
    per-device path-kernel times (each device's launches read once) and a gathered frame equal to the single-device
    render (--check-image)."""
    import json
    import os
    import subprocess
    import sys
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, RTW_RCCL_LIB=str(LOOPBACK))
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--multi-device", "8", "--diag-alias", "--config",
                        "monument-4k", "--spp", "1", "--steps", "2", "--warmup", "1", "--check-image",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert any(x.get("check_image") is True for x in lines), r.stdout
    d = lines[-1]
    assert d["n_gpus"] == 8 and d["config"]["diag_alias_devices"] == 8
    dk = d["multi_gpu"]["device_kernel_ms_per_frame"]
    assert len(dk) == 8 and all(x is not None and x > 0 for x in dk), dk
    assert len(d["multi_gpu"]["device_render_ms_per_frame"]) == 8
