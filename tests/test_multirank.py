"""World-size-2 frame partition + gather on CPU (gloo): the N>1 path of bench.py.

Each rank "renders" its tiles with a deterministic stand-in (pixel value = f(row, col)),
packs them as rtw_render_device does, all-gathers, and rank 0 unpacks with the index math
of unpack_tiles_kernel; the result must equal the single-rank frame for ragged sizes."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def fake_pixel(row, col):
    return np.stack([row * 1000.0 + col, row + 0.5, col * 0.25], -1).astype(np.float32)


def unpack(w, h, ids, packed):
    """CPU restatement of unpack_tiles_kernel (rtw_kernel.hip) for the test."""
    sys.path.insert(0, str(ROOT / "tests"))
    from conftest import load_rtw
    T = load_rtw()
    import importlib
    tiles = importlib.import_module("rtw_amd.tiles")
    img = np.zeros((h, w, 3), np.float32)
    for slot, t in enumerate(ids):
        if t >= tiles.n_tiles(w, h):
            continue
        r, c = tiles.tile_pixels(int(t), w, h)
        ok = (r < h) & (c < w)
        img[r[ok], c[ok]] = packed[slot][ok]
    return img


def worker(rank, world, w, h, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(ROOT / "tests"))
    from conftest import load_rtw
    load_rtw()
    import importlib
    tiles = importlib.import_module("rtw_amd.tiles")
    nt = tiles.n_tiles(w, h)
    pr = tiles.per_rank(nt, world)
    mine = tiles.rank_tiles(nt, world, rank)
    packed = np.zeros((pr, 64, 3), np.float32)
    for k, t in enumerate(mine):
        r, c = tiles.tile_pixels(int(t), w, h)
        packed[k] = fake_pixel(r, c)
    out = torch.zeros((world * pr, 64, 3))
    dist.all_gather_into_tensor(out, torch.from_numpy(packed))
    if rank == 0:
        img = unpack(w, h, tiles.gather_layout(nt, world), out.numpy())
        q.put(img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("w,h", [(72, 40), (64, 64), (17, 9)])
def test_two_rank_gather_rebuilds_frame(w, h):
    import torch.multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, w, h, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rows, cols = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    assert np.array_equal(img, fake_pixel(rows, cols))


def test_partition_covers_every_tile_once():
    sys.path.insert(0, str(ROOT / "tests"))
    from conftest import load_rtw
    load_rtw()
    import importlib
    tiles = importlib.import_module("rtw_amd.tiles")
    for nt in (1, 7, 32400):
        for world in (1, 2, 3, 8):
            lay = tiles.gather_layout(nt, world)
            real = np.sort(lay[lay < nt])
            assert np.array_equal(real, np.arange(nt))
            sizes = [len(tiles.rank_tiles(nt, world, r)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("w,h", [(1920, 1080), (3840, 2160), (800, 800), (17, 9)])
def test_c_abi_tile_partition_and_gather_layout(rtw, n, w, h):
    """rtw_tile_partition (what rtw_render_multi deals to each device) is the round-robin
    partition of tiles.py; the rank-major padded gather buffer that device 0 receives from the
    RCCL send/recv group, unpacked with unpack_tiles_kernel's index math, rebuilds the frame."""
    import importlib
    tiles = importlib.import_module("rtw_amd.tiles")
    nt = rtw.n_tiles(w, h)
    per = (nt + n - 1) // n
    parts = [rtw.tile_partition(w, h, n, p) for p in range(n)]
    assert all(len(ids) == per for ids, _ in parts)
    layout = np.concatenate([ids for ids, _ in parts]).astype(np.int64)
    assert np.array_equal(layout, tiles.gather_layout(nt, n))
    assert sum(k for _, k in parts) == nt and max(k for _, k in parts) - min(k for _, k in parts) <= 1
    real = layout[layout < nt]
    assert np.array_equal(np.sort(real), np.arange(nt))
    if w * h > 1_000_000:
        return  # layout checked; the pixel scatter below is exercised on the small frames
    gathered = np.zeros((n * per, 64, 3), np.float32)
    for slot, t in enumerate(layout):
        if t < nt:
            r, c = tiles.tile_pixels(int(t), w, h)
            gathered[slot] = fake_pixel(r, c)
    img = unpack(w, h, layout, gathered)
    rows, cols = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    assert np.array_equal(img, fake_pixel(rows, cols))


def test_c_abi_tile_partition_errors(rtw):
    with pytest.raises(rtw.RtwError):
        rtw.tile_partition(64, 64, 0, 0)
    with pytest.raises(rtw.RtwError):
        rtw.tile_partition(64, 64, 2, 2)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gather_layout_more_parts_than_tiles(rtw, n):
    """A frame of fewer tiles than devices: rtw_tile_partition gives the extra parts no
    tiles (n_ids = 0) and pads every part to the common size with ids equal to nt, which the unpack
    (unpack_tiles_kernel's index math) skips, so the gathered buffer still rebuilds the frame."""
    import importlib
    tiles = importlib.import_module("rtw_amd.tiles")
    w, h = 8, 8  # one tile
    nt = rtw.n_tiles(w, h)
    assert nt == 1
    parts = [rtw.tile_partition(w, h, n, p) for p in range(n)]
    assert [k for _, k in parts] == [1] + [0] * (n - 1)
    layout = np.concatenate([ids for ids, _ in parts]).astype(np.int64)
    assert layout.tolist() == [0] + [nt] * (n - 1)
    gathered = np.full((n, 64, 3), np.nan, np.float32)  # padding slots hold garbage: never read
    r, c = tiles.tile_pixels(0, w, h)
    gathered[0] = fake_pixel(r, c)
    img = unpack(w, h, layout, gathered)
    rows, cols = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    assert np.array_equal(img, fake_pixel(rows, cols))


def test_strided_render_rejects_tiles_outside_the_frame(rtw):
    """rtw_render_device_strided validates the tile progression before touching a device."""
    s = rtw.Scene()
    cam = rtw.Camera.new((0, 0, 5), (0, 0, 0), (0, 1, 0), 40, 1.0, 0.0, 1.0)
    rt = rtw.Raytracer(s, cam, (0, 0, 0), 16, 16, 1)  # 4 tiles
    for first, stride, n in ((0, 0, 1), (0, 2, 3), (4, 1, 1)):
        with pytest.raises(rtw.RtwError) as e:
            rt.render_device_strided(1, 0, first, stride, n)
        assert e.value.code == rtw.RTW_EINVAL


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rtw_bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args(**kw):
    import argparse
    d = dict(gpus=None, multi_device=0)
    d.update(kw)
    return argparse.Namespace(**d)


def test_bench_gpus_routing_without_launcher():
    """`--gpus N` always means N.  Without a launcher, N > 1 goes to the single-process
    rtw_render_multi(N) path when N GPUs are visible, and exits non-zero (no line) otherwise."""
    b = _bench_module()
    a = _args(gpus=8)
    assert b.resolve_gpus(a, world=1, visible=8) == 8 and a.gpus == 8
    a = _args()
    assert b.resolve_gpus(a, world=1, visible=8) == 0 and a.gpus == 1  # default: the one-GPU path
    a = _args(gpus=1)
    assert b.resolve_gpus(a, world=1, visible=0) == 0 and a.gpus == 1
    a = _args(multi_device=1)
    assert b.resolve_gpus(a, world=1, visible=1) == 1 and a.gpus == 1
    for kw, vis in ((dict(gpus=2), 1), (dict(gpus=8), 0), (dict(multi_device=4), 2), (dict(gpus=2, multi_device=4), 8),
                    (dict(gpus=0), 8)):
        with pytest.raises(SystemExit):
            b.resolve_gpus(_args(**kw), world=1, visible=vis)


def test_bench_gpus_routing_under_launcher():
    b = _bench_module()
    a = _args(gpus=4)
    assert b.resolve_gpus(a, world=4, visible=8) == 0 and a.gpus == 4
    a = _args()
    assert b.resolve_gpus(a, world=2, visible=8) == 0 and a.gpus == 2
    for kw in (dict(gpus=1), dict(gpus=8), dict(multi_device=4)):
        with pytest.raises(SystemExit):
            b.resolve_gpus(_args(**kw), world=4, visible=8)


def test_bench_gpus_2_without_gpus_fails_loudly():
    """`python bench.py --gpus 2` on a box without 2 visible GPUs (here: none) exits non-zero and prints no
    bench line -- never a 1-GPU number for a 2-GPU request."""
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode != 0
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            assert "n_gpus" not in json.loads(line), line
    assert "--gpus 2" in r.stderr


def test_monument_per_rank_share_is_one_pass():
    """configs[4] (monument 3840x2160x1024) over 8 GPUs: each rank's round-robin share is at most 2^32 paths, so
    enqueue_render sizes its sample buffer once for the whole share and runs ONE path-kernel pass
    (max_pass_paths = 2^32); on one GPU the frame takes two passes."""
    sys.path.insert(0, str(ROOT / "tests"))
    from conftest import load_rtw
    T = load_rtw()
    w, h, spp = 3840, 2160, 1024
    per_slot = 64 * spp
    slots_per_pass = (1 << 32) // per_slot
    for n in (1, 2, 4, 8):
        shares = [T.tile_partition(w, h, n, p)[1] for p in range(n)]
        passes = [-(-k // slots_per_pass) for k in shares]
        assert passes == [2 if n == 1 else 1] * n, (n, passes)
        if n == 8:
            assert max(shares) * per_slot * 12 < 13e9  # 12 B per path: ~12.7 GB per rank
