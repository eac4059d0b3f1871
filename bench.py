#!/usr/bin/env python3
"""bench.py — Mrays/s of the MI355X render core on BASELINE.json's headline workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config jumpy-1080p]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step = one full frame of the configured workload (default: BASELINE.json configs[1],
RTOW final random-spheres "jumpy-balls", 1920x1080, 512 spp, 50 bounces) rendered by the
hot path, with the scene already resident in HBM.  The frame's 8x8 tiles are dealt
round-robin to the N ranks (one process per GPU); each rank renders its tiles with
rtw_render_device, then one RCCL all-gather over xGMI brings every rank's packed tiles to
all ranks and rank 0 unpacks the framebuffer and copies it to the host.  Total work is
fixed as N grows ("scaling": "strong").  value = rays of the frame (world.hit queries,
lib.rs:102, counted exactly by the kernel) / max-over-ranks step time.

Also reported: `roofline` for the render kernel (algorithmic bytes per launch from the
traversal counters / its average HIP-event duration, vs 8 TB/s HBM) and `cpu_baseline`
(the oracle — the reference algorithm restated in C, flat-list closest hit — timed on the
host cores over a bounded sample of the same frame, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "raytracer-weekend_amd"

CONFIGS = {
    # name: (scene, width, height, spp, baseline config text)
    "jumpy-1080p": ("jumpy-balls", 1920, 1080, 512,
                    "Random-spheres scene, 1920x1080, 512 spp, 1xMI355X (configs[1])"),
    "cornell-800": ("cornell-box", 800, 800, 1024, "Cornell box 800x800, 1024 spp (configs[2])"),
    "cow-1080p": ("wavefront-cow-obj", 1920, 1080, 256, "cow-nonormals.obj 1920x1080, 256 spp (configs[3])"),
    "monument-4k": ("textured-monument", 3840, 2160, 1024, "monument 3840x2160, 1024 spp (configs[4])"),
    "jumpy-400": ("jumpy-balls", 400, 225, 50, "jumpy-balls 400x225, 50 spp (configs[0])"),
}
SCENE_SEED = 42      # replaces thread_rng() in scenes.rs
RENDER_SEED = 2024
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# BASELINE.md roofline definition: algorithmic bytes per ray
RAY_STATE_B = 64
NODE_BOX_B = 32            # per box tested
BOXES_PER_NODE = 4         # one DevNode4 fetch tests 4 child boxes (BVH4)
PRIM_B = [16, 36, 20, 20, 20, 36]  # sphere, moving sphere, rect xy/xz/yz, triangle


def _load(name, path, pkg_dir=None):
    if name in sys.modules:
        return sys.modules[name]
    kw = {"submodule_search_locations": [str(pkg_dir)]} if pkg_dir else {}
    spec = importlib.util.spec_from_file_location(name, path, **kw)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(rtw, scene, cam, bg, w, h, spp, budget_s: float, threads: int) -> dict:
    """The oracle (reference algorithm: flat-list closest hit, recursive sample_ray) on a
    bounded, evenly strided sample of the frame's rows, at the frame's spp."""
    orc = _load("rtw_oracle_py", ROOT / "oracle" / "oracle.py")
    o = orc.OracleScene(scene.dump(), scene.images())
    ocam = orc.camera_from_fields(cam.as_dict())
    rays = 0
    rows_done = 0
    elapsed = 0.0
    spp_s = max(1, min(spp, 8))
    order = list(range(0, h, 37)) + [j for j in range(h) if j % 37]  # strided first
    k = 0
    chunk = max(1, threads)
    while elapsed < budget_s and k < len(order):
        rows = order[k:k + chunk]
        k += chunk
        t0 = time.perf_counter()
        _, r = o.render(ocam, bg, w, h, spp_s, seed=RENDER_SEED, integrator=orc.RECURSIVE,
                        bvh_mode=orc.BVH_REFERENCE, threads=threads, rows=rows)
        elapsed += time.perf_counter() - t0
        rays += r
        rows_done += len(rows)
        chunk = min(chunk * 2, 4 * threads)
    return {"value": round(rays / elapsed / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{rows_done} of {h} rows x {w} px x {spp_s} spp of the same frame "
                      f"({rays} rays in {elapsed:.1f} s, oracle/rtw_oracle.c, {threads} threads, "
                      f"CPU {cpu_model()})"}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="jumpy-1080p", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override spp (changes the workload!)")
    ap.add_argument("--launches", type=int, default=0, help="kernel launches per frame (0 = auto)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default="", help="PMC HBM bytes per launch (from profiles/)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = CPU rehearsal of the N>1 path on one GPU")
    ap.add_argument("--check-image", action="store_true",
                    help="rank 0 checks the gathered frame bit-for-bit against a single-device render")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dev_id = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_id)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_id}"))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    rtw = _load("rtw_amd", PKG / "__init__.py", PKG)

    scene_name, w, h, spp, cfg_text = CONFIGS[args.config]
    if args.spp:
        spp = args.spp
    scene = rtw.Scene()
    cam, bg = scene.preset(scene_name, rtw.camera_aspect(w, h), seed=SCENE_SEED)
    scene.commit(device=dev)
    rt = rtw.Raytracer(scene, cam, bg, w, h, spp, seed=RENDER_SEED)

    # tiles of this rank (round-robin interleave balances sky rows against ground rows)
    nt = rtw.n_tiles(w, h)
    per_rank = (nt + world - 1) // world
    ids = torch.arange(rank, nt, world, dtype=torch.int32, device=dev)
    n_mine = int(ids.numel())
    packed = torch.zeros((per_rank, 64, 3), dtype=torch.float32, device=dev)
    gathered = torch.zeros((world * per_rank, 64, 3), dtype=torch.float32, device=dev) if world > 1 else None
    if world > 1:  # rank-major tile ids of the gathered buffer, padded with nt (= skipped)
        pad = [list(range(r, nt, world)) + [nt] * (per_rank - len(range(r, nt, world))) for r in range(world)]
        all_ids = torch.tensor(np.array(pad, np.int32).reshape(-1), dtype=torch.int32, device=dev)
    else:
        all_ids = ids
    image = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
    host_image = torch.empty((h, w, 3), dtype=torch.float32, pin_memory=True) if rank == 0 else None
    stream = torch.cuda.current_stream()

    launches = args.launches or 1  # persistent path kernel: one launch drains the whole frame
    bounds = np.linspace(0, n_mine, launches + 1).astype(int)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]

    def render_frame(record: bool):
        for k in range(launches):
            a, b = int(bounds[k]), int(bounds[k + 1])
            if record:
                ev[k][0].record(stream)
            rt.render_device(packed[a:].data_ptr(), dev, ids[a:].data_ptr(), b - a, stream.cuda_stream)
            if record:
                ev[k][1].record(stream)

    def frame_end():
        if world > 1 and args.backend == "gloo":  # CPU rehearsal: gather through host memory
            g = torch.zeros(gathered.shape, dtype=torch.float32)
            dist.all_gather_into_tensor(g, packed.cpu())
            gathered.copy_(g)
            if rank == 0:
                rtw.unpack_tiles_device(w, h, all_ids.data_ptr(), world * per_rank, gathered.data_ptr(),
                                        image.data_ptr(), dev, stream.cuda_stream)
        elif world > 1:
            dist.all_gather_into_tensor(gathered, packed)
            if rank == 0:
                rtw.unpack_tiles_device(w, h, all_ids.data_ptr(), world * per_rank, gathered.data_ptr(),
                                        image.data_ptr(), dev, stream.cuda_stream)
        else:
            rtw.unpack_tiles_device(w, h, ids.data_ptr(), n_mine, packed.data_ptr(), image.data_ptr(), dev,
                                    stream.cuda_stream)
        if rank == 0:
            host_image.copy_(image, non_blocking=True)

    # exact ray count + traversal counters of this rank's share (untimed, same seed => same work)
    st = rt.render_device(packed.data_ptr(), dev, ids.data_ptr(), n_mine, stream.cuda_stream,
                          flags=rtw.FLAG_COUNT_TRAVERSAL, want_stats=True)
    counts = torch.tensor([st["rays"], st["node_visits"]] + st["prim_tests_by_type"], dtype=torch.float64,
                          device=dev)
    if world > 1:
        dist.all_reduce(counts)
    counts = counts.cpu().numpy()
    frame_rays = int(counts[0])

    for _ in range(args.warmup):
        render_frame(False)
        frame_end()
    if args.check_image:  # the gathered frame must equal a single-device render, bit for bit
        render_frame(False)
        frame_end()
        torch.cuda.synchronize()
        if rank == 0:
            ref = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
            rt.render_device(ref.data_ptr(), dev, 0, 0, stream.cuda_stream)
            torch.cuda.synchronize()
            same = bool(torch.equal(ref.view(torch.int32), image.view(torch.int32)))
            print(json.dumps({"check_image": same, "world": world}), flush=True)
            if not same:
                raise SystemExit("gathered frame differs from the single-device render")
    torch.cuda.synchronize()
    scene.path_kernel_times(dev)  # forget the untimed launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        render_frame(True)
        frame_end()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    call_ms = float(sum(ev[k][0].elapsed_time(ev[k][1]) for k in range(launches)))  # last step: path + reduce
    # path_kernel alone: the library's HIP events around each launch on this stream, all K steps
    # (a render call splits a frame larger than MAX_PASS_PATHS into several passes, one launch each)
    pk = scene.path_kernel_times(dev)  # the last min(64, K * launches * passes) launches
    if not pk or len(pk) >= 64 or len(pk) % (args.steps * launches):
        raise SystemExit(f"path-kernel timings: got {len(pk)} for {args.steps} steps x {launches} calls "
                         "(ring of 64 overflowed or launches missing; lower --steps)")
    passes = len(pk) // (args.steps * launches)
    frame_kernel_ms = float(sum(pk)) / args.steps

    value = frame_rays * args.steps / dt / 1e6
    # roofline of the render kernel (this rank): algorithmic bytes per launch / avg launch time
    rays_r = counts[0]
    nodes_r = counts[1]
    prim_bytes = float(np.dot(counts[2:8], PRIM_B))
    alg_bytes_frame = RAY_STATE_B * rays_r + BOXES_PER_NODE * NODE_BOX_B * nodes_r + prim_bytes
    alg_bytes_rank = alg_bytes_frame / world
    achieved = alg_bytes_rank / (frame_kernel_ms * 1e-3) / 1e9
    # HBM bytes per launch from the committed rocprofv3 PMC summary of this config (FETCH_SIZE x2 +
    # WRITE_SIZE, separate passes; scripts/gpu_profile.sh + scripts/prof_summary.py), if any
    traffic, traffic_src = None, None
    tj = Path(args.traffic_json) if args.traffic_json else ROOT / "profiles" / f"pmc_{args.config}.json"
    if tj.exists() and not args.spp:
        d = json.loads(tj.read_text())
        if d.get("launches_per_frame", 1) == launches and d.get("world", 1) == world:
            traffic, traffic_src = d.get("hbm_bytes_per_launch"), str(tj.relative_to(ROOT))
    # what does bound it: SQ counters of the same config (scripts/gpu_counters.sh + valu_summary.py)
    issue = None
    vj = ROOT / "profiles" / f"valu_{args.config}.json"
    if vj.exists() and not args.spp:
        d = json.loads(vj.read_text())
        issue = {k: d.get(k) for k in ("valu_busy", "valu_lane_util", "wave_wait", "wave_issue", "l2_hit")}
        issue["source"] = str(vj.relative_to(ROOT))

    out = None
    if rank == 0:
        out = {
            "metric": "Mrays/sec at 1920x1080, 512 spp, 50 bounces; 1/2/4/8-GPU scaling",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene generator, scenes.rs restated; seed %d)" % SCENE_SEED,
            "config": {"workload": cfg_text, "backend": args.backend if world > 1 else None, "scene": scene_name, "width": w, "height": h, "spp": spp,
                       "max_depth": 50, "rays_per_frame": frame_rays, "paths_per_frame": w * h * spp,
                       "tiles": nt, "launches_per_frame": launches, "parallelism": f"tiles{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": traffic_src, "issue_counters": issue, "kernel": "path_kernel",
                         "kernel_ms_per_frame": round(frame_kernel_ms, 3),
                         "kernel_launches_per_frame": launches * passes,
                         "alg_bytes_per_launch": round(alg_bytes_rank / (launches * passes)),
                         "render_call_ms_last_frame": round(call_ms, 3),
                         "alg_bytes_per_ray": round(alg_bytes_frame / max(1, frame_rays), 2),
                         "node_fetches_per_ray": round(nodes_r / max(1, rays_r), 3),
                         "prim_tests_per_ray": round(float(counts[2:8].sum()) / max(1, rays_r), 3),
                         "simd_util_rank0": {k: (round(v, 3) if v else v) for k, v in st["simd_util"].items()},
                         "phase_share_rank0": {k: (round(v, 3) if v else v) for k, v in st["phase_share"].items()}},
            "paths_per_sec": round(w * h * spp * args.steps / dt, 1),
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(rtw, scene, cam, bg, w, h, spp, args.cpu_budget, threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
