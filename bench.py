#!/usr/bin/env python3
"""bench.py — Mrays/s of the MI355X render core on BASELINE.json's headline workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config jumpy-1080p]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N` always means N GPUs.  Under a launcher (WORLD_SIZE set) it must equal WORLD_SIZE: one
process per GPU, one RCCL all-gather.  Without a launcher and N > 1, this one process drives the N GPUs
through the C-ABI's rtw_render_multi (one RCCL send/recv gather to device 0); with fewer than N visible
GPUs it exits non-zero before rendering anything.  `--multi-device N` is the same single-process path
(also at N = 1).  The printed n_gpus is checked against N before the line is printed.

A step = one full frame of the configured workload (default: BASELINE.json configs[1],
RTOW final random-spheres "jumpy-balls", 1920x1080, 512 spp, 50 bounces) rendered by the
hot path, with the scene already resident in HBM.  On one GPU the frame renders straight into
the device image (rtw_render_device without tile ids, rtw_render's path).  On N GPUs the frame's
8x8 tiles are dealt round-robin to the N ranks (one process per GPU, rtw_tile_partition); each
rank renders its tiles with rtw_render_device, then one RCCL all-gather over xGMI brings every
rank's packed tiles to all ranks and rank 0 unpacks the framebuffer.  The step ends with the frame
in rank 0's HBM (the C-ABI's rtw_render_device output); the rate with rank 0 also copying it to pinned
host memory in every step (rtw_render's host-buffer boundary, over PCIe) is timed separately and printed
as `pcie_inclusive` -- never `value` (the single-process --multi-device path returns a host frame from
rtw_render_multi, so there the two are the same).  Total work
is fixed as N grows ("scaling": "strong").  value = rays of the frame (world.hit queries,
lib.rs:102, counted exactly by the kernel) / max-over-ranks step time.

`roofline`: the path kernel is bound by VALU issue (SQ counters), so the
roofline is FP32 VALU: algorithmic flops per launch (SURVEY.md §8d / BASELINE.md: 21 per box
tested, 23 per sphere test (+12 moving), 6 per rect, 51 per triangle, 70 per scattering segment,
64 per path; DESIGN.md §5 itemises them) / the kernel's average HIP-event duration, vs the 157.3 TFLOP/s FP32 vector
peak, and as a second figure (`exact_f32_issue`) vs the 78.6 T lane-op/s a bit-exact kernel (no FMA contraction, no
packed math: one lane-op per flop at best) can issue.  Reported beside them: the measured HBM fraction (rocprofv3 PMC bytes per launch / duration /
8 TB/s), the SQ-counter VALU lane-capacity figure (VALU busy x lane utilisation) and the
cache-level algorithmic bytes.  scripts/roofline.py recomputes all of them from profiles/.

`cpu_baseline` is the oracle (the reference algorithm restated in C, flat-list closest hit,
recursive sample_ray; -O3) on the host CPUs this process may use (the cgroup CPU quota when there
is one, else every logical CPU; `cores` states that number), best of 3 over a bounded row sample
of the same frame, rank 0 at N=1 only.

N > 1 prints, beside `value`, the per-rank path-kernel ms, the all-gather ms and the max/min
imbalance across ranks (`multi_gpu`), so a scaling run separates load imbalance from gather cost.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import math
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
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (spec): v_fma_f32 at 32 lanes/clk/SIMD, 2 flops each
# The issue ceiling of an exact-f32 kernel: compiled -ffp-contract=off and without packed math, every
# algorithmic flop is at least one non-FMA, non-packed VALU lane-op, and a SIMD-32 issues at most 32 lane-ops per
# clock (MI355X_MICROARCH.md: a wave64 VALU instruction takes 2 cycles): 256 CUs x 4 SIMDs x 32 x 2.4 GHz
EXACT_F32_ISSUE_T = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64 T lane-op/s
# FP32 flop model (BASELINE.md roofline; DESIGN.md §5 derives each constant)
FLOP_BOX = 21              # aabb.rs:23-48: per axis 1 div + 2 sub + 2 mul + min + max
FLOP_PRIM = [23, 35, 6, 6, 6, 51]  # sphere (spherical.rs:26-44), moving (+12, :117-123), rect xy/xz/yz, triangle
FLOP_SCATTER = 70          # hit record + Lambertian scatter + throughput per scattering segment
FLOP_PATH = 64             # pixel u, v + Camera::get_ray + the terminal T * colour, per path
# cache-level algorithmic bytes (the round-1 figure; operands come from L1/L2, not HBM)
RAY_STATE_B = 64
NODE_BOX_B = 32
PRIM_B = [16, 36, 20, 20, 20, 36]


def _load(name, path, pkg_dir=None):
    if name in sys.modules:
        return sys.modules[name]
    kw = {"submodule_search_locations": [str(pkg_dir)]} if pkg_dir else {}
    spec = importlib.util.spec_from_file_location(name, path, **kw)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup (cpu.max), None if unlimited / unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scene, cam, bg, w, h, spp, budget_s: float) -> dict:
    """The oracle (reference algorithm: flat-list closest hit / the reference BvhNode tree,
    recursive sample_ray) on every host core, best of 3 over the same evenly strided row sample
    of the frame (at min(spp, 8) samples per pixel)."""
    orc = _load("rtw_oracle_py", ROOT / "oracle" / "oracle.py")
    o = orc.OracleScene(scene.dump(), scene.images())
    ocam = orc.camera_from_fields(cam.as_dict())
    nproc = os.cpu_count() or 1
    quota = cpu_quota()
    # one thread per CPU the cgroup grants (a 16-CPU quota on a 256-thread EPYC: 16 threads), the
    # Rayon pool's size on that box (lib.rs:60-67 runs over the cores it has); oracle_render caps at 256
    threads = max(1, min(256, nproc, math.ceil(quota) if quota else nproc))
    spp_s = max(1, min(spp, 8))
    order = list(range(0, h, 37)) + [j for j in range(h) if j % 37]  # strided first

    def run(rows):
        t0 = time.perf_counter()
        _, r = o.render(ocam, bg, w, h, spp_s, seed=RENDER_SEED, integrator=orc.RECURSIVE,
                        bvh_mode=orc.BVH_REFERENCE, threads=threads, rows=rows)
        return time.perf_counter() - t0, r

    probe = order[:max(1, threads)]
    dt, _ = run(probe)
    n = int(min(len(order), max(len(probe), len(probe) * (budget_s / 3.0) / max(dt, 1e-3))))
    rows = order[:n]
    times, rays = [], 0
    for _ in range(3):
        dt, rays = run(rows)
        times.append(dt)
    best = min(times)
    where = (f"cgroup quota of {quota:g} CPUs on a {nproc}-thread {cpu_model()}" if quota
             else f"all {nproc} logical CPUs of a {cpu_model()}")
    return {"value": round(rays / best / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "cpu_quota_cores": quota, "nproc": nproc,
            "label": f"CPU restatement, {threads} cores ({where}); baseline only",
            "sample": f"{len(rows)} of {h} rows x {w} px x {spp_s} spp of the same frame, best of 3 "
                      f"({rays} rays in {best:.2f} s; runs {', '.join(f'{t:.2f}' for t in times)} s), "
                      f"oracle/rtw_oracle.c -O3, {threads} threads, CPU {cpu_model()}"}


def flops_model(counts: dict) -> float:
    """Algorithmic FP32 flops of the counted work."""
    # every path's last segment ends it (miss, light, absorption, depth); the others scatter
    return (FLOP_BOX * counts["boxes"] + float(np.dot(counts["prims"], FLOP_PRIM))
            + FLOP_SCATTER * max(0.0, counts["rays"] - counts["paths"]) + FLOP_PATH * counts["paths"])


def roofline(counts: dict, kernel_ms_per_launch: float, launches: int, world: int, traffic, issue) -> dict:
    """The path kernel's roofline figures for one launch (this rank's share of the frame)."""
    flops = flops_model(counts) / world / launches
    tflops = flops / (kernel_ms_per_launch * 1e-3) / 1e12
    alg_bytes = (RAY_STATE_B * counts["rays"] + NODE_BOX_B * counts["boxes"]
                 + float(np.dot(counts["prims"], PRIM_B))) / world / launches
    out = {"bound": "valu", "achieved": round(tflops, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": round(tflops / FP32_PEAK_TFLOPS, 5), "traffic": traffic,
           "flops_per_launch": round(flops), "kernel_ms_per_launch": round(kernel_ms_per_launch, 3),
           "flops_per_ray": round(flops_model(counts) / max(1, counts["rays"]), 1),
           "exact_f32_issue": {"achieved": round(tflops, 3), "peak": round(EXACT_F32_ISSUE_T, 2), "unit": "T lane-op/s",
                               "frac": round(tflops / EXACT_F32_ISSUE_T, 5),
                               "note": "second figure: the algorithmic flops against the non-FMA, non-packed VALU lane "
                                       "rate, the most a bit-exact (-ffp-contract=off, no packed math) kernel can issue "
                                       "them at; frac above stays against the 157.3 TFLOP/s spec peak"},
           "hbm": None, "valu_lane": None, "vmem_units": None,
           "cache_level": {"alg_bytes_per_launch": round(alg_bytes),
                           "GBps": round(alg_bytes / (kernel_ms_per_launch * 1e-3) / 1e9, 1),
                           "note": "node/prim operands are L1/L2 hits; not an HBM figure"}}
    if traffic:
        gbs = traffic / (kernel_ms_per_launch * 1e-3) / 1e9
        out["hbm"] = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(gbs / HBM_PEAK_GBS, 5), "bytes_per_launch": traffic}
    if issue and issue.get("valu_busy") and issue.get("valu_lane_util"):
        out["valu_lane"] = {"valu_busy": issue["valu_busy"], "lane_util": issue["valu_lane_util"],
                            "frac": round(issue["valu_busy"] * issue["valu_lane_util"], 4),
                            "source": issue.get("source")}
    if issue and issue.get("ta_busy"):  # vector-memory units (busy, but not the one binding limit)
        out["vmem_units"] = {"ta_busy": issue["ta_busy"], "td_busy": issue.get("td_busy"), "source": issue.get("source")}
    if issue and issue.get("lds_active") is not None:  # LDS array (node / sphere tables of the LDS-node kernels)
        out["lds"] = {"active": issue["lds_active"], "conflict_share": issue.get("lds_conflict_share"),
                      "source": issue.get("source")}
    return out


def resolve_gpus(args, world: int, visible: int) -> int:
    """How many GPUs this process drives through rtw_render_multi (0 = the one-GPU / one-rank path).
    Raises SystemExit (non-zero) instead of ever measuring fewer GPUs than --gpus asks for."""
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: at least 1")
    if args.multi_device and args.gpus not in (None, args.multi_device):
        raise SystemExit(f"--gpus {args.gpus} and --multi-device {args.multi_device} disagree")
    if world > 1:  # one process per GPU under torch.distributed.run
        if args.multi_device:
            raise SystemExit("--multi-device is the single-process path: do not launch it with WORLD_SIZE > 1")
        if args.gpus not in (None, world):
            raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        args.gpus = world
        return 0
    n = args.multi_device or (args.gpus if args.gpus and args.gpus > 1 else 0)
    if n and visible < n:
        raise SystemExit(f"--gpus {n} without a launcher drives {n} GPUs from this process "
                         f"(rtw_render_multi), but only {visible} are visible: nothing measured")
    args.gpus = max(1, n)
    return n


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs to measure (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="jumpy-1080p", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override spp (changes the workload!)")
    ap.add_argument("--launches", type=int, default=0, help="kernel launches per frame (0 = auto)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work (3 runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default="", help="PMC HBM bytes per launch (from profiles/)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = CPU rehearsal of the N>1 path on one GPU")
    ap.add_argument("--check-image", action="store_true",
                    help="rank 0 checks the gathered frame bit-for-bit against a single-device render")
    ap.add_argument("--multi-device", type=int, default=0,
                    help="N > 0: one process renders each frame on N GPUs through rtw_render_multi "
                         "(C-ABI, RCCL send/recv gather to device 0, frame copied to the host)")
    ap.add_argument("--diag-alias", action="store_true",
                    help="diagnostic (never a measurement): --multi-device N on ONE physical GPU, the scene's N "
                         "devices being logical ones (rtw_diag_alias_devices); needs RTW_RCCL_LIB pointing at an "
                         "RCCL stand-in that allows it (tests/loopback_rccl), as real RCCL refuses shared-GPU cliques")
    args = ap.parse_args()
    if args.diag_alias and not (args.multi_device > 1 and os.environ.get("RTW_RCCL_LIB")):
        raise SystemExit("--diag-alias needs --multi-device N > 1 and RTW_RCCL_LIB set (tests/loopback_rccl)")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --diag-alias: the N devices are logical ones on device 0 (one visible GPU suffices)
    multi = resolve_gpus(args, world, args.multi_device if args.diag_alias else torch.cuda.device_count())
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
    if args.diag_alias:
        scene.diag_alias_devices(multi)
    scene.commit(device=-1 if multi else dev)
    rt = rtw.Raytracer(scene, cam, bg, w, h, spp, seed=RENDER_SEED)

    # tiles of this rank (round-robin interleave balances sky rows against ground rows)
    nt = rtw.n_tiles(w, h)
    pad_ids, n_mine = rtw.tile_partition(w, h, world, rank)
    per_rank = len(pad_ids)
    ids = torch.tensor(pad_ids.astype(np.int32), dtype=torch.int32, device=dev)
    packed = torch.zeros((per_rank, 64, 3), dtype=torch.float32, device=dev)
    gathered = torch.zeros((world * per_rank, 64, 3), dtype=torch.float32, device=dev) if world > 1 else None
    if world > 1:  # rank-major tile ids of the gathered buffer, padded with nt (= skipped)
        lay = np.concatenate([rtw.tile_partition(w, h, world, r)[0] for r in range(world)]).astype(np.int32)
        all_ids = torch.tensor(lay, dtype=torch.int32, device=dev)
    else:
        all_ids = ids
    image = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
    host_image = torch.empty((h, w, 3), dtype=torch.float32, pin_memory=True) if rank == 0 else None
    stream = torch.cuda.current_stream()

    launches = args.launches or 1  # persistent path kernel: one launch drains the whole frame
    bounds = np.linspace(0, n_mine, launches + 1).astype(int)

    def render_frame():
        if multi:
            rt.render_multi(multi)  # blocking: renders, gathers over RCCL, copies the frame to the host
            if timing_multi is not None:
                timing_multi.append(scene.multi_times())
            return
        if world == 1 and launches == 1:  # one GPU: the whole frame straight into the image (rtw_render's path)
            rt.render_device(image.data_ptr(), dev, 0, 0, stream.cuda_stream)
            return
        if launches == 1:  # this rank's tiles rank, rank + world, ... (the kernel computes them: no id table)
            rt.render_device_strided(packed.data_ptr(), dev, rank, world, n_mine, stream.cuda_stream)
            return
        for k in range(launches):
            a, b = int(bounds[k]), int(bounds[k + 1])
            rt.render_device(packed[a:].data_ptr(), dev, ids[a:].data_ptr(), b - a, stream.cuda_stream)

    def frame_end(to_host):
        if multi:
            return
        if world > 1 and args.backend == "gloo":  # CPU rehearsal: gather through host memory
            if gev is not None:
                gev[0].record(stream)
            g = torch.zeros(gathered.shape, dtype=torch.float32)
            dist.all_gather_into_tensor(g, packed.cpu())
            gathered.copy_(g)
            if gev is not None:
                gev[1].record(stream)
                gather_ev.append(gev)
            if rank == 0:
                rtw.unpack_tiles_device(w, h, all_ids.data_ptr(), world * per_rank, gathered.data_ptr(),
                                        image.data_ptr(), dev, stream.cuda_stream)
        elif world > 1:
            if gev is not None:
                gev[0].record(stream)
            dist.all_gather_into_tensor(gathered, packed)
            if gev is not None:  # on torch's stream after the collective: includes waiting for the slowest rank
                gev[1].record(stream)
                gather_ev.append(gev)
            if rank == 0:
                rtw.unpack_tiles_device(w, h, all_ids.data_ptr(), world * per_rank, gathered.data_ptr(),
                                        image.data_ptr(), dev, stream.cuda_stream)
        elif launches > 1:
            rtw.unpack_tiles_device(w, h, ids.data_ptr(), n_mine, packed.data_ptr(), image.data_ptr(), dev,
                                    stream.cuda_stream)
        if rank == 0 and to_host:
            host_image.copy_(image, non_blocking=True)

    gev = None         # (start, end) events of the current step's all-gather (N > 1)
    gather_ev = []     # those of the timed steps
    timing_multi = None  # rtw_render_multi_times of the timed steps (single-process multi-device path)
    # exact ray count + traversal counters of this rank's share (untimed, same seed => same work)
    st = rt.render_device(packed.data_ptr(), dev, ids.data_ptr(), n_mine, stream.cuda_stream,
                          flags=rtw.FLAG_COUNT_TRAVERSAL, want_stats=True)
    counts = torch.tensor([st["rays"], st["node_visits"], st["boxes_tested"], n_mine * 64 * spp]
                          + st["prim_tests_by_type"], dtype=torch.float64, device=dev)
    rank_rays = [int(st["rays"])]
    if world > 1:
        rr = [torch.zeros_like(counts) for _ in range(world)]
        dist.all_gather(rr, counts)
        rank_rays = [int(x[0].item()) for x in rr]
        dist.all_reduce(counts)
    counts = counts.cpu().numpy()
    frame_rays = int(counts[0])
    cnt = {"rays": counts[0], "node4": counts[1], "boxes": counts[2], "paths": min(counts[3], w * h * spp),
           "prims": counts[4:10]}

    for _ in range(args.warmup):
        render_frame()
        frame_end(True)
    if args.check_image:  # the gathered frame must equal a single-device render, bit for bit
        render_frame()
        frame_end(False)
        torch.cuda.synchronize()
        if rank == 0:
            ref = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
            rt.render_device(ref.data_ptr(), dev, 0, 0, stream.cuda_stream)
            torch.cuda.synchronize()
            if multi:
                got, _ = rt.render_multi(multi)
                same = bool(np.array_equal(ref.cpu().numpy().view(np.uint32), got.view(np.uint32)))
            else:
                same = bool(torch.equal(ref.view(torch.int32), image.view(torch.int32)))
            print(json.dumps({"check_image": same, "world": world, "multi_device": multi}), flush=True)
            if not same:
                raise SystemExit("gathered frame differs from the single-device render")
    torch.cuda.synchronize()
    for d in (range(multi) if multi else [dev]):
        scene.path_kernel_times(d)  # forget the untimed launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if multi:
        timing_multi = []

    def timed(to_host, events):  # K steps between barriers + synchronize, max over ranks
        nonlocal gev
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            if world > 1 and events:
                gev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            render_frame()
            frame_end(to_host)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gev = None
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    dt = timed(False, True)
    # path_kernel alone: the library's HIP events around each launch on the launch stream, all K
    # steps (a render call splits a frame larger than 2^32 paths into several passes, one launch each)
    # every frame rendered so far is valid: no traversal guard tripped (raises otherwise)
    for d in (range(multi) if multi else [dev]):
        scene.render_status(d)
    # every device's launches, read once (a read also forgets them: rtw_path_kernel_times)
    pk_dev = {d: scene.path_kernel_times(d) for d in (range(multi) if multi else [dev])}
    pk = pk_dev[0 if multi else dev]
    if not pk or len(pk) >= 64 or len(pk) % (args.steps * launches):
        raise SystemExit(f"path-kernel timings: got {len(pk)} for {args.steps} steps x {launches} calls "
                         "(ring of 64 overflowed or launches missing; lower --steps)")
    passes = len(pk) // (args.steps * launches)
    frame_kernel_ms = float(sum(pk)) / args.steps
    # the same K steps with rank 0 copying the frame to pinned host memory in each (PCIe-inclusive; never `value`)
    dt_host = dt if multi else timed(True, False)
    for d in (range(multi) if multi else [dev]):
        scene.path_kernel_times(d)

    value = frame_rays * args.steps / dt / 1e6
    # HBM bytes per launch from the committed rocprofv3 PMC summary of this config (FETCH_SIZE x2 +
    # WRITE_SIZE, separate passes; scripts/gpu_r05_evidence.sh + scripts/summarize_round.py), if any --
    # attached only when it was measured on THIS library build (its lib_sha stamp), else null + the reason
    sha = rtw.lib_sha()
    evidence_notes = []

    def same_build(d, path):
        if d.get("lib_sha") == sha:
            return True
        evidence_notes.append(f"{path.relative_to(ROOT)} was measured on build {d.get('lib_sha') or 'unstamped'}, "
                              f"the timed library is {sha}: not attached")
        return False

    traffic, traffic_src = None, None
    tj = Path(args.traffic_json) if args.traffic_json else ROOT / "profiles" / f"pmc_{args.config}.json"
    if tj.exists() and not args.spp and not multi:
        d = json.loads(tj.read_text())
        if d.get("launches_per_frame", 1) == launches and d.get("world", 1) == world and same_build(d, tj):
            traffic, traffic_src = d.get("hbm_bytes_per_launch"), str(tj.relative_to(ROOT))
    # what bounds it: SQ counters of the same config and build (summarize_round.py)
    issue = None
    vj = ROOT / "profiles" / f"valu_{args.config}.json"
    if vj.exists() and not args.spp and not multi:
        d = json.loads(vj.read_text())
        if same_build(d, vj):
            issue = {k: d.get(k) for k in ("valu_busy", "valu_lane_util", "wave_wait", "wave_issue", "l2_hit",
                                            "ta_busy", "td_busy", "lds_active", "lds_conflict_share",
                                            "tcp_hit", "vmem_rd_per_ray")}
            issue["source"] = str(vj.relative_to(ROOT))
    multi_gpu = None
    if world > 1:  # per-rank kernel / gather time: imbalance vs gather cost (a scaling run's diagnosis)
        gms = sum(a.elapsed_time(b) for a, b in gather_ev) / len(gather_ev) if gather_ev else float("nan")
        mine_t = torch.tensor([frame_kernel_ms, gms], dtype=torch.float64, device=dev)
        allt = [torch.zeros_like(mine_t) for _ in range(world)]
        dist.all_gather(allt, mine_t)
        km = [round(float(x[0].item()), 3) for x in allt]
        gm = [round(float(x[1].item()), 3) for x in allt]
        multi_gpu = {"rank_kernel_ms_per_frame": km, "rank_gather_ms_per_frame": gm, "rank_rays_per_frame": rank_rays,
                     "kernel_imbalance_max_over_min": round(max(km) / min(km), 4) if min(km) > 0 else None,
                     "gather_ms_min_over_ranks": min(gm),
                     "note": "gather ms = all-gather on torch's stream, incl. waiting for the slowest rank; its "
                             "minimum over ranks (the slowest rank's) is the transfer cost"}
    if multi and timing_multi:  # the same diagnosis for the single-process N-GPU path (rtw_render_multi)
        dms = np.array([t[0] for t in timing_multi], dtype=np.float64)  # steps x devices
        gms_m = float(np.mean([t[1] for t in timing_multi]))
        dk = []  # path-kernel ms per frame of every device (the library's events on that device's stream)
        for d in range(multi):
            pkd = pk_dev[d]
            dk.append(round(float(sum(pkd)) / args.steps, 3) if pkd else None)
        km = [round(float(x), 3) for x in dms.mean(axis=0)]
        multi_gpu = {"device_kernel_ms_per_frame": dk, "device_render_ms_per_frame": km,
                     "gather_ms_per_frame": round(gms_m, 3),
                     "kernel_imbalance_max_over_min": round(max(km) / min(km), 4) if min(km) > 0 else None,
                     "note": "render ms = path kernel + in-order reduction per device (HIP events on its stream); "
                             "gather ms = device 0's stream from the end of its render to the last device's "
                             "tiles (RCCL send/recv group), so it includes waiting for the slowest device"}
    n_launch = launches * passes
    # per launch of this rank (multi-device: device 0's launches, its 1/N share of the frame)
    roof = roofline(cnt, frame_kernel_ms / n_launch, n_launch, multi or world, traffic, issue)

    out = None
    if rank == 0:
        n_dev = multi or world
        roof.update({"traffic_source": traffic_src, "issue_counters": issue, "lib_sha": sha,
                     "evidence_notes": evidence_notes or None, "kernel": "path_kernel",
                     "kernel_ms_per_frame": round(frame_kernel_ms, 3), "kernel_launches_per_frame": n_launch,
                     "node_fetches_per_ray": round(cnt["node4"] / max(1, cnt["rays"]), 3),
                     "boxes_per_ray": round(cnt["boxes"] / max(1, cnt["rays"]), 3),
                     "prim_tests_per_ray": round(float(cnt["prims"].sum()) / max(1, cnt["rays"]), 3),
                     "counts": {"rays": int(cnt["rays"]), "paths": int(cnt["paths"]), "node4": int(cnt["node4"]),
                                "boxes": int(cnt["boxes"]), "prims_by_type": [int(x) for x in cnt["prims"]]},
                     "simd_util_rank0": {k: (round(v, 3) if v else v) for k, v in st["simd_util"].items()},
                     "phase_share_rank0": {k: (round(v, 3) if v else v) for k, v in st["phase_share"].items()}})
        out = {
            "metric": "Mrays/sec at 1920x1080, 512 spp, 50 bounces; 1/2/4/8-GPU scaling",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n_dev,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene generator, scenes.rs restated; seed %d)" % SCENE_SEED,
            "config": {"workload": cfg_text, "backend": args.backend if world > 1 else ("rccl" if multi else None),
                       "diag_alias_devices": multi if args.diag_alias else None,
                       "scene": scene_name, "width": w, "height": h, "spp": spp, "max_depth": 50,
                       "rays_per_frame": frame_rays, "paths_per_frame": w * h * spp, "tiles": nt,
                       "launches_per_frame": launches,
                       "parallelism": f"tiles{n_dev}" + ("-single-process" if multi else "")},
            "roofline": roof,
            "paths_per_sec": round(w * h * spp * args.steps / dt, 1),
            "pcie_inclusive": {"value": round(frame_rays * args.steps / dt_host / 1e6, 2),
                               "ms_per_step": round(dt_host / args.steps * 1e3, 3),
                               "note": "the same K steps with rank 0 copying the frame (w x h x 3 f32) to pinned host "
                                       "memory in each: the rate through rtw_render's host-buffer boundary"},
        }
        if multi_gpu:
            out["multi_gpu"] = multi_gpu
        if out["n_gpus"] != args.gpus:  # never print an N = 1 line for an N-GPU request
            raise SystemExit(f"bench measured {out['n_gpus']} GPU(s) but --gpus {args.gpus} was requested")
        if n_dev == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, cam, bg, w, h, spp, args.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
