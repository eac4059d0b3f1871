"""north_star's parity criterion on the benchmarked frames themselves, at their full spp.

Two phases, so the hours of CPU oracle work cost no GPU time:
  --phase gpu     (on the GPU box)  renders each BASELINE GPU config's frame exactly as bench.py does (scene seed 42,
                  render seed 2024, full resolution and spp; rtw_render: the reference's Vec<Pixel> order) and saves
                  the sums with the frame's exact ray count.  monument-4k's 99.5 MB frame is saved as every k-th
                  8-row band (and those bands are also rendered alone, through tile ids, for their own ray count;
                  their pixels must equal the whole frame's).
  --phase oracle  (anywhere, no GPU) runs oracle/rtw_oracle.c over the same pixels at the same spp and writes the
                  comparison: mismatching pixels / components bit for bit, RMSE and max |diff| of sum/spp (north_star:
                  RMSE < 1e-4), the ray-count delta, and the RMSE against the literal recursive association (lib.rs:
                  109-116, RECURSIVE) over two bands from the middle of the frame.
The oracle evaluates jumpy-balls and cornell-box as the reference does, flat lists (hittable/mod.rs:57-69; AS_LIST =
the GPU's set semantics, the bit-exact target).  The meshes sit in a BvhNode (scenes.rs:719-771): the flat list over
5,804 / 7,798 triangles runs ~0.02-0.03 Mrays/s per 8 cores, so their frames go through the reference's own BvhNode
tree and traversal (REFERENCE, bvh.rs:19-120, which may break exact t-ties between triangles by tree position and
cull a hit by slab rounding: DESIGN.md §2's documented deviations), and a few rows each through the flat list too.

    python scripts/fullspp_parity.py --phase gpu --dir gpurun_out/fullspp
    python scripts/fullspp_parity.py --phase oracle --dir gpurun_out/fullspp --out profiles/r06/fullspp_parity.json
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]
import importlib  # noqa: E402

from bench import CONFIGS, RENDER_SEED, SCENE_SEED  # noqa: E402

MODE = {"jumpy-1080p": "AS_LIST", "cornell-800": "AS_LIST", "cow-1080p": "REFERENCE", "monument-4k": "REFERENCE"}
BAND_STRIDE = {"monument-4k": 3}  # saved as every k-th band (gpurun_out carries <= 64 MiB per call)
FLAT_ROWS = {"cow-1080p": [540, 700], "monument-4k": [1080]}  # rows also checked against the flat list
REC_BANDS = 2


def _scene(rtw, cfg):
    name, w, h, spp, _ = CONFIGS[cfg]
    s = rtw.Scene()
    cam, bg = s.preset(name, rtw.camera_aspect(w, h), seed=SCENE_SEED)
    return s, cam, bg, name, w, h, spp


def gpu_phase(cfgs, d: Path) -> None:
    import torch
    rtw = importlib.import_module("raytracer-weekend_amd")
    d.mkdir(parents=True, exist_ok=True)
    for cfg in cfgs:
        s, cam, bg, name, w, h, spp = _scene(rtw, cfg)
        s.commit(device=0)
        rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=RENDER_SEED)
        t0 = time.time()
        frame, st = rt.render()
        meta = {"config": cfg, "w": w, "h": h, "spp": spp, "frame_rays_gpu": int(st["rays"]), "lib_sha": rtw.lib_sha(),
                "gpu_s": round(time.time() - t0, 2)}
        k = BAND_STRIDE.get(cfg, 1)
        if k > 1:
            tx, ty = (w + 7) // 8, (h + 7) // 8
            bands = list(range(0, ty, k))
            rows = np.concatenate([np.arange(8 * b, min(h, 8 * b + 8)) for b in bands])
            ids = np.concatenate([np.arange(b * tx, (b + 1) * tx) for b in bands]).astype(np.int32)
            d_ids = torch.tensor(ids, device="cuda:0")
            packed = torch.zeros((len(ids), 64, 3), dtype=torch.float32, device="cuda:0")
            sb = rt.render_device(packed.data_ptr(), 0, d_ids.data_ptr(), len(ids),
                                  torch.cuda.current_stream().cuda_stream, want_stats=True)
            g = packed.cpu().numpy()
            band_px = np.zeros_like(frame)
            for q, b in enumerate(bands):
                blk = g[q * tx:(q + 1) * tx].reshape(tx, 8, 8, 3).transpose(1, 0, 2, 3).reshape(8, tx * 8, 3)
                r0, r1 = 8 * b, min(h, 8 * b + 8)
                band_px[r0:r1] = blk[:r1 - r0, :w]
            meta.update({"rows": rows.tolist(), "sample_rays_gpu": int(sb["rays"]),
                         "bands_equal_whole_frame": bool(np.array_equal(band_px[rows].view(np.uint32),
                                                                        frame[rows].view(np.uint32)))})
            frame = frame[rows]
        meta["frame_sha256"] = hashlib.sha256(np.ascontiguousarray(frame).tobytes()).hexdigest()
        np.save(d / f"{cfg}_gpu.npy", frame)
        (d / f"{cfg}_meta.json").write_text(json.dumps(meta))
        print(json.dumps(meta)[:300], flush=True)


def recursive_check(o, orc, ocam, bg, w, h, spp, mode, g, rows, threads) -> dict:
    """The frame's GPU sums against the literal recursion's association (emitted + a0 * (a1 * (...)), lib.rs:109-116)
    over two bands from the middle of the frame (the top rows are often sky): rounding differences only."""
    mid = (len(rows) // 2) // 8 * 8
    rr = rows[mid:mid + 8 * REC_BANDS]
    t0 = time.time()
    rec, _ = o.render(ocam, bg, w, h, spp, seed=RENDER_SEED, threads=threads, integrator=orc.RECURSIVE,
                      rows=[h - 1 - int(x) for x in rr], bvh_mode=mode)
    ga, ra = g[mid:mid + len(rr)].astype(np.float64) / spp, rec[rr].astype(np.float64) / spp
    return {"rows": [int(rr[0]), int(rr[-1])], "rmse_mean": float(np.sqrt(np.mean((ga - ra) ** 2))),
            "max_abs_mean": float(np.abs(ga - ra).max()),
            "max_rel_component": float(np.max(np.abs(ga - ra) / np.maximum(np.abs(ra), 1e-30))),
            "oracle_s": round(time.time() - t0, 1)}


def oracle_phase(cfgs, d: Path, out: Path, threads: int, recursive_only: bool = False) -> None:
    rtw = importlib.import_module("raytracer-weekend_amd")
    import oracle as orc
    res = {"seeds": {"scene": SCENE_SEED, "render": RENDER_SEED}, "threads": threads, "configs": []}
    if out.exists():
        res = json.loads(out.read_text())
        res["configs"] = [c for c in res["configs"] if c["config"] not in cfgs]
    for cfg in cfgs:
        meta = json.loads((d / f"{cfg}_meta.json").read_text())
        g = np.load(d / f"{cfg}_gpu.npy")
        s, cam, bg, name, w, h, spp = _scene(rtw, cfg)
        o = orc.OracleScene(s.dump(), s.images())
        ocam = orc.camera_from_fields(cam.as_dict())
        rows = np.array(meta.get("rows", range(h)))
        mode = getattr(orc, "BVH_" + MODE[cfg])
        if recursive_only:  # refresh only the recursive-association entry of an existing result
            old = json.loads(out.read_text())
            for c in old["configs"]:
                if c["config"] == cfg:
                    c["recursive"] = recursive_check(o, orc, ocam, bg, w, h, spp, mode, g, rows, threads)
                    print(json.dumps(c["recursive"]), flush=True)
            out.write_text(json.dumps(old, indent=1) + "\n")
            continue
        t0 = time.time()
        ref, rays = o.render(ocam, bg, w, h, spp, seed=RENDER_SEED, threads=threads, rows=[h - 1 - int(r) for r in rows],
                             bvh_mode=mode)
        t_orc = time.time() - t0
        ref = ref[rows]
        bad = g.view(np.uint32) != ref.view(np.uint32)
        gf, rf = g.astype(np.float64) / spp, ref.astype(np.float64) / spp
        gpu_rays = meta.get("sample_rays_gpu", meta["frame_rays_gpu"])
        r = {"config": cfg, "scene": name, "w": w, "h": h, "spp": spp, "lib_sha": meta["lib_sha"],
             "pixels": f"{len(rows)} of {h} rows x {w} px ({'whole frame' if len(rows) == h else 'every %dth 8-row band' % BAND_STRIDE[cfg]}) x {spp} spp",
             "oracle": "ITERATIVE, " + ("flat list (the bit-exact target)" if MODE[cfg] == "AS_LIST" else
                                        "the reference's BvhNode tree and traversal (bvh.rs:19-120)"),
             "rays_gpu": gpu_rays, "rays_oracle": int(rays), "ray_delta": int(gpu_rays) - int(rays),
             "mismatching_pixels": int(bad.any(axis=2).sum()), "mismatching_components": int(bad.sum()),
             "rmse_mean": float(np.sqrt(np.mean((gf - rf) ** 2))), "max_abs_mean": float(np.abs(gf - rf).max()),
             "mismatch_first": np.argwhere(bad.any(axis=2))[:8].tolist(), "oracle_s": round(t_orc, 1)}
        r["gpu_frame_sha256"] = hashlib.sha256(np.ascontiguousarray(g).tobytes()).hexdigest()
        if "bands_equal_whole_frame" in meta:
            r["bands_equal_whole_frame"] = meta["bands_equal_whole_frame"]
        if cfg in FLAT_ROWS:  # a few rows against the flat list as well, bit for bit
            fr = FLAT_ROWS[cfg]
            t0 = time.time()
            fl, _ = o.render(ocam, bg, w, h, spp, seed=RENDER_SEED, threads=threads, rows=[h - 1 - x for x in fr])
            idx = [int(np.nonzero(rows == x)[0][0]) for x in fr]
            b1 = g[idx].view(np.uint32) != fl[fr].view(np.uint32)
            r["flat_list_rows"] = {"rows": fr, "pixels": len(fr) * w, "mismatching_pixels": int(b1.any(axis=2).sum()),
                                   "oracle_s": round(time.time() - t0, 1)}
        if MODE[cfg] == "REFERENCE" and bad.any():
            # the pixels where the GPU and the reference's BvhNode tree differ, through the flat list (the GPU's set
            # semantics): are they the tree's documented deviation (ties by tree position, slab-rounding culls)?
            q = np.argwhere(bad.any(axis=2))
            px = [(h - 1 - int(rows[a]), int(i)) for a, i in q]
            t0 = time.time()
            fl, _ = o.render_pixels(ocam, bg, w, h, spp, px, seed=RENDER_SEED, threads=threads)
            b2 = g[q[:, 0], q[:, 1]].view(np.uint32) != fl.view(np.uint32)
            r["differing_pixels_vs_flat_list"] = {"pixels": len(px), "mismatching_pixels": int(b2.any(axis=1).sum()),
                                                  "oracle_s": round(time.time() - t0, 1)}
        r["recursive"] = recursive_check(o, orc, ocam, bg, w, h, spp, mode, g, rows, threads)
        print(json.dumps(r), flush=True)
        res["configs"].append(r)
        out.parent.mkdir(parents=True, exist_ok=True)
        out.write_text(json.dumps(res, indent=1) + "\n")


def verify_phase(cfgs, out: Path) -> int:
    """On the GPU box: re-render the configs with the current library and compare each frame's hash with the one the
    oracle phase validated (profiles/r06/fullspp_parity.json), so a later build inherits the whole-frame result only
    if it renders the same bits."""
    res = json.loads(out.read_text())
    known = {c["config"]: c for c in res["configs"]}
    with tempfile.TemporaryDirectory() as t:
        gpu_phase(cfgs, Path(t))
        bad = 0
        for cfg in cfgs:
            meta = json.loads((Path(t) / f"{cfg}_meta.json").read_text())
            same = known[cfg]["gpu_frame_sha256"] == meta["frame_sha256"] and \
                known[cfg]["rays_gpu"] == meta.get("sample_rays_gpu", meta["frame_rays_gpu"])
            print(json.dumps({"config": cfg, "lib_sha": meta["lib_sha"], "validated_lib_sha": known[cfg]["lib_sha"],
                              "same_frame_and_rays": same}), flush=True)
            bad += not same
    return 1 if bad else 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase", choices=["gpu", "oracle", "verify"], required=True)
    ap.add_argument("--configs", default="jumpy-1080p,cornell-800,cow-1080p,monument-4k")
    ap.add_argument("--dir", default="gpurun_out/fullspp")
    ap.add_argument("--out", default="profiles/r06/fullspp_parity.json")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--recursive-only", action="store_true", help="refresh only the RECURSIVE comparison")
    a = ap.parse_args()
    cfgs = a.configs.split(",")
    if a.phase == "verify":
        return verify_phase(cfgs, Path(a.out))
    if a.phase == "gpu":
        gpu_phase(cfgs, Path(a.dir))
    else:
        oracle_phase(cfgs, Path(a.dir), Path(a.out), a.threads, a.recursive_only)
    return 0


if __name__ == "__main__":
    sys.exit(main())
