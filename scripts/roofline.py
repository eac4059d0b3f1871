"""Recompute the path kernel's roofline figures from the committed profiles.

    python scripts/roofline.py profiles/r02 [jumpy-1080p cornell-800 cow-1080p monument-4k]

Per config it reads
  <dir>/<cfg>/bench.json          the bench.py JSON line of that config (its traversal counts:
                                  rays, paths, boxes tested, primitive tests by type)
  <dir>/<cfg>/kernel_stats.csv    rocprofv3 --kernel-trace --stats of the same command
  profiles/pmc_<cfg>.json         HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, separate passes)
  profiles/valu_<cfg>.json        SQ counters (VALU busy, lane utilisation)
and prints, from the rocprof average duration of the path kernel:
  FP32-VALU frac  = algorithmic flops per launch (bench.flops_model: 21 / box tested, 23 / sphere,
                    35 / moving sphere, 6 / rect, 51 / triangle, 70 / scattering segment,
                    64 / path)
                    / avg duration / 157.3 TFLOP/s
  HBM frac        = PMC bytes per launch / avg duration / 8 TB/s
  VALU lane frac  = VALU busy x lane utilisation (share of the SIMDs' lane-cycles doing VALU work)
next to the frac bench.py measured live with HIP events.  The two durations must agree to a few %.
"""
import csv
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (flop model and peaks; bench imports torch only inside main())


def rocprof_avg_ms(path: Path) -> float:
    for r in csv.DictReader(open(path)):
        if "path_kernel<false" in r["Name"]:
            return float(r["AverageNs"]) / 1e6
    raise SystemExit(f"no path_kernel<false,...> row in {path}")


def main():
    d = Path(sys.argv[1])
    cfgs = sys.argv[2:] or ["jumpy-1080p", "cornell-800", "cow-1080p", "monument-4k"]
    rows = []
    for cfg in cfgs:
        bj = json.loads((d / cfg / "bench.json").read_text().strip().splitlines()[-1])
        roof = bj["roofline"]
        c = roof["counts"]
        counts = {"rays": c["rays"], "paths": c["paths"], "boxes": c["boxes"], "prims": np.array(c["prims_by_type"])}
        launches = roof["kernel_launches_per_frame"]
        flops = bench.flops_model(counts) / launches
        avg = rocprof_avg_ms(d / cfg / "kernel_stats.csv")
        tf = flops / (avg * 1e-3) / 1e12
        out = {"config": cfg, "rocprof_avg_ms": round(avg, 3), "bench_kernel_ms": roof["kernel_ms_per_launch"],
               "flops_per_launch": round(flops), "flops_per_ray": round(bench.flops_model(counts) / c["rays"], 1),
               "fp32_TFLOPs": round(tf, 3), "fp32_frac": round(tf / bench.FP32_PEAK_TFLOPS, 5),
               "bench_frac": roof["frac"]}
        pj = ROOT / "profiles" / f"pmc_{cfg}.json"
        if pj.exists():
            b = json.loads(pj.read_text())["hbm_bytes_per_launch"]
            out["hbm_GBps"] = round(b / (avg * 1e-3) / 1e9, 1)
            out["hbm_frac"] = round(b / (avg * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 5)
        vj = ROOT / "profiles" / f"valu_{cfg}.json"
        if vj.exists():
            v = json.loads(vj.read_text())
            if v.get("valu_busy") and v.get("valu_lane_util"):
                out["valu_lane_frac"] = round(v["valu_busy"] * v["valu_lane_util"], 4)
        rows.append(out)
        print(json.dumps(out))
    return rows


if __name__ == "__main__":
    main()
