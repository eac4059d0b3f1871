"""Turn a scripts/gpu_r02.sh run into the committed evidence under profiles/<round>/.

    python scripts/summarize_round.py gpurun_out r02e_ profiles/r02 [configs...]

Per config it copies the rocprofv3 kernel stats and PMC / SQ counter CSVs and the bench line
(bench.json), writes profiles/pmc_<cfg>.json (HBM bytes per path-kernel launch: FETCH_SIZE x2 +
WRITE_SIZE, KiB -> B, MI355X_MICROARCH.md §HBM) and profiles/valu_<cfg>.json (VALU busy, lane
utilisation, waits; see scripts/valu_summary.py for the formulas), then prints scripts/roofline.py's
recomputation of the roofline from those files.
"""
import csv
import json
import shutil
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def per_dispatch(path, name_key="Kernel_Name", match="path_kernel<false"):
    """Counters per dispatch of the path kernel, averaged."""
    per = defaultdict(lambda: defaultdict(float))
    kernel = None
    for r in csv.DictReader(open(path)):
        if match not in r[name_key]:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id") or "0"
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        kernel = r[name_key]
    out = defaultdict(float)
    for cs in per.values():
        for c, v in cs.items():
            out[c] += v / len(per)
    return dict(out), kernel, len(per)


def main():
    src, tag, dst = Path(sys.argv[1]), sys.argv[2], Path(sys.argv[3])
    cfgs = sys.argv[4:] or ["jumpy-1080p", "cornell-800", "cow-1080p", "monument-4k"]
    for cfg in cfgs:
        s = src / f"{tag}{cfg}"
        d = dst / cfg
        d.mkdir(parents=True, exist_ok=True)
        lines = [l for l in (s / "bench.log").read_text().splitlines() if l.startswith("{")]
        (d / "bench.json").write_text(lines[-1] + "\n")
        # every run of this config in the evidence call used the same in-tree library: its stamp, as the bench
        # line saw it, goes into the published files (bench.py attaches them only to that build)
        sha = json.loads(lines[-1])["roofline"].get("lib_sha")
        for other in (s / "kt.log",):
            js = [l for l in other.read_text().splitlines() if l.startswith("{")] if other.exists() else []
            if js and json.loads(js[-1])["roofline"].get("lib_sha") != sha:
                raise SystemExit(f"{other}: another build than {s / 'bench.log'}")
        shutil.copy(s / "kt" / "kt_kernel_stats.csv", d / "kernel_stats.csv")
        rays = json.loads(lines[-1])["config"]["rays_per_frame"] / json.loads(lines[-1])["roofline"]["kernel_launches_per_frame"]
        pmc = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            f = s / f"pmc_{c}" / "pmc_counter_collection.csv"
            shutil.copy(f, d / f"pmc_{c.lower()}.csv")
            v, kernel, n = per_dispatch(f)
            pmc[c] = v[c] * 1024  # KiB -> B per launch
        pub = {"config": cfg, "world": 1, "launches_per_frame": 1, "kernel": kernel,
               "hbm_bytes_per_launch": 2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"],
               "fetch_bytes_per_launch_raw": pmc["FETCH_SIZE"], "write_bytes_per_launch": pmc["WRITE_SIZE"],
               "correction": "FETCH_SIZE x2 (gfx950 counts 64 B per 128-B request), WRITE_SIZE as is; KiB -> B",
               "source": str(d.relative_to(ROOT)), "lib_sha": sha}
        (ROOT / "profiles" / f"pmc_{cfg}.json").write_text(json.dumps(pub, indent=1))
        c = {}
        for i in (1, 2, 3, 4, 5):
            f = s / f"sq{i}" / "sq_counter_collection.csv"
            if not f.exists():
                continue
            shutil.copy(f, d / f"sq{i}_counter_collection.csv")
            v, kernel, n = per_dispatch(f)
            c.update(v)

        def ratio(a, b, k=1.0):
            return round(c[a] * k / c[b], 4) if a in c and c.get(b) else None

        valu = {"config": cfg, "kernel": kernel, "dispatches": n,
                "valu_busy": round(c["SQ_INSTS_VALU"] * 2 / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4),
                "valu_lane_util": ratio("SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", 1 / 64),
                "wave_wait": ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
                "wave_issue": ratio("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
                "l2_hit": round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4),
                # TA / TD busy: cycles summed over the 256 CUs vs GRBM_GUI_ACTIVE summed over the 8 XCDs
                "ta_busy": round(c["TA_TA_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4) if "TA_TA_BUSY_sum" in c else None,
                "td_busy": round(c["TD_TD_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4) if "TD_TD_BUSY_sum" in c else None,
                # LDS array: active cycles summed over the 256 CUs vs GRBM_GUI_ACTIVE, and the share of them
                # spent on bank conflicts (MI355X_MICROARCH.md §LDS)
                "lds_active": round(c["SQ_LDS_IDX_ACTIVE"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4) if "SQ_LDS_IDX_ACTIVE" in c else None,
                "lds_conflict_share": ratio("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                # vector L1 (TCP): hit share of its accesses (1 - requests it sends to L2 / accesses), and vector
                # loads per ray (SQ_INSTS_VMEM_RD per wave instruction, 64 lanes each, over the frame's rays)
                "tcp_hit": round(1.0 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
                if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in c else None,
                "tcp_pending_stall_share": round(c["TCP_PENDING_STALL_CYCLES_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4)
                if "TCP_PENDING_STALL_CYCLES_sum" in c and c.get("GRBM_GUI_ACTIVE") else None,
                "vmem_rd_per_ray": round(c["SQ_INSTS_VMEM_RD"] * 64 / rays, 3) if c.get("SQ_INSTS_VMEM_RD") and rays else None,
                "counters": {k: round(v) for k, v in sorted(c.items())},
                "source": f"{d.relative_to(ROOT)}/sq*_counter_collection.csv (scripts/gpu_r05_evidence.sh)",
                "lib_sha": sha}
        (ROOT / "profiles" / f"valu_{cfg}.json").write_text(json.dumps(valu, indent=1))
        print(cfg, "pmc", pub["hbm_bytes_per_launch"], "valu_busy", valu["valu_busy"], "lane", valu["valu_lane_util"])
    subprocess.run([sys.executable, str(ROOT / "scripts" / "roofline.py"), str(dst)] + cfgs, check=True)


if __name__ == "__main__":
    main()
