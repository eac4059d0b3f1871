"""Summarise a gpu_counters.sh run (SQ counters of the render kernel) into profiles/valu_<cfg>.json.

    python scripts/valu_summary.py gpurun_out r01_ jumpy-1080p

Derived figures (per path_kernel<false,...> dispatch, counters averaged over dispatches):
  valu_busy      SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   share of SIMD cycles issuing VALU
  valu_lane_util SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)        active lanes per VALU op
  wave_wait      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES                         waves parked on s_waitcnt
  wave_issue     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES                       waves issuing an instruction
  l2_hit         TCC_HIT / (TCC_HIT + TCC_MISS)
  ta_busy/td_busy TA_TA_BUSY_sum, TD_TD_BUSY_sum / (256 CUs x GRBM_GUI_ACTIVE / 8)
MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles; GRBM_GUI_ACTIVE is the sum over
the 8 XCDs; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* all count quad-cycles, so their ratios
need no correction.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def load(path):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    kernel = None
    for r in csv.DictReader(open(path)):
        if "path_kernel<false" not in r["Kernel_Name"]:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id") or "0"
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        kernel = r["Kernel_Name"]
    out = defaultdict(float)
    for cs in per.values():
        for c, v in cs.items():
            out[c] += v / len(per)
    return dict(out), kernel, len(per)


def main():
    src, tag, cfg = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
    dst = Path(sys.argv[4]) if len(sys.argv) > 4 else Path(__file__).resolve().parent.parent / "profiles"
    c, kernel, n = {}, None, 0
    for i in (1, 2, 3):
        f = src / f"{tag}sq{i}" / "sq_counter_collection.csv"
        if f.exists():
            cs, kernel, n = load(f)
            c.update(cs)
    if not c:
        raise SystemExit(f"no counter files under {src}/{tag}sq*")

    def ratio(a, b, k=1.0):
        return round(c[a] * k / c[b], 4) if a in c and c.get(b) else None

    out = {"config": cfg, "kernel": kernel, "dispatches": n,
           "valu_busy": round(c["SQ_INSTS_VALU"] * 2 / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4)
           if "SQ_INSTS_VALU" in c and c.get("GRBM_GUI_ACTIVE") else None,
           "valu_lane_util": ratio("SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", 1 / 64),
           "wave_wait": ratio("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
           "wave_issue": ratio("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
           "l2_hit": round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
           if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0 else None,
           # vector-memory address (TA) and data-return (TD) units: busy cycles summed over the 256 CUs
           # against GRBM_GUI_ACTIVE (summed over the 8 XCDs)
           "ta_busy": round(c["TA_TA_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4)
           if c.get("TA_TA_BUSY_sum") and c.get("GRBM_GUI_ACTIVE") else None,
           "td_busy": round(c["TD_TD_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4)
           if c.get("TD_TD_BUSY_sum") and c.get("GRBM_GUI_ACTIVE") else None,
           "counters": {k: round(v) for k, v in sorted(c.items())},
           "source": f"{src}/{tag}sq1..3 (scripts/gpu_r02.sh)"}
    (dst / f"valu_{cfg}.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
