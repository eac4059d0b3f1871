# Lane utilisation against trace_run's return quota: for each RTW_QUOTA16 value, the
# bench line, one SQ counter pass (valu_lane_util = SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU) and the
# RTW_LANE_DIAG lane-state shares (lib/ab/lanediag, built by `bash scripts/ab_flags.sh lanediag -DRTW_LANE_DIAG`).
#   usage: TAG=ls_ CONFIGS="jumpy-1080p" QS="1 2 4 8 12 16" bash scripts/gpu_lane_sweep.sh
set -o pipefail
export RTW_TUNING=1  # the library reads tuning knobs only with the gate open
R=$GRAFT_REPO_ROOT
TAG=${TAG:-ls_}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-jumpy-1080p}; do
  for q in ${QS:-1 2 4 8 12 16}; do
    O=$R/gpurun_out/${TAG}${c}_q$q
    mkdir -p $O
    export RTW_QUOTA16=$q
    timeout -k 10 300 python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
      -d $O/sq1 -o sq -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
    RTW_LIB_PATH=$R/raytracer-weekend_amd/lib/ab/lanediag/librtw_amd.so timeout -k 10 300 python3 $R/scripts/lane_diag.py $c > $O/lane_diag.log 2>&1 || { tail -5 $O/lane_diag.log; exit 1; }
    unset RTW_QUOTA16
    python3 - $O $c $q <<'P'
import csv, json, sys, collections
o, c, q = sys.argv[1:]
b = json.loads(open(f"{o}/bench.log").read().strip().splitlines()[-1])
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f"{o}/sq1/sq_counter_collection.csv")):
    per[r.get("Dispatch_Id", "0")][r["Counter_Name"]] += float(r["Counter_Value"])
s = collections.defaultdict(float)
for d in per.values():
    for k, v in d.items():
        s[k] += v / len(per)
lane = json.loads(open(f"{o}/lane_diag.log").read().strip().splitlines()[-1].split(" ", 1)[1])
print(json.dumps({"config": c, "quota16": int(q), "mrays_s": b["value"],
                  "valu_lane_util": round(s["SQ_THREAD_CYCLES_VALU"] / (64 * s["SQ_ACTIVE_INST_VALU"]), 4),
                  "valu_busy": round(s["SQ_INSTS_VALU"] * 2 / (1024 * s["GRBM_GUI_ACTIVE"] / 8), 4),
                  "wave_wait": round(s["SQ_WAIT_INST_ANY"] / s["SQ_WAVE_CYCLES"], 4),
                  "lane_states": lane}))
P
  done
done
echo lane-sweep-done
