# one knob over values for one config (tuning gate on): KNOB=RTW_REGEN_MIN VALS="16 24 32" CONFIG=jumpy-1080p TAG=k
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in $(seq ${REPS:-1}); do
  for v in $VALS; do
    env RTW_TUNING=1 $KNOB=$v timeout -k 10 300 python bench.py --config $CONFIG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${v}_$k.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_$k.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'])" gpurun_out/${TAG}_${v}_$k.log $KNOB=$v $CONFIG
  done
done
