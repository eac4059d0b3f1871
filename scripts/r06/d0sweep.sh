# jumpy-1080p over the far-origin split D0 (RTW_FAR_D0, a multiple of the BVH box's diagonal; tuning gate on)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in $(seq ${REPS:-1}); do
  for d0 in ${D0S:-1 0.75 1.5 2}; do
    RTW_TUNING=1 RTW_FAR_D0=$d0 timeout -k 10 300 python bench.py --config jumpy-1080p --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG:-d0}_${d0}_$k.log 2>&1 || { tail -5 gpurun_out/${TAG:-d0}_${d0}_$k.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('D0', sys.argv[2], d['value'], r['kernel_ms_per_frame'])" gpurun_out/${TAG:-d0}_${d0}_$k.log $d0
  done
done
