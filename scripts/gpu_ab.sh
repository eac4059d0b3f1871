# A/B a tuning knob: for each config and each env setting, one bench line (no CPU baseline).
#   usage: TAG=x_ CONFIGS="jumpy-1080p monument-4k" VARIANTS="RTW_OCC=5 RTW_OCC=6|RTW_QUOTA16=10" bash scripts/gpu_ab.sh
#   (one variant per word; "|" joins several variables of one variant)
set -o pipefail
export RTW_TUNING=1  # the library reads tuning knobs only with the gate open
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-ab_}
for c in ${CONFIGS:-jumpy-1080p monument-4k}; do
  for v in ${VARIANTS:-X=0}; do
    f=$(echo "$v" | tr '/|' '_+')
    env $(echo "$v" | tr '|' ' ') timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}${c}_${f}.log 2>&1 || { tail -5 gpurun_out/${TAG}${c}_${f}.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], 'Mrays/s', r['kernel_ms_per_frame'], 'ms nodes/ray', r['node_fetches_per_ray'], 'prims/ray', r['prim_tests_per_ray'], r['phase_share_rank0'])" gpurun_out/${TAG}${c}_${f}.log $c $v
  done
done
