# One bench line per tuning knob setting (jumpy-1080p unless CONFIG is set).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C=${CONFIG:-jumpy-1080p}
for kv in "${@:-X=0}"; do
  n=${kv//\//_}
  env $kv timeout -k 10 200 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/knob_$n.log 2>&1 || { tail -3 gpurun_out/knob_$n.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms_per_frame'], r['node_fetches_per_ray'], r['prim_tests_per_ray'])" gpurun_out/knob_$n.log "$kv"
done
