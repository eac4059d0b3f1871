# Round-5 call l: ids per atomic (RTW_BATCH) on small frames -- configs[0] (jumpy 400x225x50: 4.5 M paths for
# 8,192 resident waves, i.e. 4,395 batches of 1,024: half the waves get none) and one eighth of each GPU config's
# paths (the per-GPU share of an 8-GPU frame, via --spp).
set -o pipefail
export RTW_TUNING=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # config spp variant
  local f=gpurun_out/r05l_${1}_s${2}_$(echo "$3" | tr '/|' '_+').log
  local sp=""; [ "$2" != "0" ] && sp="--spp $2"
  env $3 timeout -k 10 300 python bench.py --config $1 $sp --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['kernel_ms_per_frame'], 'ms kernel')" $f $1 $2 "$3"
}
for v in X=0 RTW_BATCH=512 RTW_BATCH=256 RTW_BATCH=128 RTW_BATCH=64 X=1; do run jumpy-400 0 $v || exit 1; done
for v in X=0 RTW_BATCH=256 RTW_BATCH=128 X=1; do run jumpy-1080p 64 $v || exit 1; done
for v in X=0 RTW_BATCH=256 RTW_BATCH=128 X=1; do run cornell-800 128 $v || exit 1; done
for v in X=0 RTW_BATCH=512 RTW_BATCH=256 X=1; do run cow-1080p 32 $v || exit 1; done
for v in X=0 RTW_BATCH=512 RTW_BATCH=256 X=1; do run monument-4k 128 $v || exit 1; done
