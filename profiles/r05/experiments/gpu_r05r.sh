# Round-5 call r: where configs[0]'s time goes -- jumpy-balls 400x225 at 10 / 50 / 200 / 1000 spp (fixed cost vs
# per-path cost) and its regeneration threshold (RTW_REGEN_MIN 8 / 16 / 24 / 40).
set -o pipefail
export RTW_TUNING=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # config spp name env
  local f=gpurun_out/r05r_${1}_s${2}_${3}.log
  local sp=""; [ "$2" != "0" ] && sp="--spp $2"
  env $4 timeout -k 10 300 python bench.py --config $1 $sp --steps 5 --warmup 2 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['kernel_ms_per_frame'], 'ms kernel', d['config']['rays_per_frame'], 'rays')" $f $1 $2 $3
}
for s in 10 50 200 1000; do run jumpy-400 $s base X=0 || exit 1; done
for v in 8 16 24 40; do run jumpy-400 50 rm$v RTW_REGEN_MIN=$v || exit 1; done
