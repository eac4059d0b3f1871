# Round-5 call s: the frame's tiles in reverse order (bottom rows first: lib/ab/rev, -DRTW_EXP_REV) against the same
# build without it, interleaved.
set -o pipefail
export RTW_TUNING=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
G=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab/rev/librtw_amd.so
run() {  # config spp name env
  local f=gpurun_out/r05s_${1}_s${2}_${3}.log
  local sp=""; [ "$2" != "0" ] && sp="--spp $2"
  env $4 timeout -k 10 300 python bench.py --config $1 $sp --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['kernel_ms_per_frame'], 'ms kernel')" $f $1 $2 $3
}
for cs in "jumpy-400 0" "jumpy-1080p 64" "cow-1080p 32" "cornell-800 128" "jumpy-1080p 0" "cow-1080p 0" "cornell-800 0" "monument-4k 128"; do
  set -- $cs
  run $1 $2 base X=0 || exit 1
  run $1 $2 rev RTW_LIB_PATH=$G || exit 1
  run $1 $2 base2 X=1 || exit 1
  run $1 $2 rev2 RTW_LIB_PATH=$G || exit 1
done
