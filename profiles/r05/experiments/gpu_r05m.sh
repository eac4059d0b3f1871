# Round-5 call m: the adaptive ids-per-atomic rule (this build) against HEAD's build (lib/ab/base: fixed batches)
# on configs[0] and one eighth of each GPU config's paths, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab/base/librtw_amd.so
run() {  # config spp variant-name env
  local f=gpurun_out/r05m_${1}_s${2}_${3}.log
  local sp=""; [ "$2" != "0" ] && sp="--spp $2"
  env $4 timeout -k 10 300 python bench.py --config $1 $sp --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $f 2>&1 || { tail -5 $f; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['kernel_ms_per_frame'], 'ms kernel')" $f $1 $2 $3
}
for cs in "jumpy-400 0" "jumpy-1080p 64" "cornell-800 128" "cow-1080p 32" "monument-4k 128"; do
  set -- $cs
  run $1 $2 base RTW_LIB_PATH=$B || exit 1
  run $1 $2 new X=0 || exit 1
  run $1 $2 base2 RTW_LIB_PATH=$B || exit 1
  run $1 $2 new2 X=0 || exit 1
done
