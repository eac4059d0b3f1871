# jumpy-1080p A/B over library builds: LIBS="new r05 fard1 ..." (new = the in-tree library), REPS rounds, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-ab}
for k in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-new r05}; do
    if [ $lib = new ]; then unset RTW_LIB_PATH; else export RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/$lib/librtw_amd.so; fi
    timeout -k 10 300 python bench.py --config ${CONFIG:-jumpy-1080p} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${lib}_$k.log 2>&1 || { tail -5 gpurun_out/${TAG}_${lib}_$k.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', r['kernel_ms_per_frame'], 'ms', r.get('node_fetches_per_ray'), r.get('prim_tests_per_ray'), r['phase_share_rank0'])" gpurun_out/${TAG}_${lib}_$k.log $lib
  done
done
