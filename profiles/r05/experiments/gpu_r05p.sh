# Round-5 call p: the in-order reduction with eight samples' loads in flight per wave (lib/ab/red) against the
# r05n build (in-tree lib), interleaved; the path kernel is the same, so the step-time difference is the reduction's.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=r05p_ab_ STEPS=5 CONFIGS="cow-1080p jumpy-1080p cornell-800 monument-4k" VARIANTS="X=0 RTW_LIB_PATH=$B/red/librtw_amd.so X=1 RTW_LIB_PATH=$B/red/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base red; do
  L=""; [ $v = red ] && L="RTW_LIB_PATH=$B/red/librtw_amd.so"
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05p_kt_$v -o kt -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config cow-1080p --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r05p_kt_$v.log 2>&1 || exit 1
done
grep -h reduce_kernel $GRAFT_REPO_ROOT/gpurun_out/r05p_kt_*/*stats.csv | cut -c1-200
