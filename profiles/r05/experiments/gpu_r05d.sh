# Round-5 call d: the GPU suite on the build without the hot-loop spills (scalar wave index for the id pool, the
# throughput read where it is used, the root as a scalar), then A/B against the previous commit (lib/ab/head).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05d_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=${TAG}ab_ CONFIGS="monument-4k cow-1080p jumpy-1080p cornell-800" VARIANTS="X=0 RTW_LIB_PATH=$B/head/librtw_amd.so X=1 RTW_LIB_PATH=$B/head/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
