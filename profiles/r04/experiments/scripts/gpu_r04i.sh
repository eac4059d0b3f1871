# GPU suite, then A/Bs in one call: the SM_IMAGE shade mode on monument / cow (RTW_LIB_PATH = the build
# before it), list mode vs BVH on cornell.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04i_}
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/base/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="monument-4k" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="cow-1080p" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_LIST_MAX=0 X=0 RTW_LIST_MAX=0" bash scripts/gpu_ab.sh || exit 1
