# always-list prim indices computed instead of loaded: GPU suite, then every config against lib/ab/base, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04al_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/base/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="cornell-800 jumpy-1080p cow-1080p monument-4k" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
