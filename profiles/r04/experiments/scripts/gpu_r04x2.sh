# triangle leaf test without the normal load (n = ab x ac recomputed): GPU suite, then cow / monument A/B against lib/ab/base
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04t2_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/base/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="monument-4k cow-1080p" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
