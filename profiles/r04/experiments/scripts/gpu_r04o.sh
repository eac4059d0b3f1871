# mesh 16-bit stack occupancy sweep (RTW_MESH_S16 0/6/7/8) on monument, default vs the build before it on cow
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04o_}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k "knobs" > gpurun_out/${TAG}pytest_knobs.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest_knobs.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest_knobs.log
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/s16base/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="monument-4k" VARIANTS="X=0 RTW_MESH_S16=7 RTW_MESH_S16=8 RTW_MESH_S16=0 $B X=0" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="cow-1080p" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
