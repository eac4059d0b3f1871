# Round-5 call g: the GPU suite on the build whose mesh hit record skips the meta load of BVH triangle winners (m3),
# then A/B against the previous commit (lib/ab/head) on the meshes and cornell (hand-unrolled rect runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05g_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=${TAG}ab_ CONFIGS="monument-4k cow-1080p" VARIANTS="X=0 RTW_LIB_PATH=$B/head/librtw_amd.so X=1 RTW_LIB_PATH=$B/head/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 X=1" bash scripts/gpu_ab.sh || exit 1
