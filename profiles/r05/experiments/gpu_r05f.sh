# Round-5 call f: the GPU suite on the build with the short wrapper-chain hit record (kernels without triangles),
# then cornell A/B against the evidence build (lib/ab/head).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05f_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_LIB_PATH=$B/head/librtw_amd.so X=1 RTW_LIB_PATH=$B/head/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
