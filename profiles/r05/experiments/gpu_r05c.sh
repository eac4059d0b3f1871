# Round-5 call c: the GPU suite on the build with the LDS start args in the S16 mesh walk and the grouped list-mode
# rect loop, then A/Bs: cornell against the per-rect loop of the previous commit (lib/ab/head), the meshes at 7 waves.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05c_}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_LIB_PATH=$B/head/librtw_amd.so X=1 RTW_LIB_PATH=$B/head/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="monument-4k cow-1080p" VARIANTS="X=0 RTW_MESH_S16=7 X=1 RTW_MESH_S16=7" bash scripts/gpu_ab.sh || exit 1
