# Round-5 call b: the multi-device tests (rtw_render_multi n > 1 through logical devices + the loopback RCCL),
# the whole GPU suite, then A/Bs against the round's starting build (lib/ab/base): cornell (list-mode rect loop
# with per-chain reciprocals) and the meshes with the LDS start-args experiment (lib/ab/mslds).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05b_}
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}pytest_multi.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest_multi.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest_multi.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_LIB_PATH=$B/base/librtw_amd.so X=0 RTW_LIB_PATH=$B/base/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="monument-4k cow-1080p jumpy-1080p" VARIANTS="X=0 RTW_LIB_PATH=$B/mslds/librtw_amd.so RTW_LIB_PATH=$B/base/librtw_amd.so X=0 RTW_LIB_PATH=$B/mslds/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
