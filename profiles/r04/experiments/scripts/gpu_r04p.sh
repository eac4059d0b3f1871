# mesh walk with the path state in LDS rows: parity (knobs), then monument / cow A/B against the build before it
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04p_}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k "knobs or monument or cow" > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/nolst/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="monument-4k" VARIANTS="X=0 $B RTW_MESH_S16=7 X=0 $B RTW_MESH_S16=7" bash scripts/gpu_ab.sh || exit 1
TAG=${TAG}ab_ CONFIGS="cow-1080p" VARIANTS="X=0 RTW_MESH_S16=6 RTW_MESH_S16=7 X=0" bash scripts/gpu_ab.sh || exit 1
