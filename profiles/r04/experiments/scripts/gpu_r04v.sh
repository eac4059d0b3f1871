# time-split table with its parameters in LDS (e3): sphere-world parity, then jumpy A/B against lib/ab/base
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04v_}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/base/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="jumpy-1080p" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
