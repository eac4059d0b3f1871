# GPU suite + the list-mode chain skip A/B on cornell
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04j_}
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_CHAIN_SKIP=0 X=0 RTW_CHAIN_SKIP=0" bash scripts/gpu_ab.sh || exit 1
