# Round evidence: GPU parity tests, the default bench line (with the CPU baseline), then per config a
# rocprofv3 kernel trace + stats and FETCH_SIZE / WRITE_SIZE PMC passes.  usage: TAG=r01f_ bash scripts/gpu_round.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01f_}
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}bench.log 2>&1 || { tail -5 gpurun_out/${TAG}bench.log; exit 1; }
tail -1 gpurun_out/${TAG}bench.log
for c in ${CONFIGS:-jumpy-1080p cornell-800 cow-1080p monument-4k jumpy-400}; do
  TAG=${TAG}${c}_ ARGS="--config $c --steps 2 --warmup 1 --no-cpu-baseline" PMC_ARGS="--config $c" bash scripts/gpu_profile.sh > /dev/null || exit $?
  echo "profiled $c"
done
