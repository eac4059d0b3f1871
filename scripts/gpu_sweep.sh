# quick knob sweep: bench one config under several env settings (after the parity tests pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-sw_}
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
for kv in $SWEEP; do
  env $kv timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/${TAG}$kv.log 2>&1 || exit $?
  echo "$kv $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}$kv.log) $(grep -o '"simd_util_rank0": {[^}]*}' gpurun_out/${TAG}$kv.log) $(grep -o '"phase_share_rank0": {[^}]*}' gpurun_out/${TAG}$kv.log)"
done
