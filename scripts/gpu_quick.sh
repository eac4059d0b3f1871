# Parity tests + one bench line per config (no profiler).  usage: TAG=x_ CONFIGS="..." bash scripts/gpu_quick.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-q_}
cd $R
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
for c in ${CONFIGS:-jumpy-1080p cornell-800 cow-1080p monument-4k}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/${TAG}bench_$c.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', r['kernel_ms_per_frame'], 'ms', r['simd_util_rank0'], r['phase_share_rank0'])" gpurun_out/${TAG}bench_$c.log $c
done
