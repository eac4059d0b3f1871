# Round-5 call a: the new multi-device tests first (rtw_render_multi n > 1 through logical devices + the loopback
# RCCL), then the whole GPU suite, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r05a_}
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}pytest_multi.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest_multi.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest_multi.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}bench_default.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_default.log; exit 1; }
tail -c 400 gpurun_out/${TAG}bench_default.log; echo
for c in cornell-800 cow-1080p monument-4k; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}bench_$c.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'])" gpurun_out/${TAG}bench_$c.log $c
done
