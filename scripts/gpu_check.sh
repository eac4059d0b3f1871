# GPU-box check: parity tests, then a bench line.  usage: TAG=r2_ BENCH_ARGS="..." bash scripts/gpu_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r1_}
mkdir -p gpurun_out
(nproc; rocm-smi --showproductname 2>&1 | head -20) > gpurun_out/${TAG}info.txt || true
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}pytest.log; tail -5 gpurun_out/${TAG}pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/${TAG}bench.log
exit $rc
