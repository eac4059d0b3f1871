# Round-4 call b: the wavefront prototype's parity tests first, then the whole GPU suite, then the
# default jumpy / cornell / cow / monument lines and the wavefront A/B on jumpy (same box).
#   usage: TAG=r04b_ bash scripts/gpu_r04b.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04b_}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "wavefront" \
  > gpurun_out/${TAG}pytest_wf.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest_wf.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest_wf.log
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
for v in ${VARIANTS:-X=0 RTW_WAVEFRONT=1 RTW_WAVEFRONT=1+RTW_WF_SLOTS=4194304 RTW_WAVEFRONT=1+RTW_WF_SLOTS=1048576 X=0}; do
  f=$(echo "$v" | tr '/+' '__')
  env $(echo "$v" | tr '+' ' ') timeout -k 10 300 python bench.py --config ${CFG:-jumpy-1080p} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}ab_$f.log 2>&1 || { tail -5 gpurun_out/${TAG}ab_$f.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', r['kernel_ms_per_frame'], 'ms', r['counts']['rays'])" gpurun_out/${TAG}ab_$f.log "$v"
done
