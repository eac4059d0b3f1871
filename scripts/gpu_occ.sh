# every config under each RTW_OCC setting (after the parity tests pass)
set -o pipefail
export RTW_TUNING=1  # the library reads tuning knobs only with the gate open
cd $GRAFT_REPO_ROOT
TAG=${TAG:-oc_}
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
for o in ${OCCS:-4 5}; do
  for c in ${CONFIGS:-jumpy-1080p cornell-800 cow-1080p monument-4k}; do
    RTW_OCC=$o timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}$o$c.log 2>&1 || { tail -5 gpurun_out/${TAG}$o$c.log; exit 1; }
    echo "occ$o $c $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}$o$c.log) $(grep -o '"phase_share_rank0": {[^}]*}' gpurun_out/${TAG}$o$c.log)"
  done
done
