# bench every BASELINE.json config on one GPU (no CPU baseline, 2 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-cf_}
for c in ${CONFIGS:-jumpy-400 jumpy-1080p cornell-800 cow-1080p monument-4k}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}$c.log 2>&1 || { tail -5 gpurun_out/${TAG}$c.log; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}$c.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}$c.log) $(grep -o '"rays_per_frame": [0-9]*' gpurun_out/${TAG}$c.log) $(grep -o '"simd_util_rank0": {[^}]*}' gpurun_out/${TAG}$c.log) $(grep -o '"phase_share_rank0": {[^}]*}' gpurun_out/${TAG}$c.log)"
done
