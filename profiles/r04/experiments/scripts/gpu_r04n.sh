# mesh 16-bit stack / 6-wave knob: parity, then A/B on cow and monument; the 2-rank gloo rehearsal of the N>1 path
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04n_}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -k "knobs" > gpurun_out/${TAG}pytest_knobs.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest_knobs.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest_knobs.log
TAG=${TAG}ab_ CONFIGS="cow-1080p monument-4k" VARIANTS="X=0 RTW_MESH_S16=6 X=0 RTW_MESH_S16=6" bash scripts/gpu_ab.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 1 --warmup 1 --spp 32 --backend gloo --check-image > gpurun_out/${TAG}mr_gloo2.log 2>&1 || { tail -20 gpurun_out/${TAG}mr_gloo2.log; exit 1; }
grep -h "check_image\|\"value\"" gpurun_out/${TAG}mr_gloo2.log | cut -c1-300
