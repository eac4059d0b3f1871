# Round-3 GPU check in one call: the new GPU tests, the whole GPU suite, the default bench line (CPU
# baseline included), the one-process multi-device bench at n = 1, and the 2-rank gloo rehearsal of
# the N>1 bench path.  Each GPU step has its own time limit; the chain stops at the first failure.
#   usage: TAG=r03a_ [NOTEST=1] [NOBENCH=1] bash scripts/gpu_r03.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r03a_}
cd $R
mkdir -p gpurun_out
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo) > gpurun_out/${T}host.txt
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/${T}pytest_new.log 2>&1 || { tail -40 gpurun_out/${T}pytest_new.log; exit 1; }
  tail -1 gpurun_out/${T}pytest_new.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/${T}pytest.log 2>&1 || { tail -30 gpurun_out/${T}pytest.log; exit 1; }
  tail -1 gpurun_out/${T}pytest.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/${T}bench_default.log 2>&1 || { tail -5 gpurun_out/${T}bench_default.log; exit 1; }
  tail -c 600 gpurun_out/${T}bench_default.log; echo
  timeout -k 10 300 python bench.py --multi-device 1 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${T}multi_device1_bench.log 2>&1 || { tail -5 gpurun_out/${T}multi_device1_bench.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms_per_frame": [0-9.]*' gpurun_out/${T}multi_device1_bench.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --spp 32 --backend gloo --check-image \
    > gpurun_out/${T}multirank_gloo2.log 2>&1 || { tail -20 gpurun_out/${T}multirank_gloo2.log; exit 1; }
  grep -h "check_image\|multi_gpu" gpurun_out/${T}multirank_gloo2.log | cut -c1-300
fi
echo r03-check-done
