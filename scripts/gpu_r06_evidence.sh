# Round-6 evidence in one GPU call (round 5's script plus the random-world fuzz at two frame sizes and the
# full-spp frames' sha256 check): the GPU suite, the default bench line (CPU baseline included), the
# configs[0] line (jumpy-400: GPU frame + its CPU-restatement baseline), the one-process multi-device
# bench at n = 1, then for every GPU config: its bench line with the CPU baseline, a rocprofv3 kernel
# trace + stats, FETCH_SIZE / WRITE_SIZE PMC passes and five counter sets (the fifth: vector-L1 / TCP counters).  Every GPU step has its own
# time limit and the chain stops at the first failure.
#   usage: TAG=r06z_ [CONFIGS="..."] [NOTEST=1] bash scripts/gpu_r06_evidence.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r06z_}
cd $R
mkdir -p gpurun_out
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo) > gpurun_out/${TAG}host.txt
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}pytest.log
  RTW_FUZZ_SEEDS=3000 RTW_FUZZ_MESH_SEEDS=100 RTW_FUZZ_FRAME=64,36,4 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 180 --timeout-method thread > gpurun_out/${TAG}fuzz3000x4.log 2>&1 || { tail -30 gpurun_out/${TAG}fuzz3000x4.log; exit 1; }
  tail -1 gpurun_out/${TAG}fuzz3000x4.log
  RTW_FUZZ_SEEDS=1000 RTW_FUZZ_FRAME=96,54,8 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -q -k random_world \
    --timeout 180 --timeout-method thread > gpurun_out/${TAG}fuzz1000x8.log 2>&1 || { tail -30 gpurun_out/${TAG}fuzz1000x8.log; exit 1; }
  tail -1 gpurun_out/${TAG}fuzz1000x8.log
  timeout -k 10 600 python -u scripts/fullspp_parity.py --phase verify --configs ${FULLSPP_CONFIGS:-jumpy-1080p,cornell-800,cow-1080p,monument-4k} --out profiles/r06/fullspp_parity.json \
    > gpurun_out/${TAG}fullspp_verify.log 2>&1 || { tail -30 gpurun_out/${TAG}fullspp_verify.log; exit 1; }
  tail -3 gpurun_out/${TAG}fullspp_verify.log
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}bench_default.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_default.log; exit 1; }
  tail -c 300 gpurun_out/${TAG}bench_default.log; echo
  timeout -k 10 300 python bench.py --config jumpy-400 --steps 5 --warmup 2 > gpurun_out/${TAG}bench_jumpy-400.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_jumpy-400.log; exit 1; }
  timeout -k 10 300 python bench.py --multi-device 1 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${TAG}multi_device1_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}multi_device1_bench.log; exit 1; }
  # --gpus 2 without a launcher on a one-GPU box: must exit non-zero and print no bench line
  if timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}gpus2_no_launcher.log 2>&1; then
    echo "bench.py --gpus 2 succeeded on a one-GPU box"; exit 1
  fi
  grep -c '"n_gpus"' gpurun_out/${TAG}gpus2_no_launcher.log && { echo "a bench line was printed"; exit 1; }
  tail -1 gpurun_out/${TAG}gpus2_no_launcher.log
  # the N > 1 bench path rehearsed on this one GPU: 2 ranks, gloo gather, the gathered frame checked bit for bit
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --spp 32 --backend gloo --check-image \
    > gpurun_out/${TAG}multirank_gloo2.log 2>&1 || { tail -5 gpurun_out/${TAG}multirank_gloo2.log; exit 1; }
  grep -h "check_image" gpurun_out/${TAG}multirank_gloo2.log
fi
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-jumpy-1080p cornell-800 cow-1080p monument-4k}; do
  O=$R/gpurun_out/${TAG}$c
  mkdir -p $O
  timeout -k 10 300 python3 $R/bench.py --config $c --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 $R/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
  for p in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --output-format csv --kernel-include-regex "path_kernel|reduce_kernel" \
      -d $O/pmc_$p -o pmc -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$p.log 2>&1 || { tail -5 $O/pmc_$p.log; exit 1; }
  done
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
             "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_WAIT_INST_LDS" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "${TCP_SET:-TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE}"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
      -d $O/sq$i -o sq -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/sq$i.log 2>&1 || { tail -5 $O/sq$i.log; exit 1; }
  done
  echo "profiled $c: $(tail -c 300 $O/bench.log)"
done
echo evidence-done
