# Round-3 evidence in one GPU call: the GPU suite, the default bench line (CPU baseline included), the
# configs[0] line (jumpy-400: GPU frame + its CPU-restatement baseline), the one-process multi-device
# bench at n = 1, then for every GPU config: its bench line with the CPU baseline, a rocprofv3 kernel
# trace + stats, FETCH_SIZE / WRITE_SIZE PMC passes and four SQ counter sets.  Every GPU step has its own
# time limit and the chain stops at the first failure.
#   usage: TAG=r03z_ [CONFIGS="..."] [NOTEST=1] bash scripts/gpu_r03_evidence.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03z_}
cd $R
mkdir -p gpurun_out
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo) > gpurun_out/${TAG}host.txt
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}pytest.log
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}bench_default.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_default.log; exit 1; }
  tail -c 300 gpurun_out/${TAG}bench_default.log; echo
  timeout -k 10 300 python bench.py --config jumpy-400 --steps 5 --warmup 2 > gpurun_out/${TAG}bench_jumpy-400.log 2>&1 || { tail -5 gpurun_out/${TAG}bench_jumpy-400.log; exit 1; }
  timeout -k 10 300 python bench.py --multi-device 1 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${TAG}multi_device1_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}multi_device1_bench.log; exit 1; }
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
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
      -d $O/sq$i -o sq -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/sq$i.log 2>&1 || { tail -5 $O/sq$i.log; exit 1; }
  done
  echo "profiled $c: $(tail -c 300 $O/bench.log)"
done
echo evidence-done
