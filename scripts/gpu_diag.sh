# Vector-memory / LDS / instruction-mix counters of the path kernel (one rocprofv3 --pmc pass per set).
#   usage: TAG=dg_ CONFIGS="jumpy-1080p" bash scripts/gpu_diag.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-dg_}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-jumpy-1080p}; do
  O=$R/gpurun_out/${TAG}$c
  mkdir -p $O
  i=0
  for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL" \
             "GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SMEM SQ_IFETCH"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
      -d $O/dg$i -o dg -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $O/dg$i.log 2>&1 || { tail -5 $O/dg$i.log; exit 1; }
  done
  echo "diag $c done"
done
