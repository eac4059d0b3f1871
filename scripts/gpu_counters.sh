# SQ counter pass over bench.py (one rocprofv3 --pmc pass per counter set; no tracing domains).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01_}
ARGS=${ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
    -d $R/gpurun_out/${TAG}sq$i -o sq -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}sq$i.log 2>&1 || exit $?
done
