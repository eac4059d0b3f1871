set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
TAG=p1_ bash $R/scripts/gpu_counters.sh || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" -d $R/gpurun_out/p1_cache -o sq -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/p1_cache.log 2>&1 || exit $?
echo ok
