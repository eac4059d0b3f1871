# Vector-L1 (TCP) / TA / TD counters of the mesh kernels, one pass per set and config.
#   usage: TAG=r04h_ [CONFIGS="cow-1080p monument-4k"] bash scripts/gpu_tcp.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04h_}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/${TAG}counters_list.txt 2>&1 || true
grep -o "TCP_[A-Z0-9_]*\|TD_[A-Z0-9_]*\|TA_[A-Z0-9_]*" $R/gpurun_out/${TAG}counters_list.txt | sort -u > $R/gpurun_out/${TAG}tcp_names.txt || true
for c in ${CONFIGS:-cow-1080p monument-4k jumpy-1080p}; do
  O=$R/gpurun_out/${TAG}$c
  mkdir -p $O
  i=0
  for set in ${SETS:-"TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_READ_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES"}; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
      -d $O/tcp$i -o tcp -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp$i.log 2>&1 || { echo "set $i failed on $c"; tail -3 $O/tcp$i.log; }
  done
done
echo tcp-done
