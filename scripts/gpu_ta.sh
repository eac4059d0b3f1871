# TA/TCP counter passes over the jumpy bench, one rocprofv3 --pmc pass per ';'-separated set
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-ta_}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
i=0
IFS=';' read -ra SETS_A <<< "${SETS:-TA_TA_BUSY_sum GRBM_GUI_ACTIVE}"
for set in "${SETS_A[@]}"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
    -d $R/gpurun_out/${TAG}pmc$i -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/${TAG}pmc$i.log 2>&1 || exit $?
done
