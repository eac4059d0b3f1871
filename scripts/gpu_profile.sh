# rocprofv3 passes over bench.py: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  usage: TAG=r01_ bash scripts/gpu_profile.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01_}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
[ -n "$SKIP_KT" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}kt -o kt -- \
  python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}kt.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv --kernel-include-regex "path_kernel|reduce_kernel" \
    -d $R/gpurun_out/${TAG}pmc_$c -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline $PMC_ARGS \
    > $R/gpurun_out/${TAG}pmc_$c.log 2>&1 || exit $?
done
find $R/gpurun_out -name "*.csv" | head -20
