# GPU suite + cornell A/B (LDS sample staging vs the build before it) + WRITE_SIZE of both
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04k_}
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/nostage/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="cornell-800" VARIANTS="X=0 $B X=0 $B" bash scripts/gpu_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in X=0 $B; do
  f=$(echo "$v" | tr '/' '_')
  env $v timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "path_kernel<false" \
    -d $R/gpurun_out/${TAG}ws_$f -o ws -- python3 $R/bench.py --config cornell-800 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/${TAG}ws_$f.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}ws_$f.log; exit 1; }
  python3 -c "import csv,sys; print(sys.argv[2], 'WRITE_SIZE GB', sum(float(r['Counter_Value']) for r in csv.DictReader(open(sys.argv[1])))*1024/1e9)" $R/gpurun_out/${TAG}ws_$f/ws_counter_collection.csv "$v"
done
