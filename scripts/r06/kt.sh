# kernel trace summary of one bench config: CONFIG=jumpy-1080p TAG=x bash scripts/r06/kt.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-kt}_prof -o run -- python3 bench.py --config ${CONFIG:-jumpy-1080p} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/${TAG:-kt}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG:-kt}_bench.log; exit 1; }
f=$(find gpurun_out/${TAG:-kt}_prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:110], r['Calls'], round(float(r['TotalDurationNs'])/1e6,3),'ms total', round(float(r['AverageNs'])/1e6,3),'ms avg')
" $f
