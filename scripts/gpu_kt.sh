# rocprofv3 kernel stats of one bench config per variant (env words; "|" joins variables of one variant)
#   usage: TAG=kt_ CONFIG=jumpy-1080p VARIANTS="X=1 RTW_PRIMARY=0" bash scripts/gpu_kt.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-kt_}
C=${CONFIG:-jumpy-1080p}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-X=1}; do
  f=$(echo "$v" | tr '/|' '_+')
  v=${v//RTW_LIB_PATH=/RTW_LIB_PATH=$R/}  # relative library paths are relative to the repo (we run from /tmp)
  O=$R/gpurun_out/${TAG}${C}_$f
  mkdir -p $O
  env $(echo "$v" | tr '|' ' ') timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- \
    python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
  echo "== $v: $(tail -c 120 $O/kt.log | tr -d '\n' | cut -c1-100)"
  grep -v "true" $O/kt_kernel_stats.csv | grep -E "path_kernel|primary_kernel" | cut -d, -f1-4 | cut -c1-150
done
