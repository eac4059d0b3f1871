# HBM bytes (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes) of the path kernel for A/B libraries.
#   usage: TAG=x_ CONFIGS="jumpy-1080p" LIBS="default raytracer-weekend_amd/lib/ab/nt0/librtw_amd.so" bash scripts/gpu_pmc_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-pa_}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-jumpy-1080p}; do
  for lib in ${LIBS:-default}; do
    f=$(basename $(dirname $lib))
    O=$R/gpurun_out/${TAG}${c}_$f
    mkdir -p $O
    for p in FETCH_SIZE WRITE_SIZE; do
      if [ "$lib" = default ]; then unset RTW_LIB_PATH; else export RTW_LIB_PATH=$R/$lib; fi
      timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --output-format csv --kernel-include-regex "path_kernel|reduce_kernel" \
        -d $O/pmc_$p -o pmc -- python3 $R/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$p.log 2>&1 || { tail -5 $O/pmc_$p.log; exit 1; }
    done
    python3 - $O <<'P'
import csv, sys, collections
o = sys.argv[1]
for p in ("FETCH_SIZE", "WRITE_SIZE"):
    tot = collections.defaultdict(float)
    for r in csv.DictReader(open(f"{o}/pmc_{p}/pmc_counter_collection.csv")):
        tot[r["Kernel_Name"].split("(")[0][:40]] += float(r["Counter_Value"]) * 1024
    print(o.split("/")[-1], p, {k: round(v / 1e9, 2) for k, v in tot.items()}, "GB")
P
  done
done
