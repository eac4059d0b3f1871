# Round-5 call k: what the sample stores and the waits behind them cost (lib/ab/nostore, -DRTW_DIAG_NO_STORE,
# a timing diagnostic whose image is not computed), interleaved with the default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=r05k_ab_ CONFIGS="cornell-800 jumpy-1080p monument-4k cow-1080p" VARIANTS="X=0 RTW_LIB_PATH=$B/nostore/librtw_amd.so X=1 RTW_LIB_PATH=$B/nostore/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
