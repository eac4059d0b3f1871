# Round-5 call j: cornell knobs after the list-loop / hit-record changes (regeneration threshold, ids per atomic)
# and plain instead of non-temporal sample stores (lib/ab/plainst), interleaved with the default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=r05j_ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_REGEN_MIN=4 RTW_REGEN_MIN=16 RTW_BATCH=512 RTW_BATCH=2048 RTW_LIB_PATH=$B/plainst/librtw_amd.so X=1" bash scripts/gpu_ab.sh || exit 1
