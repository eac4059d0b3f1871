# Round-5 call o: cornell's hit record without the rect uv divisions when no texture reads uv (lib/ab/uvskip,
# -DRTW_EXP_A), interleaved with the default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=r05o_ab_ CONFIGS="cornell-800" VARIANTS="X=0 RTW_LIB_PATH=$B/uvskip/librtw_amd.so X=1 RTW_LIB_PATH=$B/uvskip/librtw_amd.so" bash scripts/gpu_ab.sh || exit 1
