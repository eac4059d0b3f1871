# main translation unit (sphere, list-mode and generic kernels) without the scheduler's load / store clustering
# (lib/ab/j1) against the default build, alternating, jumpy and cornell
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
J=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/j1/librtw_amd.so
TAG=r04j1_ab_ CONFIGS="jumpy-1080p cornell-800" VARIANTS="$J X=0 $J X=0 $J X=0" bash scripts/gpu_ab.sh || exit 1
