# confirmation of lib/ab/m2 (mesh TU: iterative-ilp without misched clustering) against the default build, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
M=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/m2/librtw_amd.so
TAG=r04m3_ab_ CONFIGS="monument-4k cow-1080p" VARIANTS="$M X=0 $M X=0 $M X=0" bash scripts/gpu_ab.sh || exit 1
