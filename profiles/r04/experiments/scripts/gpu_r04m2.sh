# mesh translation unit flag A/B (lib/ab/m1: iterative-ilp + amdgpu trackers, m2: iterative-ilp without
# misched clustering, m3: max-ilp + amdgpu trackers) against the default build, cow and monument
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
L=/root/repo/raytracer-weekend_amd/lib/ab
V="X=0 RTW_LIB_PATH=$L/m1/librtw_amd.so RTW_LIB_PATH=$L/m2/librtw_amd.so RTW_LIB_PATH=$L/m3/librtw_amd.so X=0"
TAG=r04m2_ab_ CONFIGS="cow-1080p monument-4k" VARIANTS="$V" bash scripts/gpu_ab.sh || exit 1
