# scheduler-strategy A/B: the same sources built with -amdgpu-sched-strategy iterative-ilp / max-memory-clause /
# iterative-minreg (lib/ab/<strategy>) against the default max-ilp build, every GPU config
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
L=/root/repo/raytracer-weekend_amd/lib/ab
V="X=0 RTW_LIB_PATH=$L/iterative-ilp/librtw_amd.so RTW_LIB_PATH=$L/max-memory-clause/librtw_amd.so RTW_LIB_PATH=$L/iterative-minreg/librtw_amd.so X=0"
TAG=r04z_ab_ CONFIGS="jumpy-1080p cornell-800 cow-1080p monument-4k" VARIANTS="$V" bash scripts/gpu_ab.sh || exit 1
