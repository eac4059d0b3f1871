# Round-5 call i: shading sub-phase timers (COUNT build of lib/ab/shdiag, -DRTW_SHADE_DIAG) per config: the bench
# line's phase_share keys sample / node_loop / leaf_tests / path_start then carry hit record / unit + texture /
# scatter / (unused) shares of the wave cycles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/raytracer-weekend_amd/lib/ab
TAG=r05i_ CONFIGS="cornell-800 jumpy-1080p monument-4k cow-1080p" VARIANTS="RTW_LIB_PATH=$B/shdiag/librtw_amd.so" STEPS=1 bash scripts/gpu_ab.sh || exit 1
