# A/B: tile-local id dispensing (RTW_WG_TILES) vs the build before it, per config, one call
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${TAG:-r04m_}
if [ -n "$TEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${TAG}pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}pytest.log
fi
B=RTW_LIB_PATH=/root/repo/raytracer-weekend_amd/lib/ab/nostage/librtw_amd.so
TAG=${TAG}ab_ CONFIGS="${CONFIGS:-monument-4k cow-1080p jumpy-1080p cornell-800}" VARIANTS="${VARIANTS:-$B X=0 RTW_WG_TILES=80 RTW_WG_TILES=95 $B RTW_WG_TILES=80}" bash scripts/gpu_ab.sh || exit 1
