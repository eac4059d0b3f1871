# sharded dispensers in the LDS-node kernels only: GPU suite, jumpy full / 1/8 share / configs[0] against lib/ab/r06d
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ds3_pytest.log 2>&1 || { tail -20 gpurun_out/ds3_pytest.log; exit 1; }
tail -1 gpurun_out/ds3_pytest.log
for k in 1 2; do
for lib in new r06d; do
  if [ $lib = new ]; then unset RTW_LIB_PATH; else export RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/$lib/librtw_amd.so; fi
  timeout -k 10 400 python -u scripts/r06/share8.py --configs jumpy-1080p > gpurun_out/ds3_share_${lib}_$k.log 2>&1 || { tail -5 gpurun_out/ds3_share_${lib}_$k.log; exit 1; }
  echo $lib; grep -o '"full_kernel_ms.*' gpurun_out/ds3_share_${lib}_$k.log
done
done
unset RTW_LIB_PATH
for c in jumpy-1080p jumpy-400 cornell-800; do CONFIG=$c LIBS="new r06d" REPS=2 STEPS=3 TAG=ds3_$c bash scripts/r06/abjumpy.sh || exit 1; done
