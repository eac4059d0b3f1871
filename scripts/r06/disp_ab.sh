# sharded dispensers: the GPU suite on the in-tree build, then full frames and 1/8 shares against lib/ab/r06d
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ds_pytest.log 2>&1 || { tail -20 gpurun_out/ds_pytest.log; exit 1; }
tail -1 gpurun_out/ds_pytest.log
for k in 1 2; do
  for lib in new r06d; do
    if [ $lib = new ]; then unset RTW_LIB_PATH; else export RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/$lib/librtw_amd.so; fi
    timeout -k 10 400 python -u scripts/r06/share8.py > gpurun_out/ds_share_${lib}_$k.log 2>&1 || { tail -5 gpurun_out/ds_share_${lib}_$k.log; exit 1; }
    echo $lib $k; python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['full_kernel_ms'], d['share_kernel_ms'], d['projected_efficiency_kernel'])" gpurun_out/ds_share_${lib}_$k.log
  done
done
unset RTW_LIB_PATH
CONFIG=jumpy-400 LIBS="new r06d" REPS=2 TAG=ds400 bash scripts/r06/abjumpy.sh
