# dispensers per pass (ndisp): GPU suite, full frames (bench A/B) and 1/8 shares against lib/ab/r06d
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ds2_pytest.log 2>&1 || { tail -20 gpurun_out/ds2_pytest.log; exit 1; }
tail -1 gpurun_out/ds2_pytest.log
for lib in new r06d; do
  if [ $lib = new ]; then unset RTW_LIB_PATH; else export RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/$lib/librtw_amd.so; fi
  timeout -k 10 400 python -u scripts/r06/share8.py > gpurun_out/ds2_share_${lib}.log 2>&1 || { tail -5 gpurun_out/ds2_share_${lib}.log; exit 1; }
  echo $lib; python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['full_kernel_ms'], d['share_kernel_ms'], d['projected_efficiency_kernel'])" gpurun_out/ds2_share_${lib}.log
done
unset RTW_LIB_PATH
for c in cornell-800 monument-4k jumpy-400; do CONFIG=$c LIBS="new r06d" REPS=2 STEPS=3 TAG=ds2_$c bash scripts/r06/abjumpy.sh || exit 1; done
