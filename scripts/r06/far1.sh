# Round 6, far-origin walk: its parity tests, the directed test on the round-5 library (must fail: the test is
# sensitive), and jumpy-1080p A/B (new vs round-5 library).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="timeout -k 10"
PY="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 900 $PY tests/test_gpu_far.py "tests/test_gpu_fullres.py::test_whole_frame_bit_exact" tests/test_gpu_multi.py > gpurun_out/f1_pytest.log 2>&1 || { tail -30 gpurun_out/f1_pytest.log; exit 1; }
tail -3 gpurun_out/f1_pytest.log
RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/r05/librtw_amd.so $T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_far.py -k "camera or regressions" > gpurun_out/f1_oldlib.log 2>&1
echo "old library exit $? (1 = its far-origin tests fail, as expected)"; grep -E "PASSED|FAILED" gpurun_out/f1_oldlib.log | cut -c1-150
for k in 1 2; do
  for lib in new r05; do
    if [ $lib = r05 ]; then export RTW_LIB_PATH=$PWD/raytracer-weekend_amd/lib/ab/r05/librtw_amd.so; else unset RTW_LIB_PATH; fi
    $T 300 python bench.py --config jumpy-1080p --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/f1_bench_${lib}_$k.log 2>&1 || { tail -5 gpurun_out/f1_bench_${lib}_$k.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', r['kernel_ms_per_frame'], 'ms', r.get('node_fetches_per_ray'), r.get('prim_tests_per_ray'))" gpurun_out/f1_bench_${lib}_$k.log $lib
  done
done
unset RTW_LIB_PATH
$T 300 python scripts/fullspp_parity.py --phase gpu --configs jumpy-1080p,cornell-800,cow-1080p --dir gpurun_out/fullspp > gpurun_out/f1_fullspp.log 2>&1 || { tail -5 gpurun_out/f1_fullspp.log; exit 1; }
cut -c1-200 gpurun_out/f1_fullspp.log
