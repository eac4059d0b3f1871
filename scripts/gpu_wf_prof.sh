# Profile the wavefront prototype on a reduced jumpy frame (spp 32): kernel stats, one SQ pass, FETCH / WRITE.
#   usage: TAG=r04g_ bash scripts/gpu_wf_prof.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04g_}
O=$R/gpurun_out/${TAG}wf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export RTW_WAVEFRONT=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 $R/bench.py --spp ${SPP:-32} --steps 1 --warmup 0 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
tail -c 400 $O/kt.log; echo
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv --kernel-include-regex "wf_|path_kernel" -d $O/sq1 -o sq -- \
  python3 $R/bench.py --spp ${SPP:-32} --steps 1 --warmup 0 --no-cpu-baseline > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --output-format csv --kernel-include-regex "wf_|path_kernel" \
    -d $O/pmc_$p -o pmc -- python3 $R/bench.py --spp ${SPP:-32} --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$p.log 2>&1 || { tail -5 $O/pmc_$p.log; exit 1; }
done
echo wf-prof-done
