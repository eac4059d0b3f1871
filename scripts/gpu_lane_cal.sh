# Calibrate the SQ lane-utilisation figure on kernels of known active-lane fraction (scripts/ubench/lane_cal.hip).
#   usage: TAG=x_ bash scripts/gpu_lane_cal.sh   (build the binary first, on the CPU side)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-lc_}
mkdir -p $R/gpurun_out/${TAG}lane_cal
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/scripts/ubench/lane_cal > $R/gpurun_out/${TAG}lane_cal/plain.log 2>&1 || { cat $R/gpurun_out/${TAG}lane_cal/plain.log; exit 1; }
cat $R/gpurun_out/${TAG}lane_cal/plain.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}lane_cal/sq -o sq -- $R/scripts/ubench/lane_cal \
  > $R/gpurun_out/${TAG}lane_cal/sq.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}lane_cal/sq.log; exit 1; }
echo lane-cal-done
