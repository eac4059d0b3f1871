# Round evidence in one GPU call: parity tests, the default bench line (with the CPU baseline), per
# config a rocprofv3 kernel trace + stats and FETCH_SIZE / WRITE_SIZE PMC passes, then the SQ
# counter sets of the headline config.  usage: TAG=r01i_ bash scripts/gpu_evidence.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r01i_}
TAG=$TAG bash $R/scripts/gpu_round.sh || exit $?
TAG=${TAG}jumpy-1080p_ bash $R/scripts/gpu_counters.sh || exit $?
echo evidence-done
