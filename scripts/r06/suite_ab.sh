# full GPU suite, then every config: new vs the round-5 library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-s}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for c in ${CONFIGS:-jumpy-1080p cornell-800 cow-1080p monument-4k}; do
  CONFIG=$c TAG=${TAG}_$c LIBS="${ABLIBS:-new r05}" REPS=${REPS:-1} STEPS=3 bash scripts/r06/abjumpy.sh || exit 1
done
