# mesh-config A/B over library builds (scripts/r06/abjumpy.sh per config): LIBS="new top5 ..." REPS=2
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-monument-4k cow-1080p}; do
  CONFIG=$c TAG=${TAG:-m}_$c STEPS=${STEPS:-3} bash scripts/r06/abjumpy.sh || exit 1
done
