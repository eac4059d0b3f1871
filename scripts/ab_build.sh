# Build librtw_amd.so of a git revision into raytracer-weekend_amd/lib/ab/<name>/ (for RTW_LIB_PATH A/B runs).
#   usage: bash scripts/ab_build.sh <name> [rev=HEAD]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-HEAD}
W=/tmp/ab_wt_$name
rm -rf $W && git -C $R worktree add -f --detach $W $rev >/dev/null 2>&1 || { git -C $R worktree prune; git -C $R worktree add -f --detach $W $rev >/dev/null; }
make -s -C $W/raytracer-weekend_amd -j8 lib/librtw_amd.so >/dev/null
mkdir -p $R/raytracer-weekend_amd/lib/ab/$name
cp $W/raytracer-weekend_amd/lib/librtw_amd.so $R/raytracer-weekend_amd/lib/ab/$name/
git -C $R worktree remove --force $W
echo built $R/raytracer-weekend_amd/lib/ab/$name/librtw_amd.so from $(git -C $R rev-parse --short $rev)
