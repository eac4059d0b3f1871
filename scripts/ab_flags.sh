# Build librtw_amd.so of the WORKING TREE with extra kernel flags into raytracer-weekend_amd/lib/ab/<name>/.
#   usage: bash scripts/ab_flags.sh <name> "-DRTW_SPEC_SAMPLE=0 ..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=$2
W=/tmp/ab_src_$name
rm -rf $W && mkdir -p $W && cp -r $R/raytracer-weekend_amd/csrc $R/raytracer-weekend_amd/Makefile $W/ && mkdir -p $W/../include
rm -rf /tmp/include && cp -r $R/include /tmp/include
# XFLAGS reaches both kernel translation units (rtw_kernel.hip and the mesh kernels' rtw_kernel_mesh.hip)
make -s -C $W -j8 lib/librtw_amd.so XFLAGS="$flags" >/dev/null
mkdir -p $R/raytracer-weekend_amd/lib/ab/$name
cp $W/lib/librtw_amd.so $R/raytracer-weekend_amd/lib/ab/$name/
echo built lib/ab/$name with "$flags"
