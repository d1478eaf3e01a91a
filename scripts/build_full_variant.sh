# Builds a variant of libgwo.so with extra flags applied to EVERY source (host .cpp and .hip), for macros the host
# shares with the kernels (tile sizes, grid): exp/NAME/libgwo.so.  usage: build_full_variant.sh NAME FLAGS...
set -e
NAME=$1; shift
FLAGS="$*"
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/exp/$NAME
rm -rf $OUT/obj && mkdir -p $OUT/obj
for f in $R/flink_amd/csrc/*.hip; do
  b=$(basename $f .hip); EXTRA=""
  [ "$b" = gwo_log ] && EXTRA="-mllvm -amdgpu-atomic-optimizer-strategy=None"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $EXTRA $FLAGS -c $f -o $OUT/obj/$b.hip.o &
done
for f in $R/flink_amd/csrc/*.cpp; do
  b=$(basename $f .cpp)
  g++ -O2 -std=c++17 -fPIC -Wall -Wno-unused-function -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include $FLAGS -c $f -o $OUT/obj/$b.cpp.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgwo.so $OUT/obj/*.o -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $OUT/libgwo.so
