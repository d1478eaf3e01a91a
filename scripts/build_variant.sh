# Builds an experimental variant of libgwo.so (extra HIP flags, e.g. -DGWO_KTRACE) into exp/NAME/libgwo.so, for
# A/B runs with GWO_LIB_PATH (exp/ is git-ignored; the .so travels to the GPU box with the tree).
set -e
NAME=$1; shift
FLAGS="$*"
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/exp/$NAME
rm -rf $OUT/obj && mkdir -p $OUT/obj
SRC=${SRC:-$R/flink_amd/csrc}   # SRC=dir: kernels from another tree (e.g. a commit's sources, for A/B against it)
for f in $SRC/*.hip; do
  b=$(basename $f .hip)
  EXTRA=""
  [ "$b" = gwo_log ] && EXTRA="-mllvm -amdgpu-atomic-optimizer-strategy=None"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $EXTRA $FLAGS -c $f -o $OUT/obj/$b.hip.o &
done
wait
for f in $SRC/*.hip; do [ -s $OUT/obj/$(basename $f .hip).hip.o ] || { echo "compile failed: $f"; exit 1; }; done   # (obj/ starts empty)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libgwo.so $OUT/obj/*.hip.o $R/build/obj/*.cpp.o -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $OUT/libgwo.so
