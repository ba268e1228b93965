# Build an A/B variant of libhiprag.so with one translation unit compiled with extra flags:
#   bash tools/ab/build_variant.sh <name> <source.hip> "<-D flags>"   ->  tools/ab/libhiprag_<name>.so
# (run after `make -C youtu-rag_amd/csrc`; the other objects are the product's; load it with HIPRAG_LIB_OVERRIDE)
set -e
name=$1; src=$2; flags=$3
cd "$(dirname "$0")/../../youtu-rag_amd/csrc"
mkdir -p ../../tools/ab/obj_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=fast \
  -mllvm -amdgpu-atomic-optimizer-strategy=None $flags -c $src -o ../../tools/ab/obj_$name/${src%.hip}.o
objs=""
for o in $(for f in $(sed -n 's/^SRCS = //p' Makefile) $(sed -n 's/^HOST_SRCS = //p' Makefile); do echo obj/${f%.*}.o; done); do b=$(basename $o); if [ "$b" = "${src%.hip}.o" ]; then objs="$objs ../../tools/ab/obj_$name/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o ../../tools/ab/libhiprag_$name.so
echo built tools/ab/libhiprag_$name.so
