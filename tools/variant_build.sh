#!/bin/bash
# Build a variant of libdstagnn.so with extra compile definitions into scratch/<name>/ for a
# same-box A/B (bench / traces with LD_LIBRARY_PATH=scratch/<name>; _C.so finds libdstagnn.so
# by RUNPATH, so the variant directory on LD_LIBRARY_PATH wins).
#   bash tools/variant_build.sh <name> -DDSTAGNN_GEMM_NS=3 ...
set -eu
cd "$(dirname "$0")/.."
NAME=${1:?name}; shift
OUT=scratch/$NAME
mkdir -p $OUT/obj
ls dstagnn_drought_amd/csrc/*.hip | xargs -P 8 -I{} sh -c \
  'f={}; b=$(basename $f .hip); /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result '"$*"' -c $f -o '"$OUT"'/obj/$b.o'
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libdstagnn.so $OUT/obj/*.o
echo "built $OUT/libdstagnn.so ($*)"
