#!/bin/bash
# Build an A/B variant of libdstagnn.so with tat_fused.hip recompiled under extra flags:
#   bash tools/variant_tf.sh <name> <flags...>     -> abtest/<name>/libdstagnn.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p build/var_$NAME abtest/$NAME
for src in ${VARIANT_SRCS:-tat_fused}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
    -c dstagnn_drought_amd/csrc/$src.hip -o build/var_$NAME/$src.o
done
OBJS=$(ls build/*.o | grep -v torch_ops.o)
for src in ${VARIANT_SRCS:-tat_fused}; do OBJS=$(echo "$OBJS" | grep -v "/$src.o"); done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o abtest/$NAME/libdstagnn.so $OBJS build/var_$NAME/*.o
echo "built abtest/$NAME/libdstagnn.so"
