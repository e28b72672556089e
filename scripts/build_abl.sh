#!/bin/bash
# Ablation builds of the GEMM (timing only; results are wrong by construction):
#   LOADS = no global loads in the k loop, MFMA = FMA instead of MFMA, SYNC = no barrier,
#   STAMP = per-workgroup s_memtime timeline (dstagnn_debug_stamps).
# Produces dstagnn_drought_amd/libdstagnn_abl_<X>.so; use with DSTAGNN_LIB=... DSTAGNN_NOCHECK=1.
set -e
cd "$(dirname "$0")/.."
make -s
for X in ${ABL:-LOADS MFMA SYNC}; do
  mkdir -p build/abl_$X
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DDSTAGNN_ABLATE_$X -c dstagnn_drought_amd/csrc/gemm.hip -o build/abl_$X/gemm.o &
done
wait
for X in ${ABL:-LOADS MFMA SYNC}; do
  objs=$(ls build/*.o | grep -v '/gemm.o$')
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o dstagnn_drought_amd/libdstagnn_abl_$X.so $objs build/abl_$X/gemm.o
done
