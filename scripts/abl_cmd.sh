cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python scripts/gemm_sweep.py --configs 0:32,1:32 > gpurun_out/abl_base.log 2>&1 && \
for X in ${ABL:-LOADS MFMA SYNC}; do
  DSTAGNN_NOCHECK=1 DSTAGNN_LIB=$PWD/dstagnn_drought_amd/libdstagnn_abl_$X.so timeout -k 10 300 python scripts/gemm_sweep.py --configs 0:32,1:32 > gpurun_out/abl_$X.log 2>&1 || exit $?
done
