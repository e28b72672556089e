cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python scripts/gemm_sweep.py --configs auto:32,0:32 > gpurun_out/abl_base.log 2>&1 && \
DSTAGNN_NOCHECK=1 DSTAGNN_LIB=$PWD/dstagnn_drought_amd/libdstagnn_abl_LOADS.so timeout -k 10 300 python scripts/gemm_sweep.py --configs auto:32,0:32 > gpurun_out/abl_loads.log 2>&1 && \
DSTAGNN_NOCHECK=1 DSTAGNN_LIB=$PWD/dstagnn_drought_amd/libdstagnn_abl_MFMA.so timeout -k 10 300 python scripts/gemm_sweep.py --configs auto:32,0:32 > gpurun_out/abl_mfma.log 2>&1; tail -22 gpurun_out/abl_*.log
