#!/bin/bash
# GEMM call list of one block step (host log) + per-kernel durations of the same step
# (rocprofv3 kernel trace) -> gpurun_out/gemm_calls.log, gpurun_out/gcalls/
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DSTAGNN_SIDE_STREAM=0 DSTAGNN_GEMM_LOG=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 \
  > gpurun_out/gemm_calls.log 2>&1
DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gcalls -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > gpurun_out/gcalls.log 2>&1
