#!/bin/bash
# One perf iteration on the GPU box: parity tests, bench, serialised per-kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/bench_quick.log 2>&1 || exit $?
grep -h "timed\|hot kernel" gpurun_out/bench_quick.log
DSTAGNN_SIDE_STREAM=0 DSTAGNN_GEMM_LOG=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
  --no-extras --hot-iters 1 > gpurun_out/gemm_calls.log 2>&1 || exit $?
DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gcalls -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > gpurun_out/gcalls.log 2>&1 || exit $?
python scripts/step_kernels.py gpurun_out/gcalls/run_kernel_trace.csv gpurun_out/gemm_calls.log 2 > gpurun_out/step_kernels.txt
tail -25 gpurun_out/step_kernels.txt
