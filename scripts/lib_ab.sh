#!/bin/bash
# A/B of two library builds: bench step time + serialised per-kernel trace for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  tag=$(basename $lib .so)
  DSTAGNN_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/ab_$tag.log 2>&1 || exit 1
  echo "$tag $(grep -h 'timed\|hot kernel' gpurun_out/ab_$tag.log | tr '\n' ' ')"
  DSTAGNN_LIB=$PWD/$lib DSTAGNN_SIDE_STREAM=0 DSTAGNN_GEMM_LOG=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > gpurun_out/ab_gl_$tag.log 2>&1 || exit 1
  DSTAGNN_LIB=$PWD/$lib DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > /dev/null 2>&1 || exit 1
  python scripts/step_kernels.py gpurun_out/ab_$tag/run_kernel_trace.csv gpurun_out/ab_gl_$tag.log 2 > gpurun_out/ab_steps_$tag.txt
  grep "busy\|  gemm" gpurun_out/ab_steps_$tag.txt
done
