#!/bin/bash
# one GPU iteration: full -m gpu suite, bench, serialised step trace (tag $1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
TAG=${1:-q}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/bench_$TAG.log 2>&1 || exit 1
  grep -E "timed" gpurun_out/bench_$TAG.log
done
bash tools/step_trace.sh $TAG || exit 1
