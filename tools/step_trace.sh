#!/bin/bash
# Serialised kernel trace of the benchmark step (DSTAGNN_SIDE_STREAM=0, so every duration is the
# kernel's own) with the GEMM launch log; summary by tools/step_kernels.py.
#   bash tools/step_trace.sh <tag> [extra env assignments...]   e.g. step_trace.sh flash DSTAGNN_FLASH=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 DSTAGNN_SIDE_STREAM=0 DSTAGNN_GEMM_LOG=1
for kv in "$@"; do export "$kv"; done
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 2 --prof-steps 0 \
  > $OUT/bench.log 2> $OUT/gemm.log
rc=$?
echo "== trace $TAG rc=$rc"
[ $rc -ne 0 ] && { tail -5 $OUT/gemm.log; exit $rc; }
python3 tools/step_kernels.py "$(ls $OUT/*/*kernel_trace.csv $OUT/*kernel_trace.csv 2>/dev/null | head -1)" $OUT/gemm.log 2 \
  --json $OUT/family_rocprof.json > $OUT/step_kernels.txt
tail -25 $OUT/step_kernels.txt
