#!/bin/bash
# Multi-stream kernel trace of the benchmark step (side stream on) -> tools/step_timeline.py:
# per-queue busy, union, idle gaps, kernels in start order.   bash tools/timeline.sh <tag> [env...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
OUT=gpurun_out/tl_$TAG
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
for kv in "$@"; do export "$kv"; done
timeout -k 10 180 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --hot-iters 2 --prof-steps 0 \
  > $OUT/bench.log 2>&1
rc=$?
echo "== timeline $TAG rc=$rc"
[ $rc -ne 0 ] && { tail -5 $OUT/bench.log; exit $rc; }
python3 tools/step_timeline.py "$(ls $OUT/*/*kernel_trace.csv $OUT/*kernel_trace.csv 2>/dev/null | head -1)" 15 \
  > $OUT/timeline.txt
tail -12 $OUT/timeline.txt
