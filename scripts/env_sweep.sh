#!/bin/bash
# bench step time under environment overrides: VAR=v1,v2,...  (one bench per value)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/sweep_$v.log 2>&1 || exit 1
  echo "$VAR=$v $(grep -h timed gpurun_out/sweep_$v.log)"
done
