#!/bin/bash
# Same-box interleaved A/B of the PEMS08 bench step: the baseline library (LD_LIBRARY_PATH=$1)
# against this tree's library under each of the given env settings ("-" = none).
#   bash tools/ab_step.sh abtest/base - DSTAGNN_WQKV_SIDE=1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
OLD=$1; shift
VARS=("$@")
for r in 1 2 3; do
  LD_LIBRARY_PATH=$OLD timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extras \
    > gpurun_out/ab/old_$r.log 2>&1 || { echo "FATAL old rep $r"; tail -5 gpurun_out/ab/old_$r.log; exit 9; }
  echo "rep $r old: $(grep -h timed gpurun_out/ab/old_$r.log)"
  i=0
  for v in "${VARS[@]}"; do
    i=$((i + 1))
    E=(); [ "$v" != "-" ] && E=("$v")
    env "${E[@]}" timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extras \
      > gpurun_out/ab/new${i}_$r.log 2>&1 || { echo "FATAL new $v rep $r"; tail -5 gpurun_out/ab/new${i}_$r.log; exit 9; }
    echo "rep $r new[$v]: $(grep -h timed gpurun_out/ab/new${i}_$r.log)"
  done
done
