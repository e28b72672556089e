#!/bin/bash
# Same-box interleaved A/B of runtime knobs on the PEMS08 bench (ms/step per run).
# usage: bash tools/knob_sweep.sh "ENV=a" "ENV=b" ...   (each arg: space-separated env assignments, "" = default)
# A/B of two builds: put the baseline libdstagnn.so in a directory D and pass "LD_LIBRARY_PATH=D"
# (the operator library _C.so resolves libdstagnn.so by RUNPATH, which LD_LIBRARY_PATH overrides).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REPS=${REPS:-2}
for r in $(seq 1 "$REPS"); do
  for cfg in "$@"; do
    out=$(env $cfg timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extras 2>&1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "FATAL rc=$rc cfg=[$cfg]"; echo "$out" | tail -5; exit $rc; fi
    echo "rep $r [$cfg] $(echo "$out" | grep -o 'timed 100 steps: [0-9.]* ms/step')" | tee -a gpurun_out/knob_sweep.txt
  done
done
