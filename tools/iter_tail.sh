#!/bin/bash
# one GPU iteration: full -m gpu suite, same-box knob A/B, serialised step trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/knob_sweep.sh "DSTAGNN_TAIL_CT=0" "DSTAGNN_TAIL_CT=1" "DSTAGNN_TAIL_CT=2" || exit 1
bash tools/step_trace.sh s2 || exit 1
