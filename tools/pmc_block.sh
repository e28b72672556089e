#!/bin/bash
# Per-kernel SQ counters of the block step (serialised: DSTAGNN_SIDE_STREAM=0), one pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcb
export PYTHONDONTWRITEBYTECODE=1 DSTAGNN_SIDE_STREAM=0
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1"
pass() {
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -k 10 120 rocprofv3 --pmc "${ctrs[@]}" -d gpurun_out/pmcb/$name -o run --output-format csv -- "$@" > gpurun_out/pmcb/$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
python3 -c "import json, sys; sys.path.insert(0, '.'); from dstagnn_drought_amd._lib import build_stamp; print(json.dumps(build_stamp()))" > gpurun_out/pmcb/build.json
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- $B
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE -- $B
pass c FETCH_SIZE -- $B
pass d WRITE_SIZE -- $B
