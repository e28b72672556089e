#!/bin/bash
# PMC passes over the benchmark's block step (serialised: DSTAGNN_SIDE_STREAM=0), each counter
# group in its own rocprofv3 run (--pmc only, no trace domains), plus the FETCH_SIZE /
# WRITE_SIZE width calibration (tools/fetch_calib).  Summary: tools/pmc_step_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# PMC_CONFIG=GAMBIA|SYN|PEMS04|PEMS07: that BASELINE config through tools/bench_configs.py
# (3 steps, one warmup) into gpurun_out/pmcs_<config>; default the bench block (PEMS08)
CFG=${PMC_CONFIG:-}
OUT=gpurun_out/pmcs${CFG:+_$CFG}
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 DSTAGNN_SIDE_STREAM=0
if [ -n "$CFG" ]; then
  export BENCH_CONFIGS_STEPS=2 BENCH_CONFIGS_WARMUP=1
  B="python3 tools/bench_configs.py $CFG"
else
  B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 2 --prof-steps 0"
fi
pass() {
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctrs[@]}" -d $OUT/$name -o run --output-format csv -- "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
python3 -c "import json, sys; sys.path.insert(0, '.'); from dstagnn_drought_amd._lib import build_stamp; print(json.dumps(build_stamp()))" > $OUT/build.json
pass calib_fetch FETCH_SIZE -- tools/fetch_calib
pass calib_write WRITE_SIZE -- tools/fetch_calib
pass fetch FETCH_SIZE -- $B
pass write WRITE_SIZE -- $B
pass mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -- $B
