#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, --pmc only: no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export PYTHONDONTWRITEBYTECODE=1
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
pass() {  # name, counters..., -- cmd
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  echo "== pmc $name: ${ctrs[*]}"
  timeout -k 10 300 rocprofv3 --pmc "${ctrs[@]}" -d gpurun_out/pmc/$name -o run --output-format csv -- "$@" > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  echo "== rc=$rc"; tail -3 gpurun_out/pmc/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
GEMM="python3 tools/gemm_sweep.py --child --iters 5 --only preconv"
pass fetch FETCH_SIZE -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hot-iters 5
pass write WRITE_SIZE -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hot-iters 5
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -- $GEMM
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -- $GEMM
pass sq3 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE -- $GEMM
