#!/bin/bash
# GPU-box driver: run each GPU step under its own time limit; stop at the first
# fault / abort / timeout (exit codes other than 0 or 1).  Logs in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() {
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL: $name rc=$rc, stopping"; exit $rc; fi
  if grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
    echo "FATAL: $name reported a GPU fault, stopping"; exit 99
  fi
  return 0
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
# steps appended from an (untracked) tools/.extra_steps file: extends a queued call's list
[ -f tools/.extra_steps ] && STEPS="$STEPS,$(tr -d '[:space:]' < tools/.extra_steps)"
echo "steps: $STEPS"
IFS=',' read -ra S <<< "$STEPS"
for s in "${S[@]}"; do
  case $s in
    pytest) DSTAGNN_PROFILE_OUT=gpurun_out run pytest_gpu 900 python -u -m pytest tests -m gpu --maxfail=8 -q -rf --timeout 180 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 20 --warmup 5 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    cfgab)  # same-box A/B of one env knob on BASELINE configs: CFGAB_ENV="K=V", CFGAB_CONFIGS="SYN GAMBIA"
            for r in 1 2; do
              BENCH_CONFIGS_STEPS=5 run cfgab_base_$r 300 python tools/bench_configs.py ${CFGAB_CONFIGS:-SYN}
              env ${CFGAB_ENV:-DSTAGNN_TAIL_CT24=1} BENCH_CONFIGS_STEPS=5 timeout -k 10 300 python tools/bench_configs.py ${CFGAB_CONFIGS:-SYN} > gpurun_out/cfgab_knob_$r.log 2>&1 || exit $?
              grep -h "ms_per_step" gpurun_out/cfgab_base_$r.log gpurun_out/cfgab_knob_$r.log | grep configs
            done ;;
    mstep)  run mstep 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mstep -o run --output-format csv -- python3 tools/model_step_prof.py --steps 5 ;;
    dp2)    DSTAGNN_DIST_BACKEND=gloo DSTAGNN_DEVICE_MOD=1 run dp2 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-extras ;;
    pmcs)   echo "== pmcs ($(date +%T))"; bash tools/pmc_step.sh || exit $? ;;
    pmcsum) # summarise the PMC passes on the box so the bench below reads this build's traffic
            python3 tools/pmc_step_summary.py gpurun_out/pmcs profiles/block_pmc.json > gpurun_out/pmcsum.log 2>&1 \
              && cp profiles/block_pmc.json gpurun_out/block_pmc.json || exit $? ;;
    pmcs_gambia) echo "== pmcs GAMBIA ($(date +%T))"; PMC_CONFIG=GAMBIA bash tools/pmc_step.sh || exit $? ;;
    pmcs_syn)    echo "== pmcs SYN ($(date +%T))"; PMC_CONFIG=SYN bash tools/pmc_step.sh || exit $? ;;
    pmcb)   echo "== pmcb ($(date +%T))"; bash tools/pmc_block.sh || exit $?; python3 tools/pmc_block_summary.py gpurun_out/pmcb > gpurun_out/pmcb_summary.txt ;;
    steptrace) bash tools/step_trace.sh final || exit $? ;;
    configs) BENCH_CONFIGS_STEPS=5 run configs 900 python tools/bench_configs.py ;;
    trace_cfg) for c in GAMBIA SYN; do
                 BENCH_CONFIGS_STEPS=3 BENCH_CONFIGS_WARMUP=1 run trace_$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_cfg_$c -o run --output-format csv -- python3 tools/bench_configs.py $c
               done ;;
    serial_cfg) # serialised (one stream) trace + GEMM launch log of SERIAL_CFG (default GAMBIA)
               c=${SERIAL_CFG:-GAMBIA}
               DSTAGNN_SIDE_STREAM=0 DSTAGNN_GEMM_LOG=1 BENCH_CONFIGS_STEPS=2 BENCH_CONFIGS_WARMUP=1 \
                 run serial_$c 300 rocprofv3 --kernel-trace -d gpurun_out/serial_$c -o run --output-format csv -- \
                 python3 tools/bench_configs.py $c ;;
    sweep)  run gemm_sweep 600 python tools/gemm_sweep.py ;;
    sweep1) run gemm_sweep1 300 python tools/gemm_sweep.py --configs auto:auto --iters 50 ;;
    gemmref) run gemm_ref 300 python tools/torch_gemm_ref.py ;;
    knobs)  echo "== knobs ($(date +%T))"
            # KNOB_LIST: ';'-separated env sets ("" = default), e.g. ';DSTAGNN_TAT_MFMA=0'
            IFS=';' read -ra KL <<< "${KNOB_LIST:-;DSTAGNN_TAT_MFMA=0;DSTAGNN_DE_TRANSPOSE=1}"
            REPS=${KNOB_REPS:-2} timeout -k 10 900 bash tools/knob_sweep.sh "${KL[@]}" || exit $? ;;
    gemmlab) run gemm_lab 400 python tools/gemm_lab.py --torch-ref --rounds ${LAB_ROUNDS:-3} --variants ${LAB_VARIANTS:-base} \
               --shapes ${LAB_SHAPES:-12288x288x170:nt,12288x170x96:tt,5440x512x384:nt,5440x512x768:nt,5440x512x1536:nt,5440x192x512:tt,54400x64x96:tt,32640x64x224:tt,65280x32x960:tn,5440x512x192:tn,384x5440x512:nt,12288x170x288:tn,4096x4096x2048:tt} ;;
    *) echo "unknown step $s" ;;
  esac
done
