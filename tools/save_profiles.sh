#!/bin/bash
# Copy the judged profile artefacts from gpurun_out/ (scratch) into profiles/ (tracked), tagged
# with the round; every file carries (or sits beside) the build stamp of the library it measured.
#   bash tools/save_profiles.sh r03
# Inputs (tools/gpu_check.sh steps): bench + prof (kernel trace --stats of bench.py), pmcs (PMC
# passes over the PEMS08 step), steptrace (serialised step, per-kernel times), pmcb (per-kernel
# SQ issue / wait counters), pmcs_gambia / pmcs_syn, trace_cfg (GAMBIA / SYN kernel traces),
# configs (every BASELINE config).
set -u
cd "$(dirname "$0")/.."
R=${1:?round tag, e.g. r03}
mkdir -p profiles
STAMP=$(python3 -c "import json, sys; sys.path.insert(0, '.'); from dstagnn_drought_amd._lib import build_stamp; print(json.dumps(build_stamp()))")
HEAD=$(git rev-parse --short HEAD)
hdr() { echo "# build: $STAMP  git: $HEAD  (tools/save_profiles.sh $R)"; }
if [ -f gpurun_out/prof/run_kernel_stats.csv ]; then
  cp gpurun_out/prof/run_kernel_stats.csv "profiles/${R}_bench_kernel_stats.csv"
  { hdr; python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv; } > "profiles/${R}_bench_kernel_summary.txt"
fi
[ -f gpurun_out/bench.log ] && grep -h '^{' gpurun_out/bench.log | tail -1 > "profiles/${R}_bench.json"
[ -f gpurun_out/prof.log ] && grep -h '^{' gpurun_out/prof.log | tail -1 > "profiles/${R}_bench_under_rocprof.json"
if [ -d gpurun_out/pmcs/fetch ] && [ -d gpurun_out/pmcs/write ]; then
  python3 tools/pmc_step_summary.py gpurun_out/pmcs profiles/block_pmc.json > /dev/null
  cp profiles/block_pmc.json "profiles/${R}_block_pmc.json"
fi
for c in GAMBIA SYN; do
  lc=$(echo $c | tr A-Z a-z)
  if [ -d gpurun_out/pmcs_$c/fetch ]; then
    PMC_WORKLOAD=$lc python3 tools/pmc_step_summary.py gpurun_out/pmcs_$c "profiles/${R}_${lc}_pmc.json" > /dev/null
  fi
  f=$(ls gpurun_out/trace_cfg_$c/*kernel_stats.csv gpurun_out/trace_cfg_$c/*/*kernel_stats.csv 2>/dev/null | head -1)
  t=$(ls gpurun_out/trace_cfg_$c/*kernel_trace.csv gpurun_out/trace_cfg_$c/*/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && cp "$f" "profiles/${R}_${lc}_kernel_stats.csv"
  [ -n "$t" ] && { hdr; python3 tools/trace_by_grid.py "$t" 30; } > "profiles/${R}_${lc}_kernels_by_grid.txt"
  # one step of the normal two-stream run: which stream ends the step
  [ -n "$t" ] && { hdr; python3 tools/step_timeline.py "$t" 1; } > "profiles/${R}_${lc}_step_timeline.txt" 2>&1
done
[ -f gpurun_out/prof/run_kernel_trace.csv ] && { hdr; python3 tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv; } \
  > "profiles/${R}_step_timeline_under_rocprof.txt" 2>&1
[ -f gpurun_out/trace_final/step_kernels.txt ] && { hdr; cat gpurun_out/trace_final/step_kernels.txt; } > "profiles/${R}_step_kernels.txt"
if [ -f gpurun_out/pmcb_summary.txt ]; then
  { echo "# build (measured): $(cat gpurun_out/pmcb/build.json 2>/dev/null)  git: $HEAD"; cat gpurun_out/pmcb_summary.txt; } > "profiles/${R}_step_sq_pmc.txt"
fi
[ -f gpurun_out/rccl_world1.json ] && cp gpurun_out/rccl_world1.json "profiles/${R}_rccl_world1.json"
[ -f gpurun_out/trace_final/family_rocprof.json ] && { cp gpurun_out/trace_final/family_rocprof.json profiles/family_rocprof.json;
  cp gpurun_out/trace_final/family_rocprof.json "profiles/${R}_family_rocprof.json"; }
[ -f gpurun_out/trace_final/gemm.log ] && grep -h '^\[gemm\]\|^\[fused\]' gpurun_out/trace_final/gemm.log > "profiles/${R}_step_family_calls.log"
[ -f gpurun_out/configs.log ] && grep -h '^{' gpurun_out/configs.log | tail -1 > "profiles/${R}_configs_bench.json"
ls -la profiles | grep "$R"
