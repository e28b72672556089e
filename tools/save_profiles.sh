#!/bin/bash
# Copy the judged profile artefacts from gpurun_out/ (scratch) into profiles/ (tracked),
# tagged with the round: rocprofv3 --kernel-trace --stats summary of `bench.py`, the
# per-kernel summary, the bench JSON line, and the step's PMC summary (traffic, MFMA busy).
#   bash tools/save_profiles.sh r01
set -eu
cd "$(dirname "$0")/.."
R=${1:?round tag, e.g. r01}
mkdir -p profiles
cp gpurun_out/prof/run_kernel_stats.csv "profiles/${R}_bench_kernel_stats.csv"
python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv > "profiles/${R}_bench_kernel_summary.txt"
grep -h '^{' gpurun_out/bench.log | tail -1 > "profiles/${R}_bench.json"
grep -h '^{' gpurun_out/prof.log | tail -1 > "profiles/${R}_bench_under_rocprof.json"
if [ -d gpurun_out/pmcs/fetch ] && [ -d gpurun_out/pmcs/write ]; then
  python tools/pmc_step_summary.py gpurun_out/pmcs profiles/block_pmc.json > /dev/null
  cp profiles/block_pmc.json "profiles/${R}_block_pmc.json"
fi
ls -la profiles
