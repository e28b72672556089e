#!/bin/bash
# Copy the judged profile artefacts from gpurun_out/ (scratch) into profiles/ (tracked),
# tagged with the round: rocprofv3 --kernel-trace --stats summary of `bench.py`, the
# per-kernel summary, the bench JSON line, and the hot kernel's PMC traffic.
#   bash tools/save_profiles.sh r01
set -eu
cd "$(dirname "$0")/.."
R=${1:?round tag, e.g. r01}
mkdir -p profiles
cp gpurun_out/prof/run_kernel_stats.csv "profiles/${R}_bench_kernel_stats.csv"
python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv > "profiles/${R}_bench_kernel_summary.txt"
grep -h '^{' gpurun_out/bench.log | tail -1 > "profiles/${R}_bench.json"
grep -h '^{' gpurun_out/prof.log | tail -1 > "profiles/${R}_bench_under_rocprof.json"
if [ -d gpurun_out/pmc/fetch ] && [ -d gpurun_out/pmc/write ]; then
  python tools/pmc_traffic.py gpurun_out/pmc profiles/hot_kernel_traffic.json > /dev/null
  cp profiles/hot_kernel_traffic.json "profiles/${R}_hot_kernel_traffic.json"
fi
ls -la profiles
