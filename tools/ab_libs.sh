#!/bin/bash
# Same-box interleaved A/B of the PEMS08 bench step over several libraries:
#   bash tools/ab_libs.sh abtest/ref abtest/db2 -      ("-" = this tree's library)
# REPS (default 3) rounds of 100 timed steps each; prints ms/step per library per round and the medians.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
REPS=${REPS:-3}
STEPS=${AB_STEPS:-100}
for r in $(seq 1 $REPS); do
  for lib in "$@"; do
    tag=$(echo "$lib" | tr '/' '_')
    if [ "$lib" = "-" ]; then E=(); else E=(LD_LIBRARY_PATH=$lib); fi
    env "${E[@]}" timeout -k 10 120 python bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --no-extras ${AB_ARGS:-} \
      > gpurun_out/ab/${tag}_$r.log 2>&1 || { echo "FATAL $lib rep $r"; tail -5 gpurun_out/ab/${tag}_$r.log; exit 9; }
    echo "rep $r [$lib]: $(grep -h 'timed' gpurun_out/ab/${tag}_$r.log)"
  done
done
python3 - "$@" <<'PY'
import re, sys, glob, statistics
for lib in sys.argv[1:]:
    tag = lib.replace("/", "_")
    v = []
    for f in sorted(glob.glob(f"gpurun_out/ab/{tag}_*.log")):
        m = re.search(r"timed \d+ steps: ([0-9.]+) ms/step", open(f).read())
        if m: v.append(float(m.group(1)))
    if v: print(f"{lib:24s} median {statistics.median(v):.4f} ms/step  {v}")
PY
