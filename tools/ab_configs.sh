#!/bin/bash
# Same-box interleaved A/B of two library builds on the larger configs (tools/bench_configs.py):
#   bash tools/ab_configs.sh <dir holding the baseline libdstagnn.so> [config names...]
# (_C.so resolves libdstagnn.so by RUNPATH, which LD_LIBRARY_PATH overrides.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OLD=$1; shift
CFGS=${*:-PEMS04 GAMBIA SYN}
for r in 1 2; do
  for lib in new old; do
    L=""; [ $lib = old ] && L=$OLD
    log=gpurun_out/abcfg_${r}_${lib}.log
    LD_LIBRARY_PATH=$L timeout -k 10 300 python -u tools/bench_configs.py $CFGS > $log 2>&1 || { echo "FATAL $lib rep $r"; tail -5 $log; exit 9; }
    echo "rep $r lib=$lib $(grep -h '^{' $log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["ms_per_step"] for k, v in d.items()})')"
  done
done
