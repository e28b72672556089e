cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_gpu.log 2>&1; tail -1 gpurun_out/pytest_gpu.log
for g in 0 1; do
DSTAGNN_TAIL_GENERIC=$g DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tab$g -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > /dev/null 2>&1 || exit 1
python - <<PY
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/tab$g/run_kernel_trace.csv')) if 'gtu_tail' in r['Kernel_Name']]
for k in ('fwd','bwd'):
    d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if k in r['Kernel_Name']]
    print('generic=$g', k, round(sum(d[1:])/len(d[1:]),2))
PY
done
