cd $GRAFT_REPO_ROOT
for nb in 128 256 512; do
  DSTAGNN_COLSUM_BLOCKS=$nb DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cs$nb -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > /dev/null 2>&1 || exit 1
  python - <<PY
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/cs$nb/run_kernel_trace.csv')) if 'colsum' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
print($nb, len(d), round(sum(d)/len(d),2), [round(x,1) for x in d[7:14]])
PY
done
DSTAGNN_COLSUM_2STAGE=1 DSTAGNN_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cs2 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --hot-iters 1 > /dev/null 2>&1
python - <<PY
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/cs2/run_kernel_trace.csv')) if 'colsum' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
print('2stage', len(d), round(sum(d)/len(d)*2,2))
PY
