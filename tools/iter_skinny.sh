set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_gemm.log 2>&1; rc=$?; tail -5 gpurun_out/t_gemm.log; [ $rc -eq 0 ] || exit $rc
for e in "DSTAGNN_GEMM_SKINNY=0" "DSTAGNN_SKINNY_FOLD1_KB=512" "DSTAGNN_SKINNY_FOLD1_KB=100000" "DSTAGNN_SKINNY_KPW=64" "DSTAGNN_SKINNY_KPW=128"; do
  env $e timeout -k 10 60 python tools/skinny_probe.py theta || exit 1
done
timeout -k 10 60 python tools/skinny_probe.py || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/bench_q.log 2>&1; rc=$?; grep -E "timed|hot" gpurun_out/bench_q.log; exit $rc
