cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/conc -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --hot-iters 1 > gpurun_out/conc.log 2>&1 || exit 1
for w in 8 12 16 20; do python scripts/stream_util.py gpurun_out/conc/run_kernel_trace.csv $w; done
