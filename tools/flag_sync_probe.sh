set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/flag_sync_probe d
timeout -k 10 120 ./tools/flag_sync_probe s
mkdir -p gpurun_out/fsp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/fsp/d -o run --output-format csv -- ./tools/flag_sync_probe d > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/fsp/s -o run --output-format csv -- ./tools/flag_sync_probe s > /dev/null
for v in d s; do f=$(ls gpurun_out/fsp/$v/*kernel_trace.csv gpurun_out/fsp/$v/*/*kernel_trace.csv 2>/dev/null | head -1); echo "$v: $(cut -d, -f8 $f | sort | uniq -c | tr '\n' ' ')"; done
