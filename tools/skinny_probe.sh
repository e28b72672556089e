set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/skp
for cfg in "DSTAGNN_GEMM_SKINNY=0" "DSTAGNN_SKINNY_STOP=0" "DSTAGNN_SKINNY_STOP=1" "DSTAGNN_SKINNY_STOP=2" "DSTAGNN_SKINNY_KPW=256" ; do
  tag=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/skp/$tag -o run --output-format csv -- python3 tools/skinny_probe.py > gpurun_out/skp/$tag.log 2>&1 || exit 1
  echo "$cfg: $(tail -1 gpurun_out/skp/$tag.log)"
  grep -h -E "skinny|gemm_f32|splitk" $(ls gpurun_out/skp/$tag/*kernel_stats.csv gpurun_out/skp/$tag/*/*kernel_stats.csv 2>/dev/null) | cut -c1-160
done
