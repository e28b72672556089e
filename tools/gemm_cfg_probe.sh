cd $GRAFT_REPO_ROOT
for shape in "5440 512 384 0 0" "12288 288 170 0 0" "12288 170 96 1 0" "5440 192 512 1 0" "384 5440 512 0 0"; do
  for cfg in 0 1 2; do
    DSTAGNN_GEMM_CFG=$cfg timeout -k 10 60 python3 tools/gemm_probe.py $shape 50 2>/dev/null | sed "s/^/cfg$cfg /"
  done
done
