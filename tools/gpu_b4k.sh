# B = 4,096 (configs[1]): the product build against a variant (exp/wt_<v>), twice interleaved.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
for pass in 1 2; do
  for v in ${B4K_VARIANTS:-base}; do
    echo "== $v ($pass)"
    timeout -k 10 120 ./exp/wt_$v exp/inputs_4096.bin gpurun_out/wt/b4k_$v.bin gpurun_out/wt/b4k_base.bin || exit 1
  done
done
