# Kernel timing of the variants in VARS at the batch sizes in BS (exp/inputs_<B>.bin).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
for b in ${BS:-65536}; do
  for pass in 1 2; do
    for v in $VARS; do
      echo "== $v B=$b ($pass)"
      timeout -k 10 120 ./exp/wt_$v exp/inputs_$b.bin gpurun_out/wt/${v}_$b.bin gpurun_out/wt/base_$b.bin || exit 1
    done
  done
done
