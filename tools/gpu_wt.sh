# Time every built tools/wt_<variant> on the benchmark inputs; outputs compared to wt_base.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
timeout -k 10 120 ./tools/wt_base tools/inputs_65536.bin gpurun_out/wt/base.bin || exit 1
for v in ${WT_VARIANTS:-}; do
  echo "== $v"
  timeout -k 10 120 ./tools/wt_$v tools/inputs_65536.bin gpurun_out/wt/$v.bin gpurun_out/wt/base.bin || exit 1
done
echo "== base again"
timeout -k 10 120 ./tools/wt_base tools/inputs_65536.bin gpurun_out/wt/base2.bin gpurun_out/wt/base.bin
