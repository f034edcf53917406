# Time built tools/wt_<variant> binaries on the benchmark inputs (outputs compared to the
# first one); each variant is timed twice, interleaved, to expose drift between runs.
#   WT_VARIANTS="base orig" bash tools/gpu_wt.sh
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
set -- ${WT_VARIANTS:-base}
ref=$1
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v ($pass)"
    timeout -k 10 120 ./tools/wt_$v tools/inputs_65536.bin gpurun_out/wt/$v.bin gpurun_out/wt/$ref.bin || exit 1
  done
done
