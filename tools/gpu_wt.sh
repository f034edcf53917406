# Time built exp/wt_<variant> binaries on the benchmark inputs (outputs compared to the
# first one); each variant is timed twice, interleaved, to expose drift between runs.
#   WT_VARIANTS="base v1" bash tools/gpu_wt.sh
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
[ -f exp/inputs_65536.bin ] || timeout -k 10 300 python3 tools/make_inputs.py 65536 exp || exit 1
set -- ${WT_VARIANTS:-base}
ref=$1
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v ($pass)"
    timeout -k 10 120 ./exp/wt_$v exp/inputs_65536.bin gpurun_out/wt/$v.bin gpurun_out/wt/$ref.bin || exit 1
  done
done
