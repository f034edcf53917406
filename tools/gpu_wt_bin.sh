# Time wtbin/wt_<variant> binaries (tools/build_wt.sh, copied to wtbin/, which travels to the GPU
# box) on wtbin/inputs_65536.bin, three times interleaved, outputs compared with the first variant's.
#   WT_VARIANTS="base v1" bash tools/gpu_wt_bin.sh
set -u
O=gpurun_out/${TAG:-wtb}
mkdir -p $O
set -- ${WT_VARIANTS:-base}
ref=$1
for pass in 1 2 3; do
  for v in "$@"; do
    echo "== $v ($pass)"
    timeout -k 10 120 ./wtbin/wt_$v wtbin/inputs_65536.bin $O/$v.bin $O/$ref.bin || exit 1
  done
done
