# Time exp/wt_<variant> binaries on the benchmark inputs, twice interleaved (outputs compared
# to the first variant's); with WT_PMC=1 also an SQ-instruction pass and a WRITE_SIZE pass per
# variant (tools/pmc_brief.py summarises them).
#   WT_VARIANTS="base v1" bash tools/gpu_wt3.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wt3
cd $R && mkdir -p $O
set -- ${WT_VARIANTS:-base}
ref=$1
for pass in 1 2; do
  for v in "$@"; do
    echo "== $v ($pass)"
    timeout -k 10 120 ./exp/wt_$v exp/inputs_65536.bin $O/$v.bin $O/$ref.bin || exit 1
  done
done
[ "${WT_PMC:-0}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  rm -rf $O/sq_$v $O/w_$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq_$v -- $R/exp/wt_$v $R/exp/inputs_65536.bin $O/p_$v.bin > $O/sq_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_$v -- $R/exp/wt_$v $R/exp/inputs_65536.bin $O/p_$v.bin > $O/w_$v.log 2>&1 || exit 1
done
cd $R && python3 tools/pmc_brief.py $O "$@"
