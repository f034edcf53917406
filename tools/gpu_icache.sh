# Instruction-cache and issue PMC of the solve kernel for the timing binaries named in VARS
# (one counter group per rocprofv3 pass, kernel trace only).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/ic
cd /tmp && export TMPDIR=/tmp
for v in $VARS; do
  i=0
  for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ" "SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/ic/${v}_$i -- $R/exp/wt_$v $R/exp/inputs_65536.bin /tmp/o_$v.bin > $R/gpurun_out/ic/${v}_$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    [ $rc -eq 0 ] || exit 1
  done
done
