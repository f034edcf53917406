# rocprofv3 PMC passes of the headline bench kernel (one counter group per pass, no
# sys/runtime tracing) and the kernel-trace statistics; summaries under gpurun_out/$PTAG/ (default r4).
#   BARGS: extra bench.py arguments (default: the headline configuration)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PTAG:-r4}/pmc${PSUF:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 ${BARGS:-} > $O/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"
  [ $rc -eq 0 ] || exit 1
}
P=${PASSES:-fetch write sq grbm flops}
for p in $P; do
  case $p in
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    sq) run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY ;;
    grbm) run grbm GRBM_GUI_ACTIVE GRBM_COUNT ;;
    flops) run flops SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 ;;
    valu) run valu SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 ;;
    lds) run lds SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL ;;
  esac
done
cd $R && python3 tools/pmc_summary.py $O $O/summary.json --batch ${PBATCH:-65536} > /dev/null && echo "summary ok"
[ "${STATS:-1}" = 1 ] || exit 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 ${BARGS:-} > $O/stats.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit 1
f=$(find $O/stats -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; cut -c1-200 $O/kernel_stats.csv | head -6
