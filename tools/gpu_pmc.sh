# rocprofv3 PMC passes for the benchmark kernel (one counter group per pass, no
# sys/runtime tracing).  Writes gpurun_out/pmc/<pass>/... and the counter list.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1; echo "list rc=$?"
grep -o -E "^[[:space:]]*(SQ_INSTS_VALU_[A-Z0-9_]*F64[A-Z0-9_]*|SQ_INSTS_[A-Z_]*|FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE|SQ_WAVE_CYCLES|SQ_BUSY_CYCLES)" $R/gpurun_out/pmc/counters_list.txt | sort -u | head -60
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$name -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/pmc/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"
  if [ $rc -ge 124 ]; then exit 1; fi
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
run flops SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/summary.json --batch 65536 > /dev/null && echo "summary ok"
