# Round-2 evidence on one GPU: BASELINE configs (bench lines), rocprofv3 kernel stats of
# the headline and the fp32 N=40 config, PMC passes of the headline (traffic, issue mix).
# Results under gpurun_out/final/ (copied to profiles/r2/ by hand).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/final
run() {  # name, args
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $2 > gpurun_out/final/cfg_$1.log 2>&1; rc=$?
  echo "$1 rc=$rc"; [ $rc -eq 0 ] || return 1
  tail -1 gpurun_out/final/cfg_$1.log > gpurun_out/final/cfg_$1.json
  python3 -c "import json; d=json.load(open('gpurun_out/final/cfg_$1.json')); print('  ', d['value'], d['roofline']['kernel_ms'], d['solver'])"
}
run n20 "" && run b4096 "--batch 4096" && run n40 "--horizon 40" && run n40f32 "--horizon 40 --dtype fp32" \
  && run n20f32 "--dtype fp32" && run bic25 "--model bicycle --horizon 25" && run track "--mode track" \
  && run n100 "--batch 4096 --horizon 100" || exit 1
cd /tmp && export TMPDIR=/tmp
prof() {  # name, args
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof_$1 -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 $2 > $R/gpurun_out/final/prof_$1.log 2>&1
  rc=$?; echo "prof $1 rc=$rc"; [ $rc -eq 0 ]
}
prof n20 "" && prof n40f32 "--horizon 40 --dtype fp32" || exit 1
pmc() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$name -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $R/gpurun_out/pmc/$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ]
}
rm -rf $R/gpurun_out/pmc && mkdir -p $R/gpurun_out/pmc
pmc fetch FETCH_SIZE && pmc write WRITE_SIZE \
  && pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  && pmc grbm GRBM_GUI_ACTIVE GRBM_COUNT \
  && pmc flops SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 \
  || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/final/pmc_B65536_N20.json --batch 65536 > /dev/null && echo "summary ok"
