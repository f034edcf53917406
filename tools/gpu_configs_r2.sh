# BASELINE configs on one GPU (bench lines under gpurun_out/cfg_*.json) + optional rocprof of one.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() {  # name, args
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $2 > gpurun_out/cfg_$1.log 2>&1; rc=$?
  echo "$1 rc=$rc"; [ $rc -eq 0 ] || return 1
  tail -1 gpurun_out/cfg_$1.log > gpurun_out/cfg_$1.json
  python3 -c "import json; d=json.load(open('gpurun_out/cfg_$1.json')); print('  ', d['value'], d['roofline']['kernel_ms'], d['solver'])"
}
run n20 "" && run b4096 "--batch 4096" && run n40 "--horizon 40" && run n40f32 "--horizon 40 --dtype fp32" && run n20f32 "--dtype fp32" && run bic25 "--model bicycle --horizon 25" && run track "--mode track"
