# BASELINE configs on one GPU (bench lines under gpurun_out/r3/cfg_*.json) + optional rocprof of one.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
run() {  # name, args
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 $2 > gpurun_out/r3/cfg_$1.log 2>&1; rc=$?
  echo "$1 rc=$rc"; [ $rc -eq 0 ] || return 1
  tail -1 gpurun_out/r3/cfg_$1.log > gpurun_out/r3/cfg_$1.json
  python3 -c "import json; d=json.load(open('gpurun_out/r3/cfg_$1.json')); print('  ', d['value'], d['roofline']['kernel_ms'], d['solver'], d.get('latency_b1'))"
}
for c in ${CFGS:-n20 b4096 n40 n40f32 n20f32 bic25 track}; do case $c in n20) a="";; b4096) a="--batch 4096";; n40) a="--horizon 40";; n40f32) a="--horizon 40 --dtype fp32";; n20f32) a="--dtype fp32";; bic25) a="--model bicycle --horizon 25";; track) a="--mode track";; n100) a="--batch 4096 --horizon 100";; n64) a="--horizon 64";; bic40) a="--model bicycle --horizon 40";; b1024) a="--batch 1024";; lat) a="--cpu-seconds 1";; esac; run $c "$a" || exit 1; done
