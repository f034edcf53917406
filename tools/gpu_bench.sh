# Quick GPU bench of the current build (no CPU baseline), optional extra args in BARGS.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 ${BARGS:-} > gpurun_out/bench_q.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['solver'])"
