set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bicycle or (wave and (infinity or variants))" > gpurun_out/pt_bicycle.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pt_bicycle.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 10 --model bicycle --horizon 25 > gpurun_out/bench_bicycle.log 2>&1; rc=$?
echo "bench bicycle rc=$rc"; tail -1 gpurun_out/bench_bicycle.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200
