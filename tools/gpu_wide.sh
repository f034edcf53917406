# First GPU check of the one-problem-per-wavefront kernel: parity subset, then bench.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "wave and (infinity or variants or ragged or fresh)" > gpurun_out/pt_wave.log 2>&1; rc=$?
echo "pytest wave rc=$rc"; tail -15 gpurun_out/pt_wave.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --strategy wave > gpurun_out/bench_wave.log 2>&1; rc=$?
echo "bench wave rc=$rc"; tail -2 gpurun_out/bench_wave.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --strategy wave --batch 4096 > gpurun_out/bench_wave4k.log 2>&1; rc=$?
echo "bench wave 4k rc=$rc"; tail -2 gpurun_out/bench_wave4k.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --strategy lane > gpurun_out/bench_lane.log 2>&1; rc=$?
echo "bench lane rc=$rc"; tail -2 gpurun_out/bench_lane.log
