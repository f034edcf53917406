set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_track.py -x -q -m gpu > gpurun_out/pt_track.log 2>&1; rc=$?
echo "pytest track rc=$rc"; tail -15 gpurun_out/pt_track.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --mode track > gpurun_out/bench_track.log 2>&1; rc=$?
echo "bench track rc=$rc"; tail -1 gpurun_out/bench_track.log | cut -c1-260
