# Round-3 final GPU evidence on the current tree: the -m gpu suite, smoke(), the headline
# bench line, and the rocprofv3 kernel statistics of the same bench command.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3f
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3f/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r3f/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/r3f/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3f/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/r3f/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3f/prof -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $R/gpurun_out/r3f/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit 1
f=$(find $R/gpurun_out/r3f/prof -name '*kernel_stats.csv' | head -1); cut -c1-200 "$f" | head -6
