# quick perf loop: GPU parity tests, bench, diagnostic stamps
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/bench.log 2>&1; rc3=$?
  echo "bench rc=$rc3"; tail -1 gpurun_out/bench.log | cut -c1-400
  if [ $rc3 -eq 0 ] && [ "${DIAG:-0}" = "1" ]; then
    timeout -k 10 300 python tools/diag_stamps.py 65536 > gpurun_out/diag.log 2>&1; echo "diag rc=$?"; tail -9 gpurun_out/diag.log
  fi
fi
