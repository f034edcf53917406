# Round-3 GPU check: the -m gpu suite, smoke(), the headline bench line (kernel time).
#   STEP=tests|smoke|bench (default: all three, in that order)
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/r3/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/r3/pytest_gpu.log
  [ $rc -le 1 ] || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = smoke ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 gpurun_out/r3/smoke.log; [ $rc -eq 0 ] || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 ${BARGS:-} > gpurun_out/r3/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/r3/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit 1
fi
if [ "$STEP" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/prof_${PNAME:-n20} -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 ${BARGS:-} > $R/gpurun_out/r3/prof_${PNAME:-n20}.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit 1
  f=$(find $R/gpurun_out/r3/prof_${PNAME:-n20} -name '*kernel_stats.csv' | head -1); cut -c1-220 "$f" | head -8
fi
