# Round-3 (second session) GPU check: the -m gpu suite, smoke(), the headline bench line,
# and the timing tool on the benchmark inputs (exp/wt_* built by tools/build_wt.sh).
#   STEP=tests|smoke|bench|wt|all (default all)
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r3b
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/r3b/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/r3b/pytest_gpu.log
  [ $rc -le 1 ] || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = smoke ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 gpurun_out/r3b/smoke.log; [ $rc -eq 0 ] || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 ${BARGS:-} > gpurun_out/r3b/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/r3b/bench.log | cut -c1-700; [ $rc -eq 0 ] || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = wt ]; then
  WT_VARIANTS="${WT_VARIANTS:-base}" bash tools/gpu_wt.sh || exit 1
fi
