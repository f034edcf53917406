# Quick GPU step: the kernel-variant experiment (VARS) and a selection of GPU tests (PYK).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
if [ -n "${VARS:-}" ]; then VARS="$VARS" bash tools/gpu_exp.sh || exit 1; fi
if [ -n "${PYK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "$PYK" > gpurun_out/pt_q.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pt_q.log
  [ $rc -le 1 ] || exit 1
fi
