# Run a gpurun command, retrying while the pool has no box (exit code 3) or the call failed on
# the infrastructure side before running; at most ${TRIES:-15} attempts, ${WAIT:-120} s apart.
#   bash tools/gpurun_retry.sh <timeout> '<command>'  > log
T=$1; shift
for i in $(seq 1 ${TRIES:-15}); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > /tmp/gpurun_try.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_try.log; then
    echo "attempt $i: transient (rc=$rc)"; sleep ${WAIT:-120}; continue
  fi
  cat /tmp/gpurun_try.log; echo "gpurun rc=$rc"; exit $rc
done
echo "gave up"; exit 3
