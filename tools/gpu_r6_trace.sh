# Kernel timeline of configs[2] (diagnostic): rocprofv3 kernel trace of a short bench run, then the
# per-dispatch start / end of every kernel relative to each fp32 batch launch.  gpurun_out/$TAG/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r6n}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 $R/bench.py --horizon 40 --dtype fp32 --steps 2 --warmup 1 --cpu-seconds 0 ${BARGS:-} > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit 1
cd $R && python3 tools/trace_timeline.py $(find $O/trace -name '*kernel_trace.csv' | head -1)
