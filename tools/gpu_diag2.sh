set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 python tools/diag_stamps.py 65536 > gpurun_out/diag_noinline.log 2>&1; echo "diag rc=$?"; tail -10 gpurun_out/diag_noinline.log
DIAG_FLAGS=-DMPCG_INLINE_PASSES timeout -k 10 300 python tools/diag_stamps.py 65536 > gpurun_out/diag_inline.log 2>&1; echo "diag rc=$?"; tail -10 gpurun_out/diag_inline.log
