# Round 4, first GPU call: the new instance / overflow / graph tests, the track test without its
# mask, then PC-sampling support on the headline kernel (timing tool).
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_track.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1
echo "pytest rc=$?"
tail -5 gpurun_out/r4a/pytest.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4a/list.txt 2>&1; echo "list rc=$?"
grep -i -A3 "pc.sampl\|host_trap\|stochastic" gpurun_out/r4a/list.txt | head -40
timeout -k 10 120 ./exp/wt_base exp/inputs_65536.bin gpurun_out/r4a/u0.bin > gpurun_out/r4a/wt.log 2>&1; echo "wt rc=$?"; cat gpurun_out/r4a/wt.log
