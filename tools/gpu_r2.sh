# Round-2 GPU check: gpu tests, smoke, bench, rocprofv3 kernel stats (PROF names the profile dir).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
echo "host: $(nproc) cpus; $(lscpu | grep 'Model name' | head -1)" > gpurun_out/host.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc2=$?
echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
[ $rc2 -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds ${CPUSEC:-10} > gpurun_out/bench.log 2>&1; rc3=$?
echo "bench rc=$rc3"; tail -2 gpurun_out/bench.log | cut -c1-1500
[ $rc3 -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${PROF:-prof} -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $R/gpurun_out/${PROF:-prof}.log 2>&1; echo "prof rc=$?"
find $R/gpurun_out/${PROF:-prof} -name "*kernel_stats*"
