set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
echo "host: $(nproc) cpus; $(lscpu | grep 'Model name' | head -1)" > gpurun_out/host.txt
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc2=$?
  echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
  if [ $rc2 -le 1 ]; then
    timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.log 2>&1; rc3=$?
    echo "bench rc=$rc3"; tail -3 gpurun_out/bench.log
    if [ $rc3 -eq 0 ]; then
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${PROF:-prof} -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $R/gpurun_out/${PROF:-prof}.log 2>&1; echo "prof rc=$?"
      find $R/gpurun_out/${PROF:-prof} -name "*stats*" | head
    fi
  fi
fi
