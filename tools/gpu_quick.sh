# Wave-kernel parity subset, phase timing and bench (quick iteration loop).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "wave and (infinity or variants or ragged or fresh)" > gpurun_out/pt_wave.log 2>&1; rc=$?
echo "pytest wave rc=$rc"; tail -5 gpurun_out/pt_wave.log
[ $rc -le 1 ] || exit 1
for v in w2; do
  timeout -k 10 120 ./tools/wide_prof_$v tools/inputs_65536.bin 65536 > gpurun_out/wide_prof_$v.log 2>&1; rc=$?
  echo "$v rc=$rc"; cat gpurun_out/wide_prof_$v.log
  [ $rc -eq 0 ] || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --strategy wave > gpurun_out/bench_wave.log 2>&1; rc=$?
echo "bench wave rc=$rc"; tail -1 gpurun_out/bench_wave.log | cut -c1-300
