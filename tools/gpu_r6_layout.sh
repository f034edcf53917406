# The compact layout (round 6) on the GPU: the parity suites, then the bench lines of the
# configurations it touches (N = 40 fp64, configs[2] and its fp32 phase, N = 64) and the headline.
# Outputs under gpurun_out/$TAG/.
set -u
O=gpurun_out/${TAG:-r6i}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_fp32.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 "$@" > $O/b.log 2>&1 || { tail -3 $O/b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b.log').read().strip().split(chr(10))[-1]); print(sys.argv[1:], round(d['value']), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel'], d['solver']['iters_mean'])" "$@"
}
run --horizon 40
run --horizon 40 --dtype fp32
run --horizon 40 --dtype fp32 --restoration off
run --horizon 64
run
