# The fp32 configuration's escalation workers (round 6): the fp32 GPU tests, configs[2]'s bench
# lines (two-phase, fp32 alone, N = 20 fp32) and the iteration-limit sweep.  Outputs under
# gpurun_out/$TAG/.
set -u
O=gpurun_out/${TAG:-r6m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_headline.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 "$@" > $O/b.log 2>&1 || { tail -3 $O/b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b.log').read().strip().split(chr(10))[-1]); print(sys.argv[1:], round(d['value']), round(d['roofline']['kernel_ms'],3), d['solver']['iters_mean'], d['solver']['status_counts'], d['solver'].get('fp64_phase'))" "$@"
}
run --horizon 40 --dtype fp32
run --horizon 40 --dtype fp32 --restoration off
run --dtype fp32
timeout -k 10 300 python -u tools/fp32_maxiter_probe.py 80,60,100,300 > $O/maxiter.log 2>&1; echo "probe rc=$?"; tail -4 $O/maxiter.log
