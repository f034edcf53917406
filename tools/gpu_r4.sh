# Round-4 GPU evidence on the current tree: the -m gpu suite, smoke(), the headline bench
# line, BASELINE configurations (bench lines under gpurun_out/$TAG/cfg_*.json), rocprofv3
# kernel statistics of the headline.  STEPS="tests smoke bench cfg stats" selects parts.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r4}
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
for s in ${STEPS:-tests smoke bench cfg stats}; do
case $s in
tests)
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  # (rc 1: test failures -- the measurements still run; anything else -- a fault, an abort,
  # a time limit -- ends the call)
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1 ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 1 ;;
bench)
  timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit 1 ;;
cfg)
  for c in ${CFGS:-n20 b4096 lat n40 n40f32 n40f32r n20f32 bic25 track}; do
    case $c in n20) a="";; b4096) a="--batch 4096";; n40) a="--horizon 40";; n40f32) a="--horizon 40 --dtype fp32";;
      n40f32r) a="--horizon 40 --dtype fp32 --restoration on";; n20f32) a="--dtype fp32";; bic25) a="--model bicycle --horizon 25";;
      track) a="--mode track";; n100) a="--batch 4096 --horizon 100";; n64) a="--horizon 64";; bic40) a="--model bicycle --horizon 40";;
      b1024) a="--batch 1024";; lat) a="--batch 4096 --cpu-seconds 1";; n40f32off) a="--horizon 40 --dtype fp32 --restoration off";; esac
    timeout -k 10 300 python bench.py --steps ${CSTEPS:-10} --warmup 2 --cpu-seconds 0 $a > $O/cfg_$c.log 2>&1; rc=$?
    [ "$c" = lat ] && { timeout -k 10 300 python bench.py --steps 5 --warmup 1 $a > $O/cfg_$c.log 2>&1; rc=$?; }
    echo "$c rc=$rc"; [ $rc -eq 0 ] || exit 1
    tail -1 $O/cfg_$c.log > $O/cfg_$c.json
    python3 -c "import json; d=json.load(open('$O/cfg_$c.json')); print('  ', round(d['value']), round(d['roofline']['kernel_ms'],3), d['roofline']['kernel'], d['solver']['iters_mean'], d['solver']['status_counts'], d['solver']['restoration'], d['solver'].get('fp64_phase'), d.get('latency_b1'))"
  done ;;
stats)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 2 --cpu-seconds 0 > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit 1
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; cut -c1-200 $O/kernel_stats.csv | head -6; cd $R ;;
esac
done
