# Round-5 GPU evidence: the -m gpu suite, smoke(), the headline bench line, the BASELINE
# configurations' bench lines, and WRITE_SIZE / FETCH_SIZE passes of the batch configurations.
# Outputs under gpurun_out/$TAG/ (default r5).  STEPS="tests smoke bench cfg pmc" selects parts.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r5}
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
for s in ${STEPS:-tests smoke bench cfg pmc}; do
case $s in
tests)
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1 ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit 1 ;;
bench)
  timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit 1 ;;
cfg)
  TAG=$T STEPS=cfg bash tools/gpu_r4.sh || exit 1 ;;
pmc)
  for c in ${PCFGS:-n20 n40 bic25 n40f32 b4096}; do
    b=65536
    case $c in n20) a="";; n40) a="--horizon 40";; bic25) a="--model bicycle --horizon 25";;
      n40f32) a="--horizon 40 --dtype fp32";; b4096) a="--batch 4096"; b=4096;; esac
    PTAG=$T PSUF=_$c PBATCH=$b PASSES="${PPASSES:-fetch write sq grbm flops}" STATS=0 BARGS="$a" bash tools/gpu_pmc.sh || exit 1
  done ;;
stats)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --steps 20 --warmup 2 --cpu-seconds 0 > $O/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit 1
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats.csv; cut -c1-150 $O/kernel_stats.csv | head -4; cd $R ;;
esac
done
