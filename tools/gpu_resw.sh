# resume-worker count study: bench lines per (config, MPCG_RESUME_WORKERS)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-resw}
mkdir -p $O
for c in ${CFGS:-n40 bic25}; do
  case $c in n20) a="";; n40) a="--horizon 40";; bic25) a="--model bicycle --horizon 25";; bic40) a="--model bicycle --horizon 40";; n64) a="--horizon 64";; esac
  for w in ${WORKERS:-3 8 16}; do
    MPCG_RESUME_WORKERS=$w timeout -k 10 300 python bench.py --steps ${CSTEPS:-6} --warmup 2 --cpu-seconds 0 $a > $O/${c}_w$w.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$c w$w rc=$rc"; exit 1; }
    tail -1 $O/${c}_w$w.log > $O/${c}_w$w.json
    python3 -c "import json; d=json.load(open('$O/${c}_w$w.json')); print('$c w$w', round(d['value']), round(d['ms_per_step'],2))"
  done
done
