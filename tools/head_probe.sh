# Diagnostic (a build with MPCG_EXTRA_CFLAGS=-DMPCG_HEAD_ENV): the fp32 configuration's time against
# the head's share of the batch (MPCG_HEAD_DIV: B / div problems; 0: no head).  gpurun_out/head_probe.log
set -u
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/head_probe.log
: > $O
for d in ${DIVS:-0 4096 2048 1024 512 256}; do
  for a in "--horizon 40" ""; do
    MPCG_HEAD_DIV=$d timeout -k 10 120 python3 bench.py $a --dtype fp32 --steps 10 --warmup 2 --cpu-seconds 0 > /tmp/hp.log 2>&1 || { echo "div $d failed" >> $O; tail -5 /tmp/hp.log >> $O; exit 1; }
    tail -1 /tmp/hp.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('div', '$d', 'N', d['config'].get('horizon', d['config']), round(d['ms_per_step'],3), d['solver'].get('fp64_phase'))" >> $O
  done
done
