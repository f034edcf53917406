# Diagnostic: the headline, configs[1] and B = 1 with the library as built (e.g. a build with
# MPCG_EXTRA_CFLAGS compiler flags; export the same MPCG_EXTRA_CFLAGS here).  Output: $1.log
set -u
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-flags}
mkdir -p $(dirname $O)
{
timeout -k 10 120 python3 bench.py --steps 40 --warmup 3 --cpu-seconds 0 | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('headline', round(d['ms_per_step'],3), 'ms')" &&
timeout -k 10 120 python3 bench.py --batch 4096 --steps 40 --warmup 3 --cpu-seconds 0 | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('b4096', round(d['ms_per_step'],3), 'ms')" &&
timeout -k 10 60 python3 tools/lat_b1.py
} > $O.log 2>&1
