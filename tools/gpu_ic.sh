# Instruction-cache PMC of the solve kernel (timing tool) at B = 65,536 (2 wavefronts per SIMD)
# and B = 4,096 (the lone-wavefront instance).  VARS: timing binaries.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-nolicm}; do
  for b in 65536 4096; do
    rm -rf $O/${v}_$b
    timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/${v}_$b -- $R/exp/wt_$v $R/exp/inputs_$b.bin /tmp/o_$v.bin > $O/${v}_$b.log 2>&1
    rc=$?; echo "$v $b rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/${v}_$b.log; exit 1; }
    cd $R && python3 - $O/${v}_$b <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/*/*_counter_collection.csv")[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "k_solve_wide" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = sorted(per, key=int)[-1]
print({k: int(v) for k, v in per[d].items()})
PY
    cd /tmp
  done
done
