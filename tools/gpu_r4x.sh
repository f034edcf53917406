# Round 4 measurement bundle: the headline PMC summary (tools/gpu_pmc.sh passes), instruction-
# cache counters (tools/gpu_ic.sh) and compiler-flag variants of the timing tool.
set -u
R=$GRAFT_REPO_ROOT
cd $R
PTAG=r4 STATS=0 PASSES="fetch write sq grbm flops" bash tools/gpu_pmc.sh || exit 1
VARS=base bash tools/gpu_ic.sh || exit 1
WT_VARIANTS="${XV:-base milp iilp mmc trk}" bash tools/gpu_wt3.sh || exit 1
