# Round-5 first GPU pass: the -m gpu suite, the BASELINE configurations' bench lines, and the
# WRITE_SIZE pass of the four batch configurations (slot LIFO).  Outputs under gpurun_out/r5a/.
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=r5a STEPS="tests cfg" CFGS="n20 b4096 n40 n40f32 bic25" bash tools/gpu_r4.sh || exit 1
for c in n20:"" n40:"--horizon 40" bic25:"--model bicycle --horizon 25" n40f32:"--horizon 40 --dtype fp32"; do
  n=${c%%:*}; a=${c#*:}
  PTAG=r5a PSUF=_$n PASSES="write fetch" STATS=0 BARGS="$a" bash tools/gpu_pmc.sh || exit 1
done
