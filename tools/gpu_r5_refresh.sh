# Round-5 evidence refresh on the final build (kernels unchanged since tools/gpu_r5_final.sh, whose
# PMC summaries the bench lines keep citing): the headline bench line, every configuration's
# line, the kernel statistics of the headline and of configs[2] (both phases).  gpurun_out/$TAG/.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r5g}
cd $R
TAG=$T STEPS="bench" bash tools/gpu_r5.sh || exit 1
TAG=$T STEPS=cfg CFGS="${CFGS:-n20 b4096 lat n40 n40f32 n40f32off n20f32 bic25 track b1024 n64 n100 bic40}" bash tools/gpu_r4.sh || exit 1
TAG=$T STEPS="stats" bash tools/gpu_r5.sh || exit 1
O=$R/gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof40 -- python3 $R/bench.py --horizon 40 --dtype fp32 --steps 10 --warmup 2 --cpu-seconds 0 > $O/prof40.log 2>&1
rc=$?; echo "prof40 rc=$rc"; [ $rc -eq 0 ] || exit 1
f=$(find $O/prof40 -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_N40_fp32.csv; cut -c1-150 $O/kernel_stats_N40_fp32.csv | head -5
