# Round-6 final lines: every BASELINE configuration's bench line (cfg_*.json), then the
# rocprofv3 kernel statistics of the headline and of configs[2].  Outputs under gpurun_out/$TAG/.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r6f}
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
TAG=$T STEPS=cfg CFGS="${CFGS:-n20 b4096 lat n40 n40f32 n40f32off n20f32 bic25 track b1024 n64 n100 bic40}" bash tools/gpu_r4.sh || exit 1
TAG=$T STEPS=stats bash tools/gpu_r4.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof32 -- python3 $R/bench.py --horizon 40 --dtype fp32 --steps 10 --warmup 2 --cpu-seconds 0 > $O/prof32.log 2>&1
rc=$?; echo "prof32 rc=$rc"; [ $rc -eq 0 ] || exit 1
f=$(find $O/prof32 -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_n40f32.csv; cut -c1-200 $O/kernel_stats_n40f32.csv | head -8
