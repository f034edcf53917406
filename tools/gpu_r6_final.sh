# Round-6 evidence in one call: PMC passes of every batch configuration (summaries copied to
# the names bench.py reads its roofline traffic from), then the headline bench line, every
# BASELINE configuration's line, and the rocprofv3 kernel statistics of the headline.
# Outputs under gpurun_out/$TAG/ (default r6f); copy profiles/r6/pmc_*.json back with
# tools/pmc_to_profiles.py gpurun_out/$TAG.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r6f}
cd $R
TAG=$T STEPS=pmc bash tools/gpu_r5.sh || exit 1
PTAG=$T PSUF=_n20valu PASSES=valu STATS=0 BARGS="" bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_to_profiles.py gpurun_out/$T || exit 1
TAG=$T STEPS="bench" bash tools/gpu_r5.sh || exit 1
TAG=$T STEPS=cfg CFGS="${CFGS:-n20 b4096 lat n40 n40f32 n40f32off n20f32 bic25 track b1024 n64 n100 bic40}" bash tools/gpu_r4.sh || exit 1
TAG=$T STEPS="stats" bash tools/gpu_r5.sh || exit 1
