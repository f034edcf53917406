# Round 4 full GPU pass in one call: fp32 diagnosis, the -m gpu suite, smoke, bench, BASELINE
# configurations, kernel statistics (tools/gpu_r4.sh), then the measurement bundle
# (tools/gpu_r4x.sh: PMC summary, instruction cache, compiler-flag variants).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/${TAG:-r4}
timeout -k 10 240 python tools/fp32_diag.py 4096 > gpurun_out/${TAG:-r4}/fp32diag.log 2>&1; echo "fp32diag rc=$?"
TAG=${TAG:-r4} bash tools/gpu_r4.sh || exit 1
bash tools/gpu_r4x.sh || exit 1
