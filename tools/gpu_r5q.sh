# quick check: headline + BASELINE configs timing, WRITE_SIZE of the batch configurations
set -u
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r5q} STEPS=cfg CFGS="${CFGS:-n20 n40 bic25 n40f32}" bash tools/gpu_r4.sh || exit 1
[ "${PMC:-1}" = 1 ] || exit 0
TAG=${TAG:-r5q} STEPS=pmc PPASSES="write fetch" bash tools/gpu_r5.sh || exit 1
