# fp32 N = 40 study (tools/fp32_diag.py) on the GPU box: one run per (escalation workers, option set)
#   WORKERS="16 136" OPTS="max_iter=300 max_iter=100" TAG=... bash tools/gpu_fp32opt.sh
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-f32}
mkdir -p $O
for w in ${WORKERS:-16}; do
  for o in ${OPTS:-max_iter=300}; do
    MPCG_ESCALATION_WORKERS=$w timeout -k 10 300 python -u tools/fp32_diag.py 1024 $o > $O/diag_w${w}_$o.log 2>&1; rc=$?
    echo "[workers $w $o] rc=$rc"; grep -E "within|kernel ms" $O/diag_w${w}_$o.log; [ $rc -eq 0 ] || exit 1
  done
done
