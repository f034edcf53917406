# LDS bank-conflict passes (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, round 6) of the batch
# configurations; summaries under gpurun_out/$TAG/pmc_<cfg>_lds/.
set -u
R=$GRAFT_REPO_ROOT
T=${TAG:-r6p}
cd $R
for c in ${PCFGS:-n20 n40 bic25 n40f32}; do
  case $c in n20) a="";; n40) a="--horizon 40";; bic25) a="--model bicycle --horizon 25";; n40f32) a="--horizon 40 --dtype fp32";; esac
  PTAG=$T PSUF=_${c}_lds PASSES=lds STATS=0 BARGS="$a" bash tools/gpu_pmc.sh || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$T/pmc_${c}_lds/summary.json')); c=d['counters_per_dispatch']; print('$c', {k: round(v/c['SQ_WAVES'],1) for k,v in c.items() if k!='SQ_WAVES'}, 'conflict frac', round(d.get('lds_bank_conflict_frac',-1),4))"
done
