# Timing of exp/wt_* variants with options: "name[:ENV=val]" entries in WT_RUNS.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt
[ -f exp/inputs_65536.bin ] || timeout -k 10 300 python3 tools/make_inputs.py 65536 exp || exit 1
ref=""
for pass in 1 2; do
  for run in ${WT_RUNS}; do
    v=${run%%:*}; envs=""; [ "$run" != "$v" ] && envs=${run#*:}
    [ -z "$ref" ] && ref=$v
    echo "== $run ($pass)"
    env $envs timeout -k 10 120 ./exp/wt_$v exp/inputs_65536.bin gpurun_out/wt/$v.bin gpurun_out/wt/$ref.bin || exit 1
  done
done
