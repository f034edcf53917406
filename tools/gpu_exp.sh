# Kernel variant experiment: timing (exp/wt_*) and phase split (exp/wp_*) of the variants
# named in VARS (the first is the reference for output comparison).
#   VARS="base v1" bash tools/gpu_exp.sh
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wt gpurun_out/wp
WT_VARIANTS="$VARS" bash tools/gpu_wt.sh > gpurun_out/wt/log.txt 2>&1 || { cat gpurun_out/wt/log.txt; exit 1; }
cat gpurun_out/wt/log.txt
for v in $VARS; do
  if [ -x exp/wp_$v ]; then
    timeout -k 10 120 ./exp/wp_$v exp/inputs_65536.bin 65536 > gpurun_out/wp/${v}.log 2>&1 || { echo "wp $v failed"; cat gpurun_out/wp/${v}.log; exit 1; }
    echo "== wp $v"; head -20 gpurun_out/wp/${v}.log
  fi
done
