set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for b in 256 65536; do
timeout -k 10 120 ./tools/wide_prof_w1 tools/inputs_65536.bin $b > gpurun_out/wide_prof_w1_$b.log 2>&1; rc=$?
echo "rc=$rc"; cat gpurun_out/wide_prof_w1_$b.log
[ $rc -eq 0 ] || exit 1
done
