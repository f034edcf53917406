set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./tools/wide_prof_w2 tools/inputs_65536.bin 65536 > gpurun_out/wide_prof_tl.log 2>&1; rc=$?
echo "rc=$rc"; cat gpurun_out/wide_prof_tl.log
