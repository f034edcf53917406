# Round 4: PC sampling of the headline kernel (timing tool) and WRITE_SIZE of variants.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base noacc; do
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_$v -- $R/exp/wt_$v $R/exp/inputs_65536.bin $O/u0_$v.bin > $O/w_$v.log 2>&1
  echo "write $v rc=$?"
done
timeout -s KILL 90 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10 --output-format csv -d $O/pcs -- $R/exp/wt_base $R/exp/inputs_65536.bin $O/u0_pcs.bin > $O/pcs.log 2>&1
echo "pcs host_trap rc=$?"
tail -5 $O/pcs.log
find $O/pcs -type f | head
