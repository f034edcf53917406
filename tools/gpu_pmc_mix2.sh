# Instruction-mix PMC pass over the kernel-timing tool of each variant.
#   WT_VARIANTS="base v1" bash tools/gpu_pmc_mix2.sh  -> gpurun_out/pmcwt/<variant>/mix/...
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcwt && cd /tmp && export TMPDIR=/tmp
for v in ${WT_VARIANTS:-base}; do
  for pass in "mix:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VMEM" \
              "mix2:SQ_WAVES SQ_INSTS_SENDMSG SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $R/gpurun_out/pmcwt/$v/$name -- $R/tools/wt_$v $R/tools/inputs_65536.bin /tmp/u0_$v.bin > $R/gpurun_out/pmcwt/$v.$name.log 2>&1
    rc=$?; echo "$v $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmcwt/$v.$name.log; exit 1; fi
  done
done
