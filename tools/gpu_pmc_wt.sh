# PMC passes (LDS / issue counters) over the kernel-timing tool of each variant:
#   WT_VARIANTS="base v1" bash tools/gpu_pmc_wt.sh  -> gpurun_out/pmcwt/<variant>/<pass>/...
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcwt && cd /tmp && export TMPDIR=/tmp
for v in ${WT_VARIANTS:-base}; do
  for pass in "lds:SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" \
              "ldsw:SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL" \
              "issue:SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
              "misc:SQ_WAVES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $R/gpurun_out/pmcwt/$v/$name -- $R/tools/wt_$v $R/tools/inputs_65536.bin /tmp/u0_$v.bin > $R/gpurun_out/pmcwt/$v.$name.log 2>&1
    rc=$?; echo "$v $name rc=$rc"
    if [ $rc -ne 0 ]; then exit 1; fi
  done
done
