# VALU instruction mix of k_solve_wide (kernel-timing tool of each variant).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcmix && cd /tmp && export TMPDIR=/tmp
for v in ${WT_VARIANTS:-base}; do
  for pass in "a:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU" \
              "b:SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH" \
              "c:SQ_WAVES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $R/gpurun_out/pmcmix/$v/$name -- $R/tools/wt_$v $R/tools/inputs_65536.bin /tmp/u0_$v.bin > $R/gpurun_out/pmcmix/$v.$name.log 2>&1
    rc=$?; echo "$v $name rc=$rc"
    if [ $rc -ne 0 ]; then exit 1; fi
  done
done
