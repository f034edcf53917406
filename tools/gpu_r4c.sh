# Phase profile of the nolicm build, and SQ / WRITE_SIZE counters of base vs nolicm (timing tool).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
cd $R
for b in 256 65536; do
  timeout -k 10 120 ./exp/wp_nolicm exp/inputs_65536.bin $b > $O/wp_nolicm_$b.log 2>&1 || { cat $O/wp_nolicm_$b.log; exit 1; }
  cat $O/wp_nolicm_$b.log
done
cd /tmp && export TMPDIR=/tmp
for v in base nolicm; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/sq_$v -- $R/exp/wt_$v $R/exp/inputs_65536.bin $O/u_$v.bin > $O/sq_$v.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_$v -- $R/exp/wt_$v $R/exp/inputs_65536.bin $O/u_$v.bin > $O/w_$v.log 2>&1 || exit 1
  echo "pmc $v ok"
done
