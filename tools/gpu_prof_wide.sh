# Phase timing of the wavefront solver (register-limited variants w1, w2).
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in w1 w2; do
for b in 256 65536; do
  timeout -k 10 120 ./tools/wide_prof_$v tools/inputs_65536.bin $b > gpurun_out/wide_prof_${v}_$b.log 2>&1; rc=$?
  echo "$v B=$b rc=$rc"; cat gpurun_out/wide_prof_${v}_$b.log
  [ $rc -eq 0 ] || exit 1
done
done
