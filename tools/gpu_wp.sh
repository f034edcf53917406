# Phase timing (exp/wp_<variant>, tools/build_wp.sh) at B = 256 (one wavefront per SIMD) and 65536.
#   WP_VARIANTS="base v1" bash tools/gpu_wp.sh
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wp
for v in ${WP_VARIANTS:-base}; do
  for b in ${WP_BATCHES:-256 65536}; do
    timeout -k 10 120 ./exp/wp_$v exp/inputs_65536.bin $b > gpurun_out/wp/${v}_$b.log 2>&1 || { echo "$v $b failed"; cat gpurun_out/wp/${v}_$b.log; exit 1; }
    echo "== $v B=$b"; cat gpurun_out/wp/${v}_$b.log | head -12
  done
done
