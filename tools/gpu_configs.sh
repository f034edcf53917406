# Bench lines for the other BASELINE configs (documentation): B=4096 (configs[1]),
# N=40 (configs[2], fp64), lane strategy, track mode.
set -u
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/configs
run() { name=$1; shift; timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err; rc=$?; echo "$name rc=$rc"; tail -1 gpurun_out/configs/$name.json | cut -c1-150; [ $rc -eq 0 ] || exit 1; }
run b4096 --batch 4096 --steps 10 --warmup 2
run b65536_n40 --horizon 40 --steps 3 --warmup 1
run b16384 --batch 16384 --steps 5 --warmup 1
run lane --strategy lane --steps 2 --warmup 1
run track --mode track --steps 5 --warmup 1
run b4096_cpu --batch 4096 --steps 10 --warmup 2 --cpu-seconds 10
run bicycle_n25 --model bicycle --horizon 25 --steps 3 --warmup 1
