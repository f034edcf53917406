# Build the kernel-timing tool (tools/wide_time.hip) against the product sources (name
# "base", or any name without a variants/<name>/ directory) or a modified copy under
# variants/<name>/ (diagnostic; not product).  Extra compiler flags for a variant: the
# environment variable WTF_<name> (e.g. WTF_nolicm="-mllvm -disable-machine-licm").
# Only the benchmark configuration's instance groups are linked (MPCG_HEADLINE_ONLY:
# mpcg_wide_inst.hip groups 0 and 1).  Binaries go to exp/ (git-ignored, shipped to the
# GPU box).
#   bash tools/build_wt.sh base v1 v2 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/exp/obj"
F="--offload-arch=gfx950 -O3 -std=c++17 -w -mllvm -disable-promote-alloca-to-lds -mllvm -disable-machine-licm"
for v in "$@"; do
  if [ -d "$R/variants/$v" ]; then inc="-I$R/variants/$v"; d="$R/variants/$v"; else inc="-I$R/mpc_ros_amd/csrc -I$R/include"; d="$R/mpc_ros_amd/csrc"; fi
  eval "X=\${WTF_$v:-}"
  for g in 0 1; do
    /opt/rocm/bin/hipcc -c $F $X $inc -DMPCG_INST=$g "$d/mpcg_wide_inst.hip" -o "$R/exp/obj/${v}_inst$g.o" &
  done
  /opt/rocm/bin/hipcc -c $F $X $inc -DMPCG_HEADLINE_ONLY "$R/tools/wide_time.hip" -o "$R/exp/obj/${v}_wt.o" &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 "$R/exp/obj/${v}_wt.o" "$R/exp/obj/${v}_inst0.o" "$R/exp/obj/${v}_inst1.o" -o "$R/exp/wt_$v"
done
