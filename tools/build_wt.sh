# Build the kernel-timing tool (tools/wide_time.hip) against the product sources
# (name "base") or a modified copy under variants/<name>/ (diagnostic; not product).
# Binaries go to exp/ (git-ignored, but shipped to the GPU box).
#   bash tools/build_wt.sh base v1 v2 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/exp"
for v in "$@"; do
  if [ "$v" = base ]; then inc="-I$R/mpc_ros_amd/csrc -I$R/include"; else inc="-I$R/variants/$v"; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -mllvm -disable-promote-alloca-to-lds $inc "$R/tools/wide_time.hip" -o "$R/exp/wt_$v" &
done
wait
