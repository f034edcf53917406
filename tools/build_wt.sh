# Build the kernel-timing tool (tools/wide_time.hip) against the product sources
# (name "base") or a modified copy under variants/<name>/ (diagnostic; not product).
#   bash tools/build_wt.sh base v1 v2 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for v in "$@"; do
  if [ "$v" = base ]; then inc=$R/mpc_ros_amd/csrc; else inc=$R/variants/$v; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -I "$inc" "$R/tools/wide_time.hip" -o "$R/tools/wt_$v" &
done
wait
