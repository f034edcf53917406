# Build the phase-timing tool (tools/wide_prof.hip, 2 waves per SIMD) against the product
# sources (a name without a variants/<name>/ directory) or a modified copy under
# variants/<name>/ (diagnostic; not product); extra flags from WTF_<name> (as build_wt.sh).
#   bash tools/build_wp.sh base v1 v2 ...   -> exp/wp_<name>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/exp"
for v in "$@"; do
  if [ -d "$R/variants/$v" ]; then inc="-I$R/variants/$v"; else inc="-I$R/mpc_ros_amd/csrc -I$R/include"; fi
  eval "X=\${WTF_$v:-}"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -mllvm -disable-promote-alloca-to-lds $X -DWPE=2 $inc "$R/tools/wide_prof.hip" -o "$R/exp/wp_$v" &
done
wait
