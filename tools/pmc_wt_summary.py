"""Per-dispatch PMC counters of k_solve_wide for each variant (tools/gpu_pmc_wt.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcwt"
for v in sorted(os.listdir(root)):
    d = os.path.join(root, v)
    if not os.path.isdir(d):
        continue
    c, t = load(d)
    w = c.get("SQ_WAVES", 1.0)
    print(f"== {v}  dispatch {t * 1e3 if t else 0:.3f} ms")
    for k in sorted(c):
        print(f"  {k:28s} {c[k]:16.4g}  per wave {c[k] / w:12.1f}")
