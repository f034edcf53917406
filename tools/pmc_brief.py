"""Per-solve SQ counters and per-launch WRITE_SIZE of rocprofv3 --pmc runs of the timing tool
(tools/gpu_wt3.sh WT_PMC=1): one line per variant (diagnostic).

    python tools/pmc_brief.py gpurun_out/wt3 v1 v2 ..."""
import collections
import csv
import glob
import os
import sys

root, B = sys.argv[1], 65536
for v in sys.argv[2:]:
    out = {}
    for kind in ("sq", "w"):
        fs = glob.glob(os.path.join(root, f"{kind}_{v}", "*", "*_counter_collection.csv"))
        if not fs:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(fs[0])):
            if "k_solve_wide" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        ds = sorted(per, key=int)[1:] or sorted(per, key=int)
        for c in per[ds[0]]:
            x = sum(per[d][c] for d in ds) / len(ds)
            out[c] = round(x / B, 1) if c.startswith("SQ_INSTS") else (round(x / 1024, 1) if c == "WRITE_SIZE" else x)
    print(v, out)
