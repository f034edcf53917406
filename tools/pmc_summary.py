"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) of the benchmark kernel into
profiles/<name>.json, which bench.py reads for roofline.traffic and the FP64-VALU
figures.

    python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_B65536_N20.json --batch 65536

Counters are per dispatch of mpcg::k_solve_wide (one solve of the whole batch).
FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters over the L2's
memory-side requests; MI355X_MICROARCH.md §HBM: Infinity-Cache hits are counted,
FETCH_SIZE is calibrated only for 16-B-per-lane streaming reads -- this kernel's
global reads are the 80-B-per-problem inputs and scratch (spill) traffic, so the
figure is reported raw).  SQ_WAVE_CYCLES / SQ_ACTIVE_INST_ANY / SQ_WAIT_* count
quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def load(root: str, kernel: str = "k_solve_wide"):
    """Counters averaged over the dispatches of the batch kernel: of the instances whose name
    contains `kernel`, the one with the most GPU time in the pass (configs[2] also launches
    the fp64 solver on its 64-problem head, which must not be averaged in)."""
    vals = collections.defaultdict(list)
    times = []
    files = {}
    for f in glob.glob(os.path.join(root, "*", "*", "*_counter_collection.csv")):
        d = os.path.dirname(os.path.dirname(f))  # one pass per directory: its newest file
        if d not in files or os.path.getmtime(f) > os.path.getmtime(files[d]):
            files[d] = f
    for f in sorted(files.values()):
        per = collections.defaultdict(float)
        dur = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if kernel not in name:
                continue
            per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            dur[name][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        if not dur:
            continue
        main_name = max(dur, key=lambda n: sum(dur[n].values()))
        times.extend(dur[main_name].values())
        for (n, d, c), v in per.items():
            if n == main_name:
                vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}, (sum(times) / len(times) if times else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out")
    ap.add_argument("--batch", type=int, default=65536)
    a = ap.parse_args()
    c, t = load(a.root)
    B = a.batch
    out = {"kernel": "mpcg::k_solve_wide", "batch": B, "counters_per_dispatch": c, "dispatch_s": t}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["fetch_bytes"] = c["FETCH_SIZE"] * 1024
        out["write_bytes"] = c["WRITE_SIZE"] * 1024
        # MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the bytes of a wide
        # streaming read -- doubled here as the guide prescribes (this kernel's reads are
        # narrower; the correction is the guide's, uncalibrated for them)
        out["fetch_bytes_corrected"] = 2 * out["fetch_bytes"]
        out["hbm_bytes_per_launch"] = out["fetch_bytes_corrected"] + out["write_bytes"]
    if "SQ_WAVES" in c:
        w = c["SQ_WAVES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if k in c:
                out[k.lower() + "_per_solve"] = c[k] / w
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            out["wave_cycles_per_solve"] = 4 * wc / w
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if k in c:
                    out[k.lower() + "_frac"] = c[k] / wc
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        # (the guide: BANK_CONFLICT = the extra LDS cycles, IDX_ACTIVE = all LDS-array cycles)
        out["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "GRBM_GUI_ACTIVE" in c and t:
        out["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
    if "SQ_INSTS_VALU_FLOPS_FP64" in c:
        # the FLOPS counters count per wave-instruction (ADD + MUL + 2 FMA reproduces them,
        # measured): physical lane FLOPs = x 64 lanes (idle and replicated lanes included)
        wave = c["SQ_INSTS_VALU_FLOPS_FP64"] + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)
        out["fp64_wave_flops_per_solve"] = wave / B
        out["fp64_flops_per_launch"] = 64 * wave
        out["fp64_flops_per_solve"] = 64 * wave / B
        for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"):
            if k in c:
                out[k.lower() + "_per_solve"] = c[k] / B
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
