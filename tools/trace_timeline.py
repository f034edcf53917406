"""Per-dispatch timeline of a rocprofv3 kernel trace (diagnostic): for the last launch of the
kernel whose name contains ANCHOR (default: the fp32 batch kernel), every dispatch that overlaps
the window from it to the end of the next k_warm_wide batch, in ms relative to its start.

    python tools/trace_timeline.py kernel_trace.csv [ANCHOR]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_solve_wide<0, false, float"
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")),
                  r.get("Queue_Id", r.get("Stream_Id", ""))) for r in rows))
    starts = [e for e in ev if anchor in e[2]]
    if not starts:
        print("no", anchor)
        return
    t0 = starts[-1][0]
    tend = max(e[1] for e in ev if e[0] >= t0 - 50_000_000 and "k_warm_wide" in e[2] and e[0] >= t0) if any(
        "k_warm_wide" in e[2] and e[0] >= t0 for e in ev) else starts[-1][1]
    for s, e, n, g, q in ev:
        if e < t0 - 2_000_000 or s > tend + 1_000_000:
            continue
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:8.3f} ms  grid {g:>8} q {q:>3}  {n[:80]}")


if __name__ == "__main__":
    main()
