"""Static per-basic-block opcode classes of one kernel in a hipcc -S dump (diagnostic).

    python tools/isa_blocks.py file.s kernel_substring [min_instr]

Prints each block with its loop nesting (from LLVM's block comments) and instruction classes:
fp64 arithmetic, moves, DPP, readlane/writelane, LDS, scalar, scratch, waitcnt/nop."""
import re
import sys


def classify(op, line):
    if op in ("v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32"):
        return "lane"
    if "_dpp" in op or "dpp" in line.split(op, 1)[1][:0] or " row_" in line or "quad_perm" in line or "wave_sh" in line or "row_half_mirror" in line:
        return "dpp"
    if op.startswith("v_mov") or op.startswith("v_cndmask"):
        return "mov"
    if op.startswith("v_") and "f64" in op:
        return "f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("global_") or op.startswith("buffer_"):
        return "global"
    if op in ("s_waitcnt", "s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(kern) or (kern in l and l.endswith(":") and not l.startswith("\t")))
    blocks, cur = [], None
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", l)
        if m:
            cur = {"name": m.group(1), "cmt": (m.group(2) or "").strip(), "c": {}, "n": 0}
            blocks.append(cur)
            continue
        if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;"):
            if cur is None:
                cur = {"name": "entry", "cmt": "", "c": {}, "n": 0}
                blocks.append(cur)
            op = l.split()[0]
            c = classify(op, l)
            cur["c"][c] = cur["c"].get(c, 0) + 1
            cur["n"] += 1
    keys = ["f64", "valu_other", "mov", "dpp", "lane", "lds", "salu", "wait", "scratch", "global"]
    tot = {k: 0 for k in keys}
    for b in blocks:
        for k in keys:
            tot[k] += b["c"].get(k, 0)
        if b["n"] >= mn:
            d = re.search(r"Depth=(\d+)", b["cmt"])
            h = re.search(r"Header=(\S+)", b["cmt"])
            print(f"{b['name']:>12} n={b['n']:5d} d={d.group(1) if d else '-'} hdr={h.group(1) if h else '-':>8} " +
                  " ".join(f"{k}={b['c'].get(k, 0)}" for k in keys))
    print("total", " ".join(f"{k}={v}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
