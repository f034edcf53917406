"""Static opcode census of one kernel in a hipcc -S dump (diagnostic): VALU instructions by class,
and how many of the lane reads / writes are the register allocator's SGPR spills (v_writelane into,
v_readlane out of, the VGPRs that hold spilled SGPRs) rather than the solver's own broadcasts.

    hipcc -S --offload-arch=gfx950 --cuda-device-only -O3 ... -DMPCG_INST=0 mpcg_wide_inst.hip -o inst0.s
    python tools/isa_census.py inst0.s _ZN4mpcg12k_solve_wideILi0ELb1EdLi1ELb1ELi2EEEvNS_8WideArgsE

Static counts: the solver's state machine is irreducible control flow (no natural loop around
it), so the dump carries no execution frequencies; the dynamic totals are the PMC counters'."""
import collections
import re
import sys


def kernel_lines(path, sym):
    out, on = [], False
    for line in open(path):
        if line.startswith(sym + ":"):
            on = True
            continue
        if on and (line.startswith(".Lfunc_end") or (line[:1] not in ("\t", ".", " ", ";", "\n") and line.endswith(":\n")
                                                       and not line.startswith(".L"))):
            break
        if on:
            out.append(line.rstrip("\n"))
    return out


def vclass(op, line):
    if op in ("v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32"):
        return op
    if "row_" in line or "quad_perm" in line or "wave_sh" in line or "row_bcast" in line or "_dpp" in op:
        return "dpp"
    if op.startswith("v_mov_b64"):
        return "v_mov_b64"
    if op.startswith("v_mov"):
        return "v_mov_b32"
    if op.startswith("v_cndmask"):
        return "v_cndmask"
    if op.startswith("v_cmp"):
        return "v_cmp (" + ("f64" if "f64" in op else "other") + ")"
    if "f64" in op:
        return "fp64 arithmetic"
    if "f32" in op or "f16" in op:
        return "fp32/fp16"
    return "integer / bit / other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sym)
    cls = collections.Counter()
    spill_vgprs = set()
    writes = []
    reads = []
    other = collections.Counter()
    for line in lines:
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cls[vclass(op, s)] += 1
            if op == "v_writelane_b32":
                m = re.match(r"v_writelane_b32\s+(v\d+),", s)
                if m:
                    spill_vgprs.add(m.group(1))
                    writes.append(m.group(1))
            elif op == "v_readlane_b32":
                m = re.match(r"v_readlane_b32\s+s\S+,\s*(v\d+),", s)
                if m:
                    reads.append(m.group(1))
        elif op.startswith("ds_"):
            other["LDS"] += 1
        elif op.startswith(("global_", "buffer_")):
            other["global"] += 1
        elif op.startswith("scratch_"):
            other["scratch"] += 1
        elif op.startswith("s_"):
            other["SALU / branch / wait"] += 1
    total = sum(cls.values())
    print(f"{sym}: {total} VALU instructions (static)")
    for k, v in cls.most_common():
        print(f"  {k:28s} {v:6d}  {100.0 * v / total:5.1f} %")
    rl_spill = sum(1 for r in reads if r in spill_vgprs)
    print(f"  SGPR spill VGPRs {sorted(spill_vgprs)}: {len(writes)} spill writes, {rl_spill} reloads; "
          f"{len(reads) - rl_spill} other v_readlane")
    for k, v in other.items():
        print(f"  {k:28s} {v:6d}")


if __name__ == "__main__":
    main()
