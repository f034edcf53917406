"""Inner loops (depth >= 2) of one kernel in a hipcc -S dump, with their instruction classes
(diagnostic: the Riccati stage loop, the systolic recursions, ...).

    python tools/isa_loops.py kernel.s"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
blocks, cur = [], None
for l in lines:
    m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", l)
    if m:
        cur = {"name": m.group(1), "cmt": m.group(2) or "", "n": 0, "ops": []}
        blocks.append(cur)
        continue
    if cur and re.match(r"^\s+;", l) and cur["n"] == 0:
        cur["cmt"] += l
        continue
    if cur and l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;"):
        cur["n"] += 1
        cur["ops"].append(l.split()[0])
loops = {}
for b in blocks:
    d = [int(x) for x in re.findall(r"Depth=(\d+)", b["cmt"])]
    if not d or max(d) < 2:
        continue
    if "Inner Loop Header: Depth=2" in b["cmt"]:
        hdr = b["name"].replace(".LBB", "")
    else:
        hs = re.findall(r"Header=BB(\S+) Depth=2", b["cmt"])
        hdr = hs[-1] if hs else "?"
    loops.setdefault(hdr, []).append(b)
for h, bs in sorted(loops.items(), key=lambda x: -sum(b["n"] for b in x[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    ops = [o for b in bs for o in b["ops"]]
    c = lambda f: sum(1 for o in ops if f(o))  # noqa: E731
    print(h, "blocks", len(bs), "n", len(ops), "valu", c(lambda o: o.startswith("v_")),
          "f64", c(lambda o: o.startswith("v_") and "f64" in o),
          "lane", c(lambda o: o in ("v_readlane_b32", "v_writelane_b32")), "dpp", c(lambda o: "dpp" in o),
          "mov", c(lambda o: o.startswith("v_mov") or o.startswith("v_cndmask")), "lds", c(lambda o: o.startswith("ds_")),
          "salu", c(lambda o: o.startswith("s_") and o not in ("s_waitcnt", "s_nop")), "nop", c(lambda o: o == "s_nop"))
