"""Basic blocks of one kernel in a gfx950 assembly listing (csrc/*.gfx950.s from
__graft_entry__.kernel_isa): per block the instruction count by class and its branch targets,
and the backward branches (loops).  Usage: python tools/diag/isa_blocks.py FILE.s SYMBOL_SUBSTRING"""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(sym.split()[-1]) or (l.startswith("_Z") and sym in l.split(":")[0] and l.split(":")[0].endswith(sym)))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    if cur is None:
        cur = ["entry", []]
        blocks.append(cur)
    t = l.strip()
    if l.startswith("\t") and t and not t.startswith((".", ";")):
        cur[1].append(t.split(";")[0].strip())
order = {b[0]: i for i, b in enumerate(blocks)}


def cls(op):
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "br"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "s"
    if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
        return "rl"
    if op.startswith("v_"):
        return "v"
    if op.startswith("ds_"):
        return "ds"
    return "m"


for i, (name, ins) in enumerate(blocks):
    c = Counter(cls(x.split()[0]) for x in ins)
    tg = [x.split()[-1] for x in ins if x.startswith(("s_cbranch", "s_branch"))]
    back = [t for t in tg if t in order and order[t] <= i]
    print("%-12s n=%4d v=%3d s=%3d rl=%2d ds=%2d wait=%2d br=%s%s" % (
        name, len(ins), c["v"], c["s"], c["rl"], c["ds"], c["wait"], ",".join(tg),
        "   <-- LOOP back to " + ",".join(back) if back else ""))
