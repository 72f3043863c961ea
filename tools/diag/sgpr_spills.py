"""SGPR spills of one kernel in a gfx950 assembly listing (csrc/*.gfx950.s from
__graft_entry__.kernel_isa): the VGPR lanes that hold spilled SGPRs (targets of v_writelane_b32), the
kernel's loops (backward branches), and for the outermost loop the static count of spill reloads
(v_readlane_b32 from those VGPRs), the distinct spill slots they touch, and what the reloaded SGPR
is used for first (the metric kernel's step loop).

Usage: python tools/diag/sgpr_spills.py FILE.s SYMBOL"""
import collections
import re
import sys


def analyse(path, sym):
    lines = open(path).read().split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[s:e]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    spill = set()
    for l in body:
        m = re.match(r"\s+v_writelane_b32 (v\d+),", l)
        if m:
            spill.add(m.group(1))
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"\s+s_c?branch\w* (\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    a, b = max(loops, key=lambda t: t[1] - t[0])
    seg = body[a:b + 1]
    ins = [x for x in seg if x.startswith("\t") and x.strip() and not x.strip().startswith((".", ";"))]
    reload_re = re.compile(r"\s+v_readlane_b32 (s\d+), (v\d+), (\d+)")
    slots, uses, n_reload, n_rl = collections.Counter(), collections.Counter(), 0, 0
    for i, x in enumerate(seg):
        m = reload_re.match(x)
        if not m:
            continue
        n_rl += 1
        if m.group(2) not in spill:
            continue
        n_reload += 1
        slots[(m.group(2), int(m.group(3)))] += 1
        sreg = m.group(1)
        pat = re.compile(r"\b%s\b|s\[%s:" % (sreg, sreg[1:]))
        for y in seg[i + 1:i + 12]:
            if pat.search(y) and "v_readlane" not in y:
                uses[y.split()[0]] += 1
                break
    return dict(spill_vgprs=sorted(spill), loops=len(loops), outer_loop_lines=(a, b), outer_loop_instructions=len(ins),
                readlanes=n_rl, spill_reloads=n_reload, distinct_slots=len(slots), first_uses=uses.most_common(12))


if __name__ == "__main__":
    r = analyse(sys.argv[1], sys.argv[2])
    for k, v in r.items():
        print("%-24s %s" % (k, v))
