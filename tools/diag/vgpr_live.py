"""Approximate VGPR liveness over one kernel of a gfx950 assembly listing: per instruction the
number of live VGPRs (backward dataflow over the basic blocks, every VALU / DS / memory def kills,
so partial-exec writes under-count), then the program points with the most live VGPRs and the
instructions that last defined the registers live there.  Used to find where the M <= 16 class's
register peak is.  Usage: python tools/diag/vgpr_live.py FILE.s SYMBOL_SUBSTRING [TOP]"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 5
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


# blocks: (label, [(lineno, op, defs, uses)])
blocks, cur = [], None
for ln in range(start, end):
    l = lines[ln]
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        cur = [m.group(1), []]
        blocks.append(cur)
        continue
    t = l.strip()
    if cur is None:
        cur = ["entry", []]
        blocks.append(cur)
    if not l.startswith("\t") or not t or t.startswith((".", ";")):
        continue
    t = t.split(";")[0].strip()
    op = t.split()[0]
    rest = t[len(op):]
    ops = [o.strip() for o in rest.split(",")]
    defs, uses = set(), set()
    if op.startswith(("s_", "buffer_store", "global_store", "scratch_store", "ds_write", "flat_store")) \
            or op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) or op in ("ds_nop",):
        uses = regs(rest)
    elif op.startswith(("v_", "ds_", "global_load", "buffer_load", "scratch_load", "flat_load")):
        defs = regs(ops[0]) if ops else set()
        uses = regs(",".join(ops[1:]))
        if op.startswith(("v_fmac", "v_mac", "v_writelane")) or "_dpp" in op:
            uses |= defs  # accumulators / lane writes / DPP keep the old value
    cur[1].append((ln, op, defs, uses))

label_ix = {b[0]: k for k, b in enumerate(blocks)}
succ = []
for k, (lab, ins) in enumerate(blocks):
    s = []
    last = ins[-1][1] if ins else ""
    if ins:
        txt = lines[ins[-1][0]]
        tgt = re.search(r"(\.LBB\d+_\d+)", txt)
        if last.startswith(("s_branch", "s_cbranch")) and tgt:
            s.append(label_ix[tgt.group(1)])
    if not last.startswith(("s_branch", "s_endpgm")) and k + 1 < len(blocks):
        s.append(k + 1)
    succ.append(s)

live_in = [set() for _ in blocks]
changed = True
while changed:
    changed = False
    for k in range(len(blocks) - 1, -1, -1):
        live = set()
        for j in succ[k]:
            live |= live_in[j]
        for (_, _, d, u) in reversed(blocks[k][1]):
            live = (live - d) | u
        if live != live_in[k]:
            live_in[k] = live
            changed = True

points = []
for k, (lab, ins) in enumerate(blocks):
    live = set()
    for j in succ[k]:
        live |= live_in[j]
    for (ln, op, d, u) in reversed(ins):
        points.append((len(live), ln, frozenset(live)))
        live = (live - d) | u
points.sort(reverse=True)
print("max live VGPRs %d" % points[0][0])
seen = set()
for n, ln, live in points[:200]:
    if ln // 40 in seen:
        continue
    seen.add(ln // 40)
    print("\n== %d live after line %d: %s" % (n, ln - start, lines[ln].strip()[:90]))
    # last def of each live register before this point (textual, same kernel)
    defs = {}
    for j in range(ln, start, -1):
        t = lines[j].strip()
        if not t or t.startswith((".", ";")) or not lines[j].startswith("\t"):
            continue
        op = t.split()[0]
        if op.startswith(("v_", "ds_read", "global_load", "buffer_load", "scratch_load")) and \
                not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
            for r in regs(t.split(",")[0]) & live:
                defs.setdefault(r, (j - start, t[:80]))
        if len(defs) == len(live):
            break
    for r in sorted(live):
        print("  v%-3d %s" % (r, defs.get(r, ("?", ""))))
    if len(seen) >= top:
        break
