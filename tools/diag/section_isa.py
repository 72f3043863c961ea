"""Static instruction mix of each `s_memtime` section of a -DMPCT_PROFILE kernel build: the ISA text
between consecutive `; PSTAMP <section>` markers (wave_ops.h PSTAMP), in program order, by class.
A section whose code sits in several places (the QP's check runs at the entry and in its loop) is
listed once per place.  Static counts: loops inside a section (the drop's Givens sweep, the warm
start's drop loop) are counted once.  tools/latency_model.py prices the dependent chain; these
counts give the issue side (a wave issues at most one VALU instruction per ~4 cycles).

Usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMPCT_PROFILE -S --cuda-device-only \
           model-predictive-control-tuning_amd/csrc/gpc_small.hip -o /tmp/gs_prof.s
       python tools/diag/section_isa.py /tmp/gs_prof.s [--kernel gpc_small_kernel]"""
import argparse
import re
import sys


def classify(op):
    if op.startswith("v_"):
        if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
            return "valu_dpp"
        if op.startswith("v_readlane") or op.startswith("v_readfirstlane") or op.startswith("v_writelane"):
            return "lane_xfer"
        if op.startswith("v_permlane"):
            return "permlane"
        if "_f64" in op:
            return "valu_f64"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return None


COLS = ["valu_f64", "valu_dpp", "valu_other", "lane_xfer", "permlane", "lds", "vmem", "salu", "branch", "wait"]
VALU = ("valu_f64", "valu_dpp", "valu_other", "lane_xfer", "permlane")


def section_counts(path, kernel=None):
    """[(section closed by the stamp, {class: count})] in program order"""
    lines = open(path).read().splitlines()
    body, on = [], kernel is None
    for ln in lines:
        if kernel and re.match(r"^\S*%s\S*:" % re.escape(kernel), ln):
            on = True
        if on:
            body.append(ln)
            if kernel and ln.strip().startswith("s_endpgm"):
                break
    cur, counts, order = "(start)", {}, []
    dpp_re = re.compile(r"\b(quad_perm|row_|row_newbcast|row_half_mirror|row_mirror)")
    for ln in body:
        m = re.search(r";\s*PSTAMP\s+(\S+)", ln)
        if m:
            cur = "%s #%d" % (m.group(1), sum(1 for o in order if o.startswith(m.group(1) + " ")))
            order.append(cur)
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = classify(op)
        if c is None:
            continue
        if c.startswith("valu") and dpp_re.search(t):
            c = "valu_dpp"
        counts.setdefault(cur, {}).setdefault(c, 0)
        counts[cur][c] += 1
    # counts[cur] are the instructions AFTER stamp `cur`, i.e. the section that the NEXT stamp closes
    names = ["(start)"] + order
    out = []
    for k, n in enumerate(names):
        if n in counts:
            out.append((names[k + 1] if k + 1 < len(names) else "(end)", counts[n]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default=None, help="only the body of this kernel (a substring of its symbol)")
    a = ap.parse_args()
    print("%-24s %6s " % ("section (ends at stamp)", "total") + " ".join("%10s" % c for c in COLS))
    for closer, row in section_counts(a.asm, a.kernel):
        print("%-24s %6d " % (closer, sum(row.values())) + " ".join("%10d" % row.get(c, 0) for c in COLS))


if __name__ == "__main__":
    sys.exit(main())
