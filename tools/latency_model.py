"""Latency roofline of the metric kernel: the dependent chain of one closed-loop
step of gpc_small_kernel, priced with the primitive latencies measured on the GPU
(tools/latency_probe.hip -> profiles/r05_latency_probe.json), against the cycles the heaviest
simulations actually spend (the -DMPCT_PROFILE build's s_memtime section stamps and section
counts, tools/kprof.py with MPCT_PROF_OUT).

Each section of the step (gpc_small.hip, gpc_qp16.h; the sections of mpct_dev.h PROF_*) is a chain
of primitives whose results the next one waits for; work off that chain (the A rows' loads, the
other three accumulators of a FOR4, the J1 cost) is not counted.  chain(section) = sum over its
primitives of their measured dependent latency; model = sum over sections of chain x executions;
latency_frac = model / measured.  1.0 would mean the kernel runs at the speed of its own dependency
chain with nothing else in the way (issue contention of the SIMD's other waves, instruction issue
of the off-chain work, LDS bank conflicts, waits the compiler's schedule adds).

A second, issue-side figure (--isa): one wave issues at most one VALU instruction per 4 cycles
(a wave64 instruction occupies the 16-lane SIMD for 4 passes; the dependent FMA latency the probe
measures is 5.3 cycles), so a section also costs at least 4 x its VALU instructions.  The static
counts per section come from the profile build's ISA (tools/diag/section_isa.py, minus the stamp's
own VALU); sections with loops inside (the warm start, the QP entry test in qp(rest)) keep their
chain price.  issue_frac = sum over sections of max(chain, issue) x executions / measured.

Usage: python tools/latency_model.py PROBE.json PROF.bin [--isa PROF.s] [--out FILE]
  PROF.bin: the per-simulation section words of the profiled heavy batch (MPCT_PROF_OUT)."""
import argparse
import json
import sys

import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag"))
from section_isa import VALU, section_counts  # noqa: E402

SECTIONS = ["prologue", "plant", "y_update", "unconstrained", "qp(rest)", "u_update", "open_loop",
            "qp.check", "qp.d+z", "qp.r+t1", "qp.add", "qp.drop", "qp.warm", "qp.rotations",
            "qp.w.entry", "qp.w.rebuild", "qp.w.gather", "qp.w.solve", "qp.w.drop", "qp.w.rotations", "qp.w.readds"]

# The chain of each section, per execution, as primitive -> count.  Read off gpc_small.hip's step
# loop and gpc_qp16.h (file:line in the comments); names are tools/latency_probe.hip's probes.
CHAINS = {
    # ring store of the last step's u update -> lds_sync -> the term's ring read -> coef * hv ->
    # v_permlane16/32 row sum over the four term rows -> two quad DPP stages (gpc_small.hip:164-169)
    "plant": {"lds_handoff": 1, "fma_f64": 1, "row4_sum_permlane": 1, "dpp_stage_f64": 2},
    # n1 = y - y(t-1), n2 = n1 - o1, n3 = n2 - o2, stored, lds_sync, read by the product (:173-195)
    "y_update": {"add_f64": 3, "lds_handoff": 1},
    # 6 dependent FMAs per accumulator over quarter 0's 12 columns, the pair add, the row4 sum (:198-221)
    "unconstrained": {"fma_f64": 6, "add_f64": 1, "row4_sum_permlane": 1},
    # the QP entry on a feasible x_u: box slacks (block prefix over the MV's moves), the four
    # slacks' min, the ballot (gpc_qp16.h:336-369); u(t-1) of the row's MV arrives off the chain
    "qp(rest)": {"block_prefix16_nu5": 1, "add_f64": 4, "ballot_branch": 1},
    # the first move by ds_bpermute from the QP's register result, u = u(t-1) + du, ring store (:234-247)
    "u_update": {"shfl_bpermute": 1, "add_f64": 1},
    # most violated inactive constraint: slacks at x, the min over the lane's four kinds, the exact
    # 16-lane argmin and its lane-0 broadcast (wave_ops.h qargmin), the branch (gpc_qp16.h)
    "qp.check": {"block_prefix16_nu5": 1, "add_f64": 4, "qargmin16_exact": 1, "uniform_branch": 1},
    # d = J'n_p (row16 DPP sum, four chains side by side), the products' d^2 FOR4 chain and one
    # permlane row4 sum (the five run side by side) (gpc_qp16.h:192-225, :478-484)
    "qp.d+z": {"row_sum16": 1, "mul_f64": 2, "add_f64": 4, "row4_sum_permlane": 1},
    # ratio test: qp_div (rcp + Newton), the exact argmin, t2 beside it, two uniform branches,
    # x += t z (gpc_qp16.h:485-506)
    "qp.r+t1": {"rcp_nr": 1, "mul_f64": 1, "qargmin16_exact": 1, "uniform_branch": 2, "fma_f64": 1},
    # add: d_q by readlane, |d(q:)| by rsq, 2/v'v by rcp, the J column update, B / R_A columns to LDS,
    # lds_sync before the next read (gpc_qp16.h:229-263)
    "qp.add": {"bcast_readlane": 1, "rsq_nr": 1, "fma_f64": 2, "rcp_nr": 1, "mul_f64": 1, "lds_handoff": 1},
    # drop: readlane of the id, R_A / B column shifts and the Givens sweep through LDS (per rotation:
    # two entries read, rsq, the RMW of R_A and B, lds_sync), B's row shift (gpc_qp16.h:268-322);
    # priced per drop with one rotation (the counted rotations add per rotation below)
    "qp.drop": {"bcast_readlane": 1, "lds_handoff": 3, "dpp_stage_f64": 1},
    # warm start (round 6: five stamps instead of one).  Pre-r06 dumps price the
    # whole warm start as one pass of its solve loop per QP (the first model, 14.7x below measured)
    "qp.warm": {"shfl_bpermute": 1, "mul_f64": 1, "row_sum16": 1, "fma_f64": 4, "row4_sum_permlane": 1,
                "add_f64": 1, "qargmin16_exact": 1, "uniform_branch": 1},
    # the entry test of an infeasible x_u: box slacks, their min, the ballot (gpc_qp16.h gi_qp16 entry)
    "qp.w.entry": {"block_prefix16_nu5": 1, "add_f64": 4, "ballot_branch": 1},
    # the slacks' gather of c = b_A - N_A'x_u by ds_bpermute after the hand-off of the rebuild
    "qp.w.gather": {"lds_handoff": 1, "shfl_bpermute": 1},
    # one pass of the equality solve: B's row (LDS read), w = B'c (row16 DPP), x = x_u + J w and
    # lambda = B w (FOR4 chains + permlane row4 sums), the multipliers' exact argmin
    "qp.w.solve": {"lds_read_chase": 1, "mul_f64": 1, "row_sum16": 1, "fma_f64": 4, "row4_sum_permlane": 1,
                   "add_f64": 1, "qargmin16_exact": 1},
    # one warm drop: the branch into it, the drop (as qp.drop), c's lane shift; its rotations below
    "qp.w.drop": {"uniform_branch": 1, "bcast_readlane": 1, "lds_handoff": 3, "dpp_stage_f64": 2},
    # the rebuild: J <- R^-1 (one hand-off); per re-add below
    "qp.w.rebuild": {"lds_handoff": 1},
}
# one re-add of the rebuild: the hand-off, B's row, d = J'n_p, the products, the add
READD = {"lds_handoff": 2, "row_sum16": 1, "mul_f64": 2, "add_f64": 4, "row4_sum_permlane": 1,
         "bcast_readlane": 1, "rsq_nr": 1, "fma_f64": 2, "rcp_nr": 1}
# one Givens rotation of the drop: entries read, a^2 + b^2, rsq + Newton, cs / sn, the RMW of R_A's
# two rows, lds_sync (gpc_qp16.h:289-310)
ROTATION = {"lds_handoff": 1, "fma_f64": 1, "rsq_nr": 1, "mul_f64": 1}
# the profile build's stamp closing each section (section_isa.py names; #1: the QP loop's check)
ISA_SECTION = {"plant": "PROF_PLANT #0", "y_update": "PROF_YUPD #0", "unconstrained": "PROF_UNC #0",
               "u_update": "PROF_UUPD #0", "qp.check": "PROF_QCHECK #1", "qp.d+z": "PROF_QD #0",
               "qp.r+t1": "PROF_QR #0", "qp.add": "PROF_QADD #0", "qp.drop": "PROF_QDROP #0",
               "qp.w.entry": "PROF_QWENTRY #0", "qp.w.gather": "PROF_QWGATH #0", "qp.w.solve": "PROF_QWSOLVE #0",
               "qp.w.drop": "PROF_QWDROP #0"}
STAMP_VALU = 6  # ProfAcc.add: lane id copy, compare, two selects, 64-bit add (wave_ops.h)


def chain_cycles(chain, lat):
    return sum(n * lat[k] for k, n in chain.items())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("probe")
    ap.add_argument("prof")
    ap.add_argument("--isa", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    valu = {}
    if a.isa:
        for closer, row in section_counts(a.isa, "gpc_small_kernel"):
            valu.setdefault(closer, sum(row.get(c, 0) for c in VALU) - STAMP_VALU)
    lat = json.load(open(a.probe))
    raw = np.fromfile(a.prof, dtype=np.uint64)
    # r06 dumps: 21 words per simulation; r05: 14 (no warm-start split); before: 13
    width = next(w for w in (len(SECTIONS), 14, 13) if raw.size % w == 0)
    raw = raw.reshape(-1, width)
    shift = 40 if width > 14 else 48  # count field: 24 bits since r06 (wave_ops.h kProfCountShift)
    cyc = (raw & np.uint64((1 << shift) - 1)).astype(np.float64)
    cnt = (raw >> np.uint64(shift)).astype(np.float64)
    S = raw.shape[0]
    rows = {}
    model = measured = bound = 0.0
    for k, name in enumerate(SECTIONS[:width]):
        if name not in CHAINS:
            continue
        per = chain_cycles(CHAINS[name], lat)
        n = cnt[:, k].mean()
        if name == "qp.check":  # the QP's entry stamp closes a near-empty section once per step
            n -= cnt[:, SECTIONS.index("plant")].mean()
        m = cyc[:, k].mean()
        mod = per * n
        if name == "qp.drop" and width > 13:  # plus the counted Givens rotations of every drop
            mod += chain_cycles(ROTATION, lat) * cnt[:, SECTIONS.index("qp.rotations")].mean()
        if name == "qp.w.drop":  # the warm drops' rotations
            mod += chain_cycles(ROTATION, lat) * cnt[:, SECTIONS.index("qp.w.rotations")].mean()
        if name == "qp.w.rebuild":  # its re-adds
            mod += chain_cycles(READD, lat) * cnt[:, SECTIONS.index("qp.w.readds")].mean()
        if name == "qp.warm" and width > 14:  # split into the qp.w.* sections: the rest is a stamp
            per, mod = 0.0, 0.0
        rows[name] = dict(executions=round(n, 1), chain_cycles=round(per, 1), model=round(mod),
                          measured=round(m), frac=round(mod / m, 3) if m else None)
        b = mod
        if name in ISA_SECTION and ISA_SECTION[name] in valu:
            iss = 4.0 * valu[ISA_SECTION[name]]
            b = max(per, iss) * n + (mod - per * n)
            rows[name].update(valu_static=valu[ISA_SECTION[name]], issue_cycles=round(iss),
                              bound=round(b), bound_frac=round(b / m, 3) if m else None)
        model += mod
        bound += b
        measured += m
    rep = dict(simulations=int(S), probe=a.probe, model_cycles=round(model), measured_cycles=round(measured),
               latency_frac=round(model / measured, 3),
               issue_frac=round(bound / measured, 3) if valu else None, sections=rows,
               note="measured excludes the prologue (once per simulation); cycles per simulation, mean over "
                    "the batch; stamps add ~11 % to the measured side (MI355X_MICROARCH.md)")
    print(json.dumps(rep, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
