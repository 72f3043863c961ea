"""Where the NMPC kernel's issued FP64 goes: config 5's 4096 candidates (GAM mode,
bench.py --workload vandevusse) on the -DMPCT_PROFILE build (libmpct_prof.so), whose count slots
(mpct_dev.h PROF_NM_NPASS / POINTS / USED / ROWS) record per simulation the full passes, the points
they were asked for, the points an iteration went on to use, and the point rows each pass occupies,
beside the section cycles.

A full pass runs the RK4 prediction with forward tangents and the streamed QR on every lane of the
wave: point g on 16-lane row g (M <= 15 class, G = 4 rows) or on the whole wave (M > 15, G = 1),
lane m < M + 1 of a point's row carrying tangent column m (the M increments and the residual).
Every FP64 instruction of a pass is issued for all 64 lanes, so per pass and prediction step the
issued lane-slots split into
  * useful: (M + 1) lanes of each point whose linearisation an iteration used;
  * speculation / rejection: (M + 1) lanes of each point computed and never used (a later call that
    did not start from the speculated point, the Anderson candidate or the alpha = 1 step that lost);
  * idle lanes: the other lanes (beyond M + 1 in every row, and rows without a point);
and a tangent-free Armijo trial issues all 64 lanes for one lane's worth of prediction.  The weights
per pass and per trial are their measured cycles per execution (both are FP64-issue bound: DESIGN §12).
Usage: python tools/nmpc_fp64_split.py [C] [--out FILE]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCT_LIB", os.path.join(ROOT, "model-predictive-control-tuning_amd", "csrc", "libmpct_prof.so"))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np  # noqa: E402

NAMES = ["full_pass", "rinv+step", "qp", "anderson_pass", "ls_full_pass", "ls_trials", "plant_rk4", "other",
         "n.passes", "n.points", "n.used", "n.rows"]
SHIFT = 40  # wave_ops.h kProfCountShift


def split(raw, N, Nu, nu=2):
    """The lane-slot split from the per-simulation words raw [S][PROF_N] and the horizons."""
    cyc = (raw & np.uint64((1 << SHIFT) - 1)).astype(np.float64)
    cnt = (raw >> np.uint64(SHIFT)).astype(np.float64)
    k = {n: i for i, n in enumerate(NAMES)}
    M1 = nu * Nu.astype(np.float64) + 1.0
    passes, points, used, rows = (cnt[:, k[n]] for n in ("n.passes", "n.points", "n.used", "n.rows"))
    lanes_row = np.where(M1 - 1 <= 15, 16.0, 64.0)  # a point's row: 16 lanes, or the whole wave
    # measured cycles of one full pass per simulation (first, Anderson and alpha = 1 passes alike)
    full_cyc = cyc[:, k["full_pass"]] + cyc[:, k["anderson_pass"]] + cyc[:, k["ls_full_pass"]]
    per_pass = np.where(passes > 0, full_cyc / np.maximum(passes, 1), 0.0)
    trials = cnt[:, k["ls_trials"]]
    per_trial = np.where(trials > 0, cyc[:, k["ls_trials"]] / np.maximum(trials, 1), 0.0)
    # issued lane-slots, weighted by the cycles of what issued them
    issued_full = passes * per_pass * 64.0
    useful = used * per_pass * M1
    spec = np.maximum(points - used, 0.0) * per_pass * M1
    idle = issued_full - useful - spec
    issued_trial = trials * per_trial * 64.0
    trial_useful = trials * per_trial * 1.0
    tot = issued_full.sum() + issued_trial.sum()
    rep = {
        "simulations": int(raw.shape[0]),
        "per_simulation_mean": {"full_passes": float(passes.mean()), "points": float(points.mean()),
                                "points_used": float(used.mean()), "rows_per_pass": float((rows / np.maximum(passes, 1)).mean()),
                                "trials": float(trials.mean()), "M_plus_1": float(M1.mean())},
        "share_of_issued_lane_slots": {
            "useful_tangent_columns": float(useful.sum() / tot),
            "speculated_or_rejected_points": float(spec.sum() / tot),
            "idle_lanes": float(idle.sum() / tot),
            "trial_pass_redundancy": float((issued_trial.sum() - trial_useful.sum()) / tot),
            "trial_pass_useful": float(trial_useful.sum() / tot),
        },
        "idle_lanes_by_class": {
            "M<=15 (16-lane rows)": float(idle[M1 - 1 <= 15].sum() / tot),
            "M>15 (whole wave)": float(idle[M1 - 1 > 15].sum() / tot),
        },
        "cycle_share": {n: float(cyc[:, k[n]].sum() / cyc[:, :8].sum()) for n in NAMES[:8]},
        "note": "lane-slot shares of the FP64 work issued by full (tangent) and trial passes, each pass weighted "
                "by its measured cycles; the QP, R^-1 and the plant (%.1f %% of the cycles) are not split" % (
                    100.0 * (cyc[:, k["qp"]] + cyc[:, k["rinv+step"]] + cyc[:, k["plant_rk4"]]).sum()
                    / cyc[:, :8].sum()),
    }
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("C", nargs="?", type=int, default=4096)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from mpct.engine import eval_batch
    from mpct.nmpc import nmpc_candidate_grid, vandevusse

    sc, r, _ = vandevusse()
    N, Nu, d, l = nmpc_candidate_grid(a.C)
    dump = (a.out or "nmpc_prof") + ".bin"
    os.environ["MPCT_PROF_OUT"] = dump
    res = eval_batch(sc, N, Nu, d, l, r[None])
    raw = np.fromfile(dump, dtype=np.uint64)
    raw = raw.reshape(N.size, -1)
    rep = split(raw, N, Nu)
    rep["gauss_newton_iterations_mean"] = float(res.qp_iters.mean())
    print(json.dumps(rep, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
