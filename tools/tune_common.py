"""Shared driver plumbing of the end-to-end tuning runs (tools/tune_*.py): a heartbeat line every
minute (a GAM phase can run minutes without a log line), mpc_tuning on the GPU engine, and the
score of a point under the reference's own objectives (VNS2.m:147-195 F, GAM_fun.m:110-111 J1)."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]


def log(*a):
    print(*a, flush=True)


def heartbeat(t0):
    def beat():
        while True:
            time.sleep(60)
            log("... tuning, %.0f s" % (time.time() - t0))

    threading.Thread(target=beat, daemon=True).start()


def score_point(sc, r, N, Nu, delta, lam, w, mdv=None, vns_refs=None):
    """(F_vns, J1, Pareto-weighted J1) of one (N, Nu, delta, lambda) point: VNS2.m:147-195 with the
    point's weights and GAM_fun.m:81-111 J1 against Par.Yref, weighted by the GAM weights w."""
    from mpct.objectives import gam_fun, vns_objective

    F, _, _, _, res = vns_objective(sc, [int(np.max(N))], [int(np.max(Nu))], np.reshape(delta, (1, -1)),
                                    np.reshape(lam, (1, -1)), refs=vns_refs, mdv=mdv)
    X = np.concatenate([np.ravel(delta), np.ravel(lam)])[None]
    J1, r1 = gam_fun(sc, X, N, Nu, r, mdv=mdv)
    return float(F[0]), J1[0], float(J1[0] @ np.asarray(w)), int(res.status.max() | r1.status.max())


def run(name, sc, r, my, ny, w, nbp, nbc, dmin, q0, w0, scale=None, mdv=None, lineal=True, out=None,
        gam_max_iter=400):
    """Environment knobs for A/B runs: MPCT_GAM_SPECULATE=1 (each trial point scored with its
    difference points), MPCT_FGAM_FROM=returned, MPCT_STALE_ROWS=0 (the round-2 quirk handling),
    MPCT_GAM_MAX_FEVALS=n (fgoalattain's MaxFunctionEvaluations; default 100 * numel(x0))."""
    from mpct.tuning import mpc_tuning

    out = out or os.path.join(ROOT, "gpurun_out", "%s_Tuning.mat" % name)
    t0 = time.time()
    heartbeat(t0)
    fev = os.environ.get("MPCT_GAM_MAX_FEVALS")
    log("%s: MPCTuning(nbp=%d, nbc=%d, w=%s, q0=%s, w0=%s, GAM max %d iterations, max %s evaluations) speculate=%s "
        "fgam=%s stale=%s"
        % (name, nbp, nbc, list(np.round(w, 6)), list(q0), list(w0), gam_max_iter, fev or "100*numel(x0)",
           os.environ.get("MPCT_GAM_SPECULATE", "0"), os.environ.get("MPCT_FGAM_FROM", "last_eval"),
           os.environ.get("MPCT_STALE_ROWS", "1")))
    N, Nu, delta, lam, Fob = mpc_tuning(sc, r, my=my, ny=ny, w=w, nbp=nbp, nbc=nbc, dmin=dmin, q0=q0, w0=w0,
                                        log=log, save_path=out, scale=scale, gam_max_iter=gam_max_iter,
                                        lineal=lineal, mdv=mdv,
                                        gam_speculate=os.environ.get("MPCT_GAM_SPECULATE", "0") == "1",
                                        fgam_from=os.environ.get("MPCT_FGAM_FROM", "last_eval"),
                                        stale_rows=os.environ.get("MPCT_STALE_ROWS", "1") != "0",
                                        gam_max_fun_evals=int(fev) if fev else None)
    dt = time.time() - t0
    log("N=%s Nu=%s delta=%s lambda=%s Fob=%s  (%.1f s)" % (N, Nu, delta, lam, Fob, dt))
    return N, Nu, delta, lam, Fob, dt
