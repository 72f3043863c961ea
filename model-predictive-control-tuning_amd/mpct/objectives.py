"""Batched mirrors of the tuner's objective functions, evaluated on the GPU engine.

gam_fun      GAM_fun.m:55-116  — g = J1 per output for a batch of weight vectors X
vns_objective VNS2.m:147-195   — F for a batch of (N, Nu) neighbours at fixed weights (square
             plants: one simulation per output, VNS2.m:148-165; non-square: one simulation with
             Xsp, VNS2.m:166-169); measured disturbances Par.mdv are passed to every simulation
             (VNS2.m:153,168, GAM_fun.m:81)
vns_row1_broadcast  VNS2.m:172-195 with only row 1 of Xy assigned (implicit expansion)
precon       PreCon.m:23-27
failed       which statuses make a simulation unusable (the reference's swallowed exception)
rank         stable ranking of candidates (primary cost, candidate-index tiebreak)
"""
from __future__ import annotations

import numpy as np

from ._lib import ST_BADHORIZON, ST_NONFINITE, ST_NOT_RUN, ST_QP_INFEAS, ST_SKIPPED
from .engine import eval_batch
from .scenarios import vns_step_refs

# A simulation is unusable only when the reference's sim/nlmpcmove would have thrown (caught and
# skipped with fprintf, VNS2.m:161-163, GAM_fun.m:82-84) or produced no trajectory: an infeasible
# QP, a non-finite state, a skipped or invalid candidate -- or a slot that no kernel launch
# simulated (ST_NOT_RUN, an internal dispatch fault: its costs are the prefill's NaN).  An iteration cap (QP_MAXITER, NMPC
# SQP_MAXITER) or an NMPC closed loop that grazed its state bounds keeps the last iterate and a
# finite cost, as mpcmove / nlmpcmove do (closedloop_toolbox_nmpc.m:69 uses the last iterate).
FATAL_STATUS = ST_QP_INFEAS | ST_NONFINITE | ST_SKIPPED | ST_BADHORIZON | ST_NOT_RUN


def failed(status) -> np.ndarray:
    """Boolean mask of simulations whose costs must not be used (FATAL_STATUS bits)."""
    return (np.asarray(status) & FATAL_STATUS) != 0


def precon(N, Nu) -> bool:
    N, Nu = np.atleast_1d(N), np.atleast_1d(Nu)
    return bool(N.min() > Nu.max() and np.all(N != 0) and np.all(Nu != 0))


def gam_fun(sc, X, N, Nu, Xsp, ov_weights=None, mdv=None):
    """[g,h] = GAM_fun(X,Par) for each row of X (C x (my+nu)): delta = |X(1:my)|,
    lambda = |X(my+1:end)|; outputs whose initial OV weight is 0 stay 0 (band mode,
    GAM_fun.m:62-72); mdv = Par.mdv (nd x nit, GAM_fun.m:81).  Returns (g (C x my), EvalResult)."""
    X = np.atleast_2d(np.asarray(X, dtype=float))
    Cn = X.shape[0]
    delta = np.abs(X[:, : sc.my]).copy()
    lam = np.abs(X[:, sc.my: sc.my + sc.nu])
    if ov_weights is not None:
        delta[:, np.asarray(ov_weights) == 0] = 0.0
    N2 = np.full(Cn, int(np.max(N)), dtype=np.int32)
    Nuv = np.full(Cn, int(np.max(Nu)), dtype=np.int32)
    v = None if mdv is None or np.size(mdv) == 0 else np.asarray(mdv, dtype=float)[None]
    res = eval_batch(sc, N2, Nuv, delta, lam, np.asarray(Xsp)[None], v=v, open_loop=False)
    return res.J1, res


def vns_refs_nonlinear(Xsp):
    """Nonlinear models keep the driver's setpoint Par.Xsp (VNS2.m:67-71 leaves it as is) and
    simulate Xsp.*sel, one output selected at a time (VNS2.m:148-155): the unselected outputs get
    a zero reference, as in the reference."""
    Xsp = np.asarray(Xsp, dtype=float)
    my = Xsp.shape[0]
    return np.stack([Xsp * (np.arange(my) == i)[:, None] for i in range(my)])


def vns_refs_nonsquare(my, nit, inK=10):
    """Non-square linear plants: the single VNS simulation uses Xsp with every output stepped to 1
    at inK (VNS2.m:58-61 overwrite Xsp, VNS2.m:168 passes it whole)."""
    R = np.zeros((1, my, nit))
    R[0, :, inK - 1:] = 1.0
    return R


def vns_objective(sc, N2, Nu, delta, lam, inK=10, device=-1, refs=None, mdv=None):
    """F = sum(j21 + j22) + N(1) + sum(Jnu) (VNS2.m:195) for C candidates.
    Square plant (my == nu): my simulations per candidate, output i / MV i taken from simulation
    i (VNS2.m:148-165).  Non-square: ONE simulation per candidate with Xsp (VNS2.m:166-169), all
    my outputs and nu MVs from it.  refs: the reference sets (default: the linear models' unit
    steps at inK, VNS2.m:58-61; vns_refs_nonlinear for an NMPC scenario).  mdv = Par.mdv (nd x
    nit), passed to every simulation (VNS2.m:153,168).
    Returns (F (C,), j21 (C,my), j22 (C,my), Jnu (C,nu), EvalResult)."""
    N2 = np.atleast_1d(N2).astype(np.int32)
    Cn = N2.size
    square = sc.my == sc.nu
    if refs is None:
        refs = vns_step_refs(sc.my, sc.nit, inK) if square else vns_refs_nonsquare(sc.my, sc.nit, inK)
    refs = np.asarray(refs, dtype=float).reshape(-1, sc.my, sc.nit)
    v = None if mdv is None or np.size(mdv) == 0 else np.asarray(mdv, dtype=float)[None]
    res = eval_batch(sc, N2, Nu, delta, lam, refs, v=v, open_loop=True, device=device)
    nref = refs.shape[0]
    if square:
        if nref != sc.my:
            raise ValueError("a square plant's VNS runs one simulation per output (%d refs)" % sc.my)
        idx = np.arange(sc.my)
        j21 = res.j21.reshape(Cn, sc.my, sc.my)[:, idx, idx]
        j22 = res.j22.reshape(Cn, sc.my, sc.my)[:, idx, idx]
        jnu = res.Jnu.reshape(Cn, sc.my, sc.nu)[:, idx, idx]
    else:
        if nref != 1:
            raise ValueError("a non-square plant's VNS runs one simulation with Xsp (VNS2.m:168)")
        j21, j22, jnu = res.j21, res.j22, res.Jnu
    F = j21.sum(1) + j22.sum(1) + N2 + jnu.sum(1)
    return F, j21, j22, jnu, res


def vns_row1_broadcast(sc, N2, Nu, delta, lam, inK=10, device=-1, refs=None, mdv=None) -> float:
    """VNS2.m:172-195 when Xy holds only row 1 (a square plant's simulations of outputs 2..my have
    all failed so far in this VNS2 pass, VNS2.m:151-163): errYref = Xy - Yref broadcasts row 1
    against every output's Yref (MATLAB implicit expansion), j21 and Jnu stay scalars, so
    sum(j21 + j22) + sum(Jnu) = my j21_1 + sum_i sum_{t >= inK} (y_1(t) - Yref_i(t))^2 + Jnu_1.
    Returns that (F without N(1)) from simulation 1 (output 1 stepped) with its trajectory."""
    refs = vns_step_refs(sc.my, sc.nit, inK) if refs is None else np.asarray(refs, dtype=float)
    refs = refs.reshape(-1, sc.my, sc.nit)[:1]
    v = None if mdv is None or np.size(mdv) == 0 else np.asarray(mdv, dtype=float)[None]
    res = eval_batch(sc, np.array([N2], np.int32), np.array([Nu], np.int32),
                     np.asarray(delta, dtype=float).reshape(1, sc.my), np.asarray(lam, dtype=float).reshape(1, sc.nu),
                     refs, v=v, open_loop=True, want_traj=True, device=device)
    y1 = res.y[0, 0, inK - 1:]
    B = ((y1[None, :] - np.asarray(sc.yref, dtype=float)[:, inK - 1:]) ** 2).sum(1)
    return float(sc.my * res.j21[0, 0] + B.sum() + res.Jnu[0, 0])


def rank(cost) -> np.ndarray:
    """Candidate order by ascending cost, ties broken by candidate index (stable sort)."""
    return np.argsort(np.asarray(cost), kind="stable")
