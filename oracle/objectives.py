"""Tuning objectives restated (oracle; tests only): GAM_fun (A12), VNS2 objective (A13),
PreCon (A15)."""
from __future__ import annotations

import numpy as np

from .toolbox_gpc import closedloop_toolbox
from .scenarios import vns_step_refs


def precon(N, Nu) -> bool:
    """PreCon.m:23-27."""
    N = np.atleast_1d(N)
    Nu = np.atleast_1d(Nu)
    return bool(N.min() > Nu.max() and np.all(N != 0) and np.all(Nu != 0))


def gam_j1(y, yref):
    """GAM_fun.m:110-111: J1 = diag(errFA*errFA'), errFA = Xy - Yref (all nit samples)."""
    e = y - yref
    return np.einsum("ij,ij->i", e, e)


def vns_terms(y_i, ys_i, yref_i, uopt_n, inK=10):
    """VNS2.m:172-191 for ONE row (output i of simulation i / MV row i of its uopt):
    j21 = sum (y - ys)^2, j22 = sum (y - Yref)^2 from inK, Jnu = sum (|uopt(1)|/|diff(uopt)|)^2
    with inf/NaN mapped to 0."""
    e2 = y_i[inK - 1:] - ys_i[inK - 1:]
    e3 = y_i[inK - 1:] - yref_i[inK - 1:]
    j21 = float(e2 @ e2)
    j22 = float(e3 @ e3)
    d = np.abs(np.diff(uopt_n))
    with np.errstate(divide="ignore", invalid="ignore"):
        xnu = np.abs(uopt_n[0]) / d
    xnu[~np.isfinite(xnu)] = 0.0
    return j21, j22, float(xnu @ xnu)


def vns_objective(sc, yref, N2, Nu, delta, lam, nit, inK=10):
    """VNS2.m:147-195 for one (N, Nu) neighbour with the current GAM weights.
    Square plant: my simulations, each with a unit step on one output (sel).  Returns
    (F, j21[my], j22[my], Jnu[ny])."""
    my, nu = sc.my, sc.nu
    j21 = np.zeros(my)
    j22 = np.zeros(my)
    jnu = np.zeros(nu)
    if my == nu:
        for i, r in enumerate(vns_step_refs(my, nit, inK)):
            res = closedloop_toolbox(sc, r, None, N2, Nu, delta, lam, nit, open_loop=True)
            j21[i], j22[i], jnu[i] = vns_terms(res.y[i], res.ys[i], yref[i], res.uopt[i], inK)
    else:
        raise NotImplementedError("non-square VNS (VNS2.m:168) — Shell 7x5, round 2")
    F = float(np.sum(j21 + j22) + N2 + np.sum(jnu))  # VNS2.m:195, N(1) = max(N) = N2
    return F, j21, j22, jnu
