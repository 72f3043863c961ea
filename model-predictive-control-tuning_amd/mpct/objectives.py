"""Batched mirrors of the tuner's objective functions, evaluated on the GPU engine.

gam_fun      GAM_fun.m:55-116  — g = J1 per output for a batch of weight vectors X
vns_objective VNS2.m:147-195   — F for a batch of (N, Nu) neighbours at fixed weights
precon       PreCon.m:23-27
rank         stable ranking of candidates (primary cost, candidate-index tiebreak)
"""
from __future__ import annotations

import numpy as np

from .engine import eval_batch
from .scenarios import vns_step_refs


def precon(N, Nu) -> bool:
    N, Nu = np.atleast_1d(N), np.atleast_1d(Nu)
    return bool(N.min() > Nu.max() and np.all(N != 0) and np.all(Nu != 0))


def gam_fun(sc, X, N, Nu, Xsp, ov_weights=None):
    """[g,h] = GAM_fun(X,Par) for each row of X (C x (my+nu)): delta = |X(1:my)|,
    lambda = |X(my+1:end)|; outputs whose initial OV weight is 0 stay 0 (band mode,
    GAM_fun.m:62-72).  Returns (g (C x my), EvalResult)."""
    X = np.atleast_2d(np.asarray(X, dtype=float))
    Cn = X.shape[0]
    delta = np.abs(X[:, : sc.my]).copy()
    lam = np.abs(X[:, sc.my: sc.my + sc.nu])
    if ov_weights is not None:
        delta[:, np.asarray(ov_weights) == 0] = 0.0
    N2 = np.full(Cn, int(np.max(N)), dtype=np.int32)
    Nuv = np.full(Cn, int(np.max(Nu)), dtype=np.int32)
    res = eval_batch(sc, N2, Nuv, delta, lam, np.asarray(Xsp)[None], open_loop=False)
    return res.J1, res


def vns_refs_nonlinear(Xsp):
    """Nonlinear models keep the driver's setpoint Par.Xsp (VNS2.m:67-71 leaves it as is) and
    simulate Xsp.*sel, one output selected at a time (VNS2.m:148-155): the unselected outputs get
    a zero reference, as in the reference."""
    Xsp = np.asarray(Xsp, dtype=float)
    my = Xsp.shape[0]
    return np.stack([Xsp * (np.arange(my) == i)[:, None] for i in range(my)])


def vns_objective(sc, N2, Nu, delta, lam, inK=10, device=-1, refs=None):
    """F = sum(j21 + j22) + N(1) + sum(Jnu) (VNS2.m:195) for C candidates (square plant: my
    simulations per candidate, output i / MV i taken from simulation i, VNS2.m:148-165).
    refs: the my reference sets (default: the linear models' unit steps at inK, VNS2.m:58-61;
    vns_refs_nonlinear for an NMPC scenario).
    Returns (F (C,), j21 (C,my), j22 (C,my), Jnu (C,nu), EvalResult)."""
    if sc.my != sc.nu:
        raise NotImplementedError("non-square VNS path (VNS2.m:168) is a later-round item")
    N2 = np.atleast_1d(N2).astype(np.int32)
    Cn = N2.size
    if refs is None:
        refs = vns_step_refs(sc.my, sc.nit, inK)
    res = eval_batch(sc, N2, Nu, delta, lam, refs, open_loop=True, device=device)
    idx = np.arange(sc.my)
    j21 = res.j21.reshape(Cn, sc.my, sc.my)[:, idx, idx]
    j22 = res.j22.reshape(Cn, sc.my, sc.my)[:, idx, idx]
    jnu = res.Jnu.reshape(Cn, sc.my, sc.nu)[:, idx, idx]
    F = j21.sum(1) + j22.sum(1) + N2 + jnu.sum(1)
    return F, j21, j22, jnu, res


def rank(cost) -> np.ndarray:
    """Candidate order by ascending cost, ties broken by candidate index (stable sort)."""
    return np.argsort(np.asarray(cost), kind="stable")
