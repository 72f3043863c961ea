"""Scenario builders for the reference's driver scripts (product host code).

shell3x3(): MPC-Tuning/Shell3x3.m with caso = 2, nominal, rest = true — BASELINE config 2.
The CondMin scaling is taken from the committed tuning result (MPCTuning.m:155 CondMin's
fmincon optimum is not unique: cond() is scale invariant), transcribed below from
MPC-Tuning/Shell3x3_Tuning_25Jul2023_12_06.mat (Tuning_Parameters.scale.L / .R).
"""
from __future__ import annotations

import numpy as np

from .engine import Scenario
from .lti import c2d, lsim

# Shell3x3.m:52-57 nominal model, Ts, nit
SHELL3_K = np.array([[4.05, 1.77, 5.88], [5.39, 5.72, 6.9], [4.38, 4.42, 7.2]])
SHELL3_TAU = np.array([[50, 60, 50], [50, 60, 40], [33, 44, 19]], dtype=float)
SHELL3_DELAY = np.array([[27, 28, 27], [18, 14, 15], [20, 22, 0]], dtype=float)
SHELL3_TS, SHELL3_NIT = 4.0, 500
# Shell3x3_Tuning_25Jul2023_12_06.mat: Tuning_Parameters.scale (diagonals)
SHELL3_L = np.array([0.43577812475231503, 0.4205588479390135, 0.5932860051199568])
SHELL3_R = np.array([0.661867070834956, 0.2756082654542081, 0.41172304878568067])
# ... and the tuned point it stores (N=24, Nu=[6 2 2])
SHELL3_TUNED = dict(N=24, Nu=(6, 2, 2),
                    delta=(0.010659948215964849, 0.004019856475662751, 0.0007926546087416782),
                    lam=(9.247457388705409e-05, 0.0005523146971406108, 0.0015219790494510478))


def shell3x3_xsp(nit=SHELL3_NIT):
    """Setpoint of Shell3x3.m:89-92 (1-based inclusive ranges, later ones overwrite)."""
    X = np.zeros((3, max(nit, 500)))
    levels = [(0.2, 0.0, 0.1, 0.0), (0.2, 0.4, 0.3, 0.0), (0.2, 0.1, 0.0, 0.0)]
    for i, (a, b, c, d) in enumerate(levels):
        X[i, 9:80] = a
        X[i, 79:200] = b
        X[i, 199:400] = c
        X[i, 399:500] = d
    return X[:, :nit]


def shell3x3_yref(X, caso=2):
    """Yref = lsim(Pref, Xsp, t, 'zoh') (Shell3x3.m:71-76, 98-99)."""
    taus = (5.0, 9.0, 5.7) if caso == 1 else (30.0, 30.0, 30.0)
    delays = (27.0, 14.0, 0.0)
    return np.stack([lsim(c2d([1.0], [taus[i], 1.0], SHELL3_TS, delays[i]), X[i]) for i in range(3)])


def shell3x3_plant(L=SHELL3_L, R=SHELL3_R):
    """Pze = L * c2d(Ps, Ts, 'zoh') * R  (Shell3x3.m:65, MPCTuning.m:162)."""
    return [[c2d([SHELL3_K[i, j]], [SHELL3_TAU[i, j], 1.0], SHELL3_TS, SHELL3_DELAY[i, j]).scale(L[i] * R[j])
             for j in range(3)] for i in range(3)]


def shell3x3(n2_max=30, nu_max=5, nit=SHELL3_NIT, L=SHELL3_L, R=SHELL3_R, window="toolbox",
             weights_squared=True, exact_carima=True):
    """Returns (Scenario, r, yref): r = L*Xsp, yref = L*Yref (MPCTuning.m:188-189) as row signals.
    Bounds: Shell3x3.m:120-123 scaled by R (MPCTuning.m:170-178)."""
    P = shell3x3_plant(L, R)
    X = shell3x3_xsp(nit)
    yref = L[:, None] * shell3x3_yref(X)
    r = L[:, None] * X
    sc = Scenario(P, P, nu=3, du_min=-0.05 / R, du_max=0.05 / R, u_min=-1.0 / R, u_max=0.5 / R,
                  yref=yref, n2_max=n2_max, nu_max=nu_max, Ts=SHELL3_TS, window=window,
                  weights_squared=weights_squared, exact_carima=exact_carima)
    return sc, r, yref


def vns_step_refs(my, nit, inK=10):
    """VNS2.m:58-61 + 147-150: one simulation per output with a unit step on that output."""
    R = np.zeros((my, my, nit))
    for i in range(my):
        R[i, i, inK - 1:] = 1.0
    return R


def candidate_grid(C=4096, my=3, nu=3, N2=30, Nu=5, seed=20250307, tuned=SHELL3_TUNED):
    """BASELINE config 2 grid: log10 delta ~ U(-4,0), log10 lambda ~ U(-5,-1),
    numpy default_rng(20250307); candidate 0 is the fixture-tuned (delta, lambda) at N2, Nu."""
    rng = np.random.default_rng(seed)
    delta = 10.0 ** rng.uniform(-4, 0, size=(C, my))
    lam = 10.0 ** rng.uniform(-5, -1, size=(C, nu))
    if tuned is not None and C > 0:
        delta[0] = tuned["delta"]
        lam[0] = tuned["lam"]
    return (np.full(C, N2, dtype=np.int32), np.full(C, Nu, dtype=np.int32), delta, lam)
