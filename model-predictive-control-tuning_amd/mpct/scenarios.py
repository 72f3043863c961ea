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


# ---------------------------------------------------------------------------------------------
# Shell 7x5 (config 3): MPC-Tuning/Shell7x5.m, nominal (e1..e5 = 0, :38-43).  [Gs Ds] of
# Shell7x5.m:73-91 (3 MVs, 2 measured disturbances), Ts = 4, nit = 200.  Scaling from the
# committed Shell7x5_Tuning_14Sep2024_14_22.mat (Tuning_Parameters.scale), which also holds the
# tuned point below.
SHELL7_K = np.array([[4.05, 1.77, 5.88, 1.20, 1.44], [5.39, 5.72, 6.9, 1.52, 1.83],
                     [3.66, 1.65, 5.53, 1.16, 1.27], [5.92, 2.54, 8.10, 1.73, 1.79],
                     [4.13, 2.38, 6.23, 1.31, 1.26], [4.06, 4.18, 6.53, 1.19, 1.17],
                     [4.38, 4.42, 7.2, 1.14, 1.26]])
SHELL7_TAU = np.array([[50, 60, 50, 45, 40], [50, 60, 40, 25, 20], [9, 30, 40, 11, 6],
                       [12, 27, 20, 5, 19], [8, 19, 10, 2, 22], [13, 33, 9, 19, 24],
                       [33, 44, 19, 24, 32]], dtype=float)
SHELL7_DELAY = np.array([[27, 28, 27, 27, 27], [18, 14, 15, 15, 15], [2, 20, 2, 0, 0], [11, 12, 2, 0, 0],
                         [5, 7, 2, 0, 0], [8, 4, 1, 0, 0], [20, 22, 0, 0, 0]], dtype=float)
SHELL7_TS, SHELL7_NIT = 4.0, 200
SHELL7_YMX = np.array([0.005, 0.005, 0.5, 0.5, 0.5, 0.5, 0.5])   # Shell7x5.m:106-107
SHELL7_ECR = np.array([0.1, 0.5, 1, 1, 1, 1, 1])                   # Shell7x5.m:143-152
SHELL7_L = np.array([0.4400615063022943, 0.2319273262887009, 0.6265090010777253, 0.5431290766409146,
                     0.6006058918173808, 0.20692945405215463, 0.39416907820719865])
SHELL7_R = np.array([0.2639712478155768, 0.1350971290956903, 0.1156440799331315, 0.781865375367461,
                     0.4665315477471682])
SHELL7_TUNED = dict(N=27, Nu=(2, 2, 2), delta=(0.0,) * 7,
                    lam=(0.055949075594369936, 0.016702486485524682, 1.6101890690935143))
SHELL7_W = np.array([1e-4, 1e-4, 1, 0.5, 1, 0.5, 1])               # Shell7x5.m:202 (GAM weights)


CONFIG3_N2 = (16, 24, 32, 48, 64, 96, 112, 127)
CONFIG3_NU = (2, 3, 4, 6, 8, 10, 12, 15)


def config3_grid(per=1024, seed=20250307):
    """BASELINE config 3 grid: N2 x Nu cells (N2-major, 64 cells) x ``per``
    lambda draws log10 U(-3, 1) (numpy default_rng(seed)), delta = 0 (band mode, Shell7x5.m:190).
    Candidate c sits in cell c // per: N2 = CONFIG3_N2[cell // 8], Nu = CONFIG3_NU[cell % 8]."""
    rng = np.random.default_rng(seed)
    N2 = np.repeat(np.array([n for n in CONFIG3_N2 for _ in CONFIG3_NU], np.int32), per)
    Nu = np.repeat(np.array([u for _ in CONFIG3_N2 for u in CONFIG3_NU], np.int32), per)
    lam = 10.0 ** rng.uniform(-3, 1, size=(N2.size, 3))
    return N2, Nu, np.zeros((N2.size, 7)), lam


def config3_stratified(per_cell=128, per=1024):
    """Indices of the first ``per_cell`` lambda draws of every config-3 cell (the parity sample)."""
    return (np.arange(64)[:, None] * per + np.arange(per_cell)[None, :]).ravel()


def shell7x5_plant(L=SHELL7_L, R=SHELL7_R):
    """Pze = L * c2d([Gs Ds], Ts, 'zoh') * R  (Shell7x5.m:93-98, MPCTuning.m:162)."""
    return [[c2d([SHELL7_K[i, j]], [SHELL7_TAU[i, j], 1.0], SHELL7_TS, SHELL7_DELAY[i, j]).scale(L[i] * R[j])
             for j in range(5)] for i in range(7)]


def shell7x5_signals(nit=SHELL7_NIT, tmd=20, L=SHELL7_L, R=SHELL7_R):
    """(r, v, yref): r = L*Xsp = 0 (Shell7x5.m:118), v = Rv\\mdv with mdv = 0.5 from tmd
    (:121-123, MPCTuning.m:191), yref = L*lsim(Pref, Xref) with Xref(i, tmd:tmd+5) = Ymx(i) and
    Pref = 1/(50s+1) delayed by min over row i of [Gs Ds].iodelay (:126-135, MPCTuning.m:188)."""
    X = np.zeros((7, nit))
    X[:, tmd - 1: tmd + 5] = SHELL7_YMX[:, None]
    dl = SHELL7_DELAY.min(axis=1)
    Yref = np.stack([lsim(c2d([1.0], [50.0, 1.0], SHELL7_TS, dl[i]), X[i]) for i in range(7)])
    mdv = np.zeros((2, nit))
    mdv[:, tmd - 1:] = 0.5
    return np.zeros((7, nit)), mdv / R[3:, None], L[:, None] * Yref


def shell7x5(n2_max=127, nu_max=15, nit=SHELL7_NIT, L=SHELL7_L, R=SHELL7_R):
    """Returns (Scenario, r, v, yref) for the toolbox MPC of Shell7x5.m after MPCTuning's
    scaling: MV bounds +-0.5/R (:110-111, 135-138; no rate bounds), soft OV bands L*Ymn..L*Ymx
    with MinECR/MaxECR (:141-152), OV ScaleFactor = L*Yrange unless Yrange == 1 (:162-168,
    MPCTuning.m:182-184), MV ScaleFactor 1 (Urange = 1), Weights.ECR = 1e4 (:191)."""
    P = shell7x5_plant(L, R)
    r, v, yref = shell7x5_signals(nit, L=L, R=R)
    umx = 0.5 / R[:3]
    yr = 2 * SHELL7_YMX
    bands = dict(y_min=-L * SHELL7_YMX, y_max=L * SHELL7_YMX, ecr_min=SHELL7_ECR, ecr_max=SHELL7_ECR,
                 y_scale=np.where(yr != 1.0, L * yr, yr), u_scale=np.ones(3), rho=1e4)
    inf = np.full(3, np.inf)
    sc = Scenario(P, P, nu=3, du_min=-inf, du_max=inf, u_min=-umx, u_max=umx, yref=yref,
                  n2_max=n2_max, nu_max=nu_max, Ts=SHELL7_TS, window="toolbox", bands=bands)
    return sc, r, v, yref


# ---------------------------------------------------------------------------------------------
# WoodBerry.m (toolbox MPC, caso = 1, nominal, rest = true): [Gs Ds] with one measured
# disturbance, Ts = 1, nit = 400.  The reference commits no WoodBerry tuning .mat, so CondMin's
# scaling is not pinned: L = R = I unless given.
WB_K = np.array([[12.8, -18.9, 3.8], [6.6, -19.4, 4.9]])          # WoodBerry.m:48-52
WB_TAU = np.array([[16.7, 21.0, 14.9], [10.9, 14.4, 13.2]])
WB_DELAY = np.array([[1.0, 2.0, 8.1], [2.0, 1.0, 3.4]])
WB_W = np.array([0.1, 0.5])                                        # WoodBerry.m:155


def woodberry_toolbox(n2_max=30, nu_max=10, nit=400, caso=1, L=np.ones(2), R=np.ones(3)):
    """Returns (Scenario, r, v, yref) of WoodBerry.m:43-148: rate bounds +-0.05, amplitude
    +-0.5 (:118-134, scaled by R), unbounded outputs; Xsp(1, 10:) = 0.8, Xsp(2, 200:) = 0.5
    (:87-89); mdv(300:) = -0.25 (:92-94); Yref = lsim(Pref, Xsp) with Pref diag(1/(10s+1),
    1/(7s+1)) (caso 1) or diag(1/(15s+1), 1/(12s+1)), delays [1, 1] (:69-75, :98)."""
    P = [[c2d([WB_K[i, j]], [WB_TAU[i, j], 1.0], 1.0, WB_DELAY[i, j]).scale(L[i] * R[j]) for j in range(3)]
         for i in range(2)]
    X = np.zeros((2, nit))
    X[0, 9:] = 0.8
    X[1, 199:] = 0.5
    taus = (10.0, 7.0) if caso == 1 else (15.0, 12.0)
    Yref = np.stack([lsim(c2d([1.0], [taus[i], 1.0], 1.0, 1.0), X[i]) for i in range(2)])
    mdv = np.zeros((1, nit))
    mdv[0, 299:] = -0.25
    Ru = R[:2]
    sc = Scenario(P, P, nu=2, du_min=-0.05 / Ru, du_max=0.05 / Ru, u_min=-0.5 / Ru, u_max=0.5 / Ru,
                  yref=L[:, None] * Yref, n2_max=n2_max, nu_max=nu_max, Ts=1.0, window="toolbox")
    return sc, L[:, None] * X, mdv / R[2:, None], L[:, None] * Yref
