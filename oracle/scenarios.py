"""Scenario definitions transcribed from the reference driver scripts (oracle; tests only).

Shell 3x3 (config 2, the metric): MPC-Tuning/Shell3x3.m with caso = 2, nominal = true,
rest = true; scaling L, R from the committed MPC-Tuning/Shell3x3_Tuning_25Jul2023_12_06.mat
(CondMin's fmincon result is not reproducible: cond() is scale invariant).
"""
from __future__ import annotations

import json
import os

import numpy as np

from .matlab import DTF, c2d_zoh, lsim_dtf
from .toolbox_gpc import Scenario

_FX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "tuning_parameters_mat.json")

# Shell3x3.m:52-57 nominal model
SHELL3_K = np.array([[4.05, 1.77, 5.88], [5.39, 5.72, 6.9], [4.38, 4.42, 7.2]])
SHELL3_TAU = np.array([[50, 60, 50], [50, 60, 40], [33, 44, 19]], dtype=float)
SHELL3_L = np.array([[27, 28, 27], [18, 14, 15], [20, 22, 0]], dtype=float)
SHELL3_TS = 4.0
SHELL3_NIT = 500


def load_fixture(key="shell3x3_25jul2023"):
    with open(_FX) as f:
        return json.load(f)[key]


def shell3x3_xsp(nit=SHELL3_NIT):
    """Shell3x3.m:89-92 (1-based inclusive ranges; later assignments overwrite)."""
    X = np.zeros((3, nit))

    def put(i, a, b, val):
        X[i, a - 1: b] = val

    inK = 10
    put(0, inK, 80, 0.2); put(0, 80, 200, 0.0); put(0, 200, 400, 0.1); put(0, 400, 500, 0.0)
    put(1, inK, 80, 0.2); put(1, 80, 200, 0.4); put(1, 200, 400, 0.3); put(1, 400, 500, 0.0)
    put(2, inK, 80, 0.2); put(2, 80, 200, 0.1); put(2, 200, 400, 0.0); put(2, 400, 500, 0.0)
    return X[:, :nit]


def shell3x3_yref(X, caso=2):
    """Shell3x3.m:71-76,98-99: Yref = lsim(Pref, Xsp, t, 'zoh'), Pref diagonal first order."""
    taus = [5, 9, 5.7] if caso == 1 else [30, 30, 30]
    delays = [27, 14, 0]
    Y = np.zeros_like(X)
    for i in range(3):
        Y[i] = lsim_dtf(c2d_zoh([1.0], [taus[i], 1.0], SHELL3_TS, delays[i]), X[i])
    return Y


def shell3x3_plant_scaled(L, R):
    """Pze = L * c2d(Ps, Ts, 'zoh') * R  (Shell3x3.m:65, MPCTuning.m:162)."""
    P = []
    for i in range(3):
        row = []
        for j in range(3):
            d = c2d_zoh([SHELL3_K[i, j]], [SHELL3_TAU[i, j], 1.0], SHELL3_TS, SHELL3_L[i, j])
            row.append(d.scaled(L[i] * R[j]))
        P.append(row)
    return P


def shell3x3(window="toolbox", weights_squared=True, round_roots=False):
    """Return (Scenario, r (scaled Xsp), yref (scaled), fixture dict)."""
    fx = load_fixture()
    L = np.array(fx["scale"]["L"])
    R = np.array(fx["scale"]["R"])
    P = shell3x3_plant_scaled(L, R)
    # Shell3x3.m:120-123 bounds, scaled by R (MPCTuning.m:170-178)
    du = 0.05 / R
    umx = 0.5 / R
    umn = -1.0 / R
    sc = Scenario(plant=P, model=P, nu=3, du_min=-du, du_max=du, u_min=umn, u_max=umx,
                  window=window, weights_squared=weights_squared, round_roots=round_roots)
    X = shell3x3_xsp()
    Yref = shell3x3_yref(X)
    r = L[:, None] * X          # MPCTuning.m:189
    yref = L[:, None] * Yref    # MPCTuning.m:188
    return sc, r, yref, fx


def vns_step_refs(my, nit, inK=10):
    """VNS2.m:58-61,147-150: Xsp(1:my,inK:end) = 1 and sel picks one output per simulation."""
    refs = []
    for i in range(my):
        X = np.zeros((my, nit))
        X[i, inK - 1:] = 1.0
        refs.append(X)
    return refs


def candidate_grid(C=4096, my=3, nu=3, N2=30, Nu=5, seed=20250307, fx=None):
    """log10 delta ~ U(-4,0), log10 lambda ~ U(-5,-1), default_rng(seed);
    candidate 0 = the fixture-tuned point (delta, lambda) at N2=30, Nu=5."""
    rng = np.random.default_rng(seed)
    delta = 10.0 ** rng.uniform(-4, 0, size=(C, my))
    lam = 10.0 ** rng.uniform(-5, -1, size=(C, nu))
    if fx is not None:
        delta[0] = fx["delta"]
        lam[0] = fx["lambda"]
    N2v = np.full(C, N2, dtype=np.int32)
    Nuv = np.full(C, Nu, dtype=np.int32)
    return N2v, Nuv, delta, lam


# ---------------------------------------------------------------------------------------------
# Shell 7x5 (config 3): MPC-Tuning/Shell7x5.m, nominal = true (e1..e5 = 0, :38-43)
SHELL7_K = np.array([[4.05, 1.77, 5.88, 1.20, 1.44], [5.39, 5.72, 6.9, 1.52, 1.83],
                     [3.66, 1.65, 5.53, 1.16, 1.27], [5.92, 2.54, 8.10, 1.73, 1.79],
                     [4.13, 2.38, 6.23, 1.31, 1.26], [4.06, 4.18, 6.53, 1.19, 1.17],
                     [4.38, 4.42, 7.2, 1.14, 1.26]])          # Shell7x5.m:73-91 [Gs Ds]
SHELL7_TAU = np.array([[50, 60, 50, 45, 40], [50, 60, 40, 25, 20], [9, 30, 40, 11, 6],
                       [12, 27, 20, 5, 19], [8, 19, 10, 2, 22], [13, 33, 9, 19, 24],
                       [33, 44, 19, 24, 32]], dtype=float)
SHELL7_L = np.array([[27, 28, 27, 27, 27], [18, 14, 15, 15, 15], [2, 20, 2, 0, 0], [11, 12, 2, 0, 0],
                     [5, 7, 2, 0, 0], [8, 4, 1, 0, 0], [20, 22, 0, 0, 0]], dtype=float)
SHELL7_TS = 4.0
SHELL7_NIT = 200
SHELL7_YMX = np.array([0.005, 0.005, 0.5, 0.5, 0.5, 0.5, 0.5])   # Shell7x5.m:106-107
SHELL7_ECR = np.array([0.1, 0.5, 1, 1, 1, 1, 1])                   # Shell7x5.m:143-152


def shell7x5_plant_scaled(L, R):
    """Pze = L * c2d([Gs Ds], Ts, 'zoh') * R  (Shell7x5.m:93-98, MPCTuning.m:162)."""
    return [[c2d_zoh([SHELL7_K[i, j]], [SHELL7_TAU[i, j], 1.0], SHELL7_TS, SHELL7_L[i, j]).scaled(L[i] * R[j])
             for j in range(5)] for i in range(7)]


def shell7x5_yref(nit=SHELL7_NIT, tmd=20):
    """Shell7x5.m:128-135: Xref(i, tmd:tmd+5) = Ymx(i); Yref = lsim(Pref, Xref, t, 'zoh'), Pref =
    blkdiag of 1/(50s+1) with iodelay = min over row i of Ps.iodelay (Gs and Ds columns)."""
    X = np.zeros((7, nit))
    X[:, tmd - 1: tmd + 5] = SHELL7_YMX[:, None]
    dl = SHELL7_L.min(axis=1)
    Y = np.zeros_like(X)
    for i in range(7):
        Y[i] = lsim_dtf(c2d_zoh([1.0], [50.0, 1.0], SHELL7_TS, dl[i]), X[i])
    return Y


def shell7x5(nit=SHELL7_NIT):
    """Return (BandScenario, r = L*Xsp (zeros), v = Rv\\mdv, yref = L*Yref, fixture)."""
    from .toolbox_band import BandScenario

    fx = load_fixture("shell7x5_14sep2024")
    L = np.array(fx["scale"]["L"])
    R = np.array(fx["scale"]["R"])
    P = shell7x5_plant_scaled(L, R)
    Ru, Rv = R[:3], R[3:]
    # MV bounds Shell7x5.m:110-111,135-138 scaled (MPCTuning.m:170-178); no rate bounds
    umx = 0.5 / Ru
    inf = np.full(3, np.inf)
    # OV ScaleFactor = Yrange (Shell7x5.m:162-168); MPCTuning.m:182-184 multiplies by L only
    # when the factor is not 1 (Yrange = 1 for outputs 3..7 stays 1)
    yr = 2 * SHELL7_YMX
    sy = np.where(yr != 1.0, L * yr, yr)
    su = np.ones(3)                      # Urange = 1 -> unchanged
    sc = BandScenario(plant=P, nu=3, du_min=-inf, du_max=inf, u_min=-umx, u_max=umx,
                      y_min=-L * SHELL7_YMX, y_max=L * SHELL7_YMX, ecr_min=SHELL7_ECR.copy(),
                      ecr_max=SHELL7_ECR.copy(), sy=sy, su=su, rho=1e4)
    r = np.zeros((7, nit))                                   # L*Xsp, Xsp = 0 (Shell7x5.m:118)
    mdv = np.zeros((2, nit))
    mdv[:, 19:] = 0.5                                        # Shell7x5.m:121-123 (1-based 20:end)
    v = mdv / Rv[:, None]                                    # MPCTuning.m:191
    yref = L[:, None] * shell7x5_yref(nit)                   # MPCTuning.m:188
    return sc, r, v, yref, fx


# ---------------------------------------------------------------------------------------------
# WoodBerry.m toolbox MPC (caso 1, nominal, rest): one measured disturbance, no output bounds.
# No committed WoodBerry .mat: CondMin's scaling is not pinned, L = R = I.
WB_K = np.array([[12.8, -18.9, 3.8], [6.6, -19.4, 4.9]])          # WoodBerry.m:48-52
WB_TAU = np.array([[16.7, 21.0, 14.9], [10.9, 14.4, 13.2]])
WB_L = np.array([[1.0, 2.0, 8.1], [2.0, 1.0, 3.4]])


def woodberry_toolbox(nit=400):
    """Return (BandScenario, r, v, yref) of WoodBerry.m:43-148 (see mpct.scenarios)."""
    from .toolbox_band import BandScenario

    P = [[c2d_zoh([WB_K[i, j]], [WB_TAU[i, j], 1.0], 1.0, WB_L[i, j]) for j in range(3)] for i in range(2)]
    inf = np.full(2, np.inf)
    sc = BandScenario(plant=P, nu=2, du_min=np.full(2, -0.05), du_max=np.full(2, 0.05),
                      u_min=np.full(2, -0.5), u_max=np.full(2, 0.5), y_min=-inf, y_max=inf,
                      ecr_min=np.ones(2), ecr_max=np.ones(2), sy=np.ones(2), su=np.ones(2), rho=1e4)
    X = np.zeros((2, nit))
    X[0, 9:] = 0.8
    X[1, 199:] = 0.5
    Y = np.stack([lsim_dtf(c2d_zoh([1.0], [tau, 1.0], 1.0, 1.0), X[i]) for i, tau in enumerate((10.0, 7.0))])
    v = np.zeros((1, nit))
    v[0, 299:] = -0.25
    return sc, X, v, Y
