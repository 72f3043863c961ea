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
