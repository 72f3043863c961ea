"""Nonlinear MPC host mirror (config 5): the Van de Vusse reactor of ``VanDeVusse_NMPC.m`` over the
libmpct C ABI (``mpct_nmpc_scenario_create``, include/mpct.h).

  NmpcScenario              the candidate-independent part of ``closedloop_toolbox_nmpc``'s
                            arguments (nmpcobj constraints / scales, model, init, Yref)
  vandevusse()              the driver's scenario (``VanDeVusse_NMPC.m:35-185``)
  closedloop_toolbox_nmpc   drop-in for ``closedloop_toolbox_nmpc.m:1`` (one candidate)

Evaluate batches with ``mpct.engine.eval_batch`` / ``eval_batch_device`` exactly as for the
linear scenarios (N2 := N).  Every closed loop runs in ``nmpc_kernel.hip``; the only host
arithmetic here is the scenario setup: the steady state x0 (``fsolve`` at u0, :78) and the
reference trajectory Yref (:180-185).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .engine import MpctError, eval_batch

# nmpc_vandevusse_state.m:43-58, in the ABI's params order
VDV_PARAMS = np.array([1.287e12, 1.287e12, 9.043e9, -9758.3, -9758.3, -8560.0, -4.20, 11.00, 41.85,
                       0.9342, 3.01, 4032.0, 0.215, 10.0, 130.00, 5.10])
VDV_TS, VDV_NIT = 0.05, 60                       # VanDeVusse_NMPC.m:35-36
VDV_U0 = np.array([20.0, 130.0])                 # :70
VDV_X0_GUESS = np.array([5.1, 1.1163, 130.0])    # :64-67
VDV_UMIN, VDV_UMAX = np.array([0.0, 40.0]), np.array([150.0, 150.0])        # :49-55
VDV_XMIN, VDV_XMAX = np.array([0.0, 0.0, 40.0]), np.array([6.0, 1.2, 150.0])  # :45-58
VDV_XC = (2, 3)                                   # :82 (1-based)
VDV_TAU_REF = np.array([0.05, 0.0875])            # :170 Pref (fast)
# VanDeVusse_NMPC_Tuning_25Jul2023_11_04.mat / _06Dec2023_09_50.mat (identical): the tuned point
VDV_TUNED = dict(N=3, Nu=(2, 2), delta=(0.09302224780430422, 0.11333840205801392),
                 lam=(0.245996189227521, 0.12310801096548595))
VDV_W = np.array([0.7, 0.3])                      # :202 Pareto weights


def _vdv_rhs_jac(x, u, p=VDV_PARAMS):
    k10, k20, k30, e1, e2, e3, dab, dbc, dad, rho, cp, kw, ar, vr, t0, ca0 = p
    ca, cb, T = x
    th = T + 273.15
    k1, k2, k3 = k10 * np.exp(e1 / th), k20 * np.exp(e2 / th), k30 * np.exp(e3 / th)
    d1, d2, d3 = -e1 / th ** 2 * k1, -e2 / th ** 2 * k2, -e3 / th ** 2 * k3
    a, b = 1.0 / (rho * cp), kw * ar / (rho * cp * vr)
    fov, tk = u
    f = np.array([fov * (ca0 - ca) - k1 * ca - k3 * ca * ca,
                  -fov * cb + k1 * ca - k2 * cb,
                  a * (k1 * ca * dab + k2 * cb * dbc + k3 * ca * ca * dad) + fov * (t0 - T) + b * (tk - T)])
    J = np.array([[-fov - k1 - 2 * k3 * ca, 0.0, -d1 * ca - d3 * ca * ca],
                  [k1, -fov - k2, d1 * ca - d2 * cb],
                  [a * (k1 * dab + 2 * k3 * ca * dad), a * k2 * dbc,
                   a * (d1 * ca * dab + d2 * cb * dbc + d3 * ca * ca * dad) - fov - b]])
    return f, J


def steady_state(u0=VDV_U0, x=VDV_X0_GUESS, params=VDV_PARAMS):
    """X0 = fsolve(@(x) model(ts,x,u0), X0) (VanDeVusse_NMPC.m:78), by Newton's method."""
    x = np.array(x, dtype=float)
    for _ in range(50):
        f, J = _vdv_rhs_jac(x, u0, params)
        dx = np.linalg.solve(J, -f)
        x = x + dx
        if np.max(np.abs(dx) / np.maximum(1.0, np.abs(x))) < 1e-15:
            break
    return x


def vandevusse_signals(x0, nit=VDV_NIT, ts=VDV_TS):
    """r (VanDeVusse_NMPC.m:89-90) and Yref = lsim(Pref, r - x0(xc), t, 'zoh') + x0(xc) (:180-185)."""
    r = np.zeros((2, nit))
    r[0, :] = x0[1]
    r[0, 9:] = 1.0
    r[1, :] = x0[2]
    r[1, 40:] = 130.0
    e = r - x0[1:, None]
    yref = np.zeros_like(r)
    for j in range(2):
        a = np.exp(-ts / VDV_TAU_REF[j])
        for k in range(1, nit):
            yref[j, k] = a * yref[j, k - 1] + (1.0 - a) * e[j, k - 1]
    return r, yref + x0[1:, None]


class NmpcScenario:
    """Candidate-independent NMPC description (MPCTuning's Par for a nonlinear model)."""

    def __init__(self, x0, u0, u_min, u_max, x_min, x_max, yref, n_max, nu_max, ts=VDV_TS, nsub=10,
                 xc=VDV_XC, params=VDV_PARAMS, y_scale=None, u_scale=None, vns_ink=10, sqp_max=100,
                 sqp_tol=1e-8):
        self.lib = _lib.load()
        self.yref = np.ascontiguousarray(np.asarray(yref, dtype=float).reshape(len(xc), -1))
        self.my, self.nu, self.nd, self.nq = len(xc), 2, 0, 0
        self.nit = self.yref.shape[1]
        self.n2_max, self.nu_max = int(n_max), int(nu_max)
        self.Ts = float(ts)
        x_min, x_max = np.asarray(x_min, float), np.asarray(x_max, float)
        xcz = np.asarray(xc, dtype=np.int32) - 1
        # ScaleFactors (VanDeVusse_NMPC.m:150-164): ranges of the bounds
        ys = np.asarray(y_scale if y_scale is not None else (x_max - x_min)[xcz], dtype=float)
        us = np.asarray(u_scale if u_scale is not None else np.asarray(u_max, float) - np.asarray(u_min, float),
                        dtype=float)
        arrs = dict(params=params, x0=x0, u0=u0, u_min=u_min, u_max=u_max, x_min=x_min, x_max=x_max,
                    y_scale=ys, u_scale=us)
        self._keep = {k: np.ascontiguousarray(np.asarray(v, dtype=float)) for k, v in arrs.items()}
        self._keep["xc"] = np.ascontiguousarray(np.asarray(xc, dtype=np.int32))
        self._keep["yref"] = self.yref
        d = _lib.MpctNmpcDesc()
        d.abi_version = _lib.ABI_VERSION
        d.model = _lib.NMPC_VANDEVUSSE
        d.nx, d.ny, d.nu = 3, self.my, 2
        d.params = self._keep["params"].ctypes.data_as(_lib.c_double_p)
        d.xc = self._keep["xc"].ctypes.data_as(_lib.c_int32_p)
        d.ts, d.nsub = self.Ts, int(nsub)
        for k in ("x0", "u0", "u_min", "u_max", "x_min", "x_max", "y_scale", "u_scale"):
            setattr(d, k, self._keep[k].ctypes.data_as(_lib.c_double_p))
        d.n_max, d.nu_max, d.nit = self.n2_max, self.nu_max, self.nit
        d.yref = self.yref.ctypes.data_as(_lib.c_double_p)
        d.vns_ink, d.sqp_max, d.sqp_tol = int(vns_ink), int(sqp_max), float(sqp_tol)
        h = C.c_void_p()
        rc = self.lib.mpct_nmpc_scenario_create(C.byref(d), C.byref(h))
        if rc != 0:
            raise MpctError("mpct_nmpc_scenario_create failed (%d): %s" % (rc, _lib.last_error()))
        self._h = h
        self.x0 = self._keep["x0"]
        self.u0 = self._keep["u0"]

    @property
    def handle(self):
        return self._h

    def lds_bytes(self, N=None, Nu=None) -> int:
        return int(self.lib.mpct_lds_bytes(self._h, N or self.n2_max, Nu or self.nu_max))

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mpct_scenario_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def vandevusse(n_max=31, nu_max=15, nit=VDV_NIT, nsub=10):
    """The VanDeVusse_NMPC.m scenario (rest = true, caso = 1, nominal): returns (sc, r, yref)."""
    x0 = steady_state()
    r, yref = vandevusse_signals(x0, nit)
    sc = NmpcScenario(x0, VDV_U0, VDV_UMIN, VDV_UMAX, VDV_XMIN, VDV_XMAX, yref, n_max, nu_max, nsub=nsub)
    return sc, r, yref


def nmpc_candidate_grid(C=4096, seed=20250307, n_max=31, nu_max=15, tuned=VDV_TUNED):
    """Config 5 grid: N in 2..31, Nu in 2..min(N-1, 15), log10 delta ~ U(-2, 1),
    log10 lambda ~ U(-3, 0); candidate 0 is the committed tuning (N = 3, Nu = 2)."""
    rng = np.random.default_rng(seed)
    N = rng.integers(3, n_max + 1, size=C).astype(np.int32)
    Nu = np.array([rng.integers(2, min(n - 1, nu_max) + 1) for n in N], dtype=np.int32)
    d = 10.0 ** rng.uniform(-2, 1, size=(C, 2))
    lam = 10.0 ** rng.uniform(-3, 0, size=(C, 2))
    if tuned is not None and C > 0:
        N[0], Nu[0] = tuned["N"], max(tuned["Nu"])
        d[0], lam[0] = tuned["delta"], tuned["lam"]
    return N, Nu, d, lam


def closedloop_toolbox_nmpc(sc: NmpcScenario, r, N, Nu, delta, lam, nit=None):
    """[y,u,yopt,uopt] = closedloop_toolbox_nmpc(nmpcobj,model,init,r,N,Nu,delta,lambda,nit)
    (closedloop_toolbox_nmpc.m:1); N, Nu may be vectors (max taken, :47-50)."""
    nit = sc.nit if nit is None else int(nit)
    if nit != sc.nit:
        raise ValueError("scenario was built for nit=%d" % sc.nit)
    res = eval_batch(sc, [int(np.max(N))], [int(np.max(Nu))], np.reshape(delta, (1, -1)),
                     np.reshape(lam, (1, -1)), np.asarray(r, dtype=float)[None], open_loop=True, want_traj=True)
    return res.y[0], res.u[0], res.ys[0], res.uopt[0]
