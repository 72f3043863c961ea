"""Van de Vusse NMPC closed loop (config 5) — restatement of ``closedloop_toolbox_nmpc.m`` for
the reactor of ``VanDeVusse_NMPC.m``.  Oracle; test infrastructure only.

Reference pieces restated here:

* Model: ``nmpc_vandevusse_state.m:43-82`` (identical to ``vandevusse_model.m``): Arrhenius rates
  k1..k3 (``:71-73``) and the three state equations (``:78-82``); outputs are states 2:3
  (``VanDeVusse_NMPC.m:81-84,122``).
* Scenario: ``VanDeVusse_NMPC.m:35-90``: Ts = 0.05 h, nit = 60, u0 = [20 130], x0 = the steady
  state at u0 from fsolve started at [5.1 1.1163 130] (``:62-79``; here Newton's method on the
  analytic Jacobian, the same root), references r (``:89-90``), MV bounds (``:54-55,131-138``),
  OV bounds (``:139-142``, soft: OV MinECR = MaxECR = 1 per the committed tuning file), state
  bounds (``:143-146``), ScaleFactors (``:150-164``), Yref (``:170-185``).
* Closed loop (``closedloop_toolbox_nmpc.m:64-77``): U(:,1) = u0; for i = 2..nit the controller
  acts on X(:,i-1) with last move U(:,i-1) and reference r(:,i); the plant integrates over Ts.
  Open loop (``:79-95``): one controller call at (x0, u0, r(:,end)), MVopt padded with its last
  row, simulated from x0.

What cannot be restated (closed source) and what replaces it — the GPU path uses the SAME
replacements, so this is the oracle it is checked against (parity with MATLAB's nlmpc: unpinned):

* ode15s (plant) and the toolbox's own discretisation of the continuous prediction model are
  replaced by one fixed-step classical RK4 with ``NSUB`` = 10 sub-steps per Ts for both.
* nlmpc's fmincon SQP over multiple-shooting variables is replaced by single-shooting
  Gauss-Newton SQP over the moves: residuals of the documented standard cost
      sum_{i=1..N} sum_j (w^y_j/s^y_j)^2 (y_j(k+i) - r_j)^2
      + sum_{l=0..Nu-1} sum_j (w^du_j/s^u_j)^2 du_j(k+l)^2          (MVs held after Nu)
  with exact sensitivities of the RK4 map, MV bounds hard; each QP is a bounded least-squares
  problem (scipy ``lsq_linear``, BVLS: an exact active-set method) in the ABSOLUTE moves
  (the device works in increments: a different parametrisation of the same QP).  Warm start:
  the previous step's solution shifted by one move.  Each Gauss-Newton step is globalised by
  Armijo backtracking on the cost (c1 = 1e-4, up to ``LS_MAX`` halvings, cost changes below
  1e-14 relative count as no increase; pure Gauss-Newton
  2-cycles on this reactor's large-residual steps).  Iterate until the full step satisfies
  max_j |step_j|/s^u_j <= ``SQP_TOL`` (then taken in full) or ``SQP_MAX`` iterations.
  Gauss-Newton converges only linearly on this large-residual problem (contraction up to ~0.9 per
  iteration after a setpoint change: 1.1 % of the config-5 grid's simulations needed more than 100
  iterations at some step), so the fixed-point map v -> G(v) = v + d(v) is Anderson-accelerated
  with depth ``AA_DEPTH`` = 1 (a secant step on the last two Gauss-Newton points): with the
  previous pair (d', G(v')), gamma = <df, d>/<df, df> in the absolute moves scaled by 1/s^u
  (df = d - d'), candidate v+ = clip(G(v) - gamma (G(v) - G(v'))); v+ is taken when its cost meets
  the Armijo decrease demanded of the full Gauss-Newton step (f(v+) <= f0 + c1 dd) and its
  predicted states respect the hard state bounds, otherwise the Armijo search on d runs as above.
  The stopping test and the solution (a stationary point of the same problem) are unchanged.
* State bounds (hard in the toolbox, ``VanDeVusse_NMPC.m:143-146``) are linearised along the
  prediction in every Gauss-Newton subproblem (x_min <= x_i + dx_i/du d <= x_max, i = 1..N).
  The OV bounds (``:139-142``) are the same limits on states 2:3, softened (MinECR = MaxECR = 1),
  so the hard ones dominate and no slack is needed.  ``bounds_ok`` reports whether the closed
  loop itself stayed inside them (the linearisation can be violated between iterations).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# nmpc_vandevusse_state.m:43-58
K10, K20, K30 = 1.287e12, 1.287e12, 9.043e9
E1, E2, E3 = -9758.3, -9758.3, -8560.0
DHAB, DHBC, DHAD = -4.20, 11.00, 41.85
RHO, CP, KW, AR, VR = 0.9342, 3.01, 4032.0, 0.215, 10.0
T0, CA0 = 130.0, 5.10

TS = 0.05          # VanDeVusse_NMPC.m:35
NIT = 60           # :36
NX, NY, NU = 3, 2, 2
U0 = np.array([20.0, 130.0])                       # :70
X0_GUESS = np.array([5.1, 1.1163, 130.0])          # :64-67
LB = np.array([0.0, 40.0])                         # :54-55 (Flow, Qlow)
UB = np.array([150.0, 150.0])                      # (Fupp, Qupp)
XMIN = np.array([0.0, 0.0, 40.0])                  # :57
XMAX = np.array([6.0, 1.2, 150.0])                 # :58
SU = UB - LB                                       # :150,155  Urange
SY = XMAX[1:] - XMIN[1:]                           # :151,159  Yrange
TAU_REF = np.array([0.05, 0.0875])                 # :170 Pref (fast)
INK = 4                                            # :41 inK

NSUB = 10          # RK4 sub-steps per Ts
SQP_TOL = 1e-8     # stop when max_j |step_j| / s^u_j <= SQP_TOL
SQP_MAX = 100
AA_DEPTH = 1       # Anderson acceleration of the Gauss-Newton map (0: plain Gauss-Newton + Armijo)
LS_MAX = 12        # Armijo backtracking halvings per iteration (the last alpha is taken regardless)
LS_C1 = 1e-4
LS_FLAT = 1e-14    # cost changes below LS_FLAT * cost count as no increase


def rhs(x, u):
    """nmpc_vandevusse_state.m:64-82."""
    ca, cb, T = x
    fov, tk = u
    k1 = K10 * np.exp(E1 / (T + 273.15))
    k2 = K20 * np.exp(E2 / (T + 273.15))
    k3 = K30 * np.exp(E3 / (T + 273.15))
    return np.array([
        fov * (CA0 - ca) - k1 * ca - k3 * ca * ca,
        -fov * cb + k1 * ca - k2 * cb,
        (1.0 / (RHO * CP)) * (k1 * ca * DHAB + k2 * cb * DHBC + k3 * ca * ca * DHAD)
        + fov * (T0 - T) + (KW * AR / (RHO * CP * VR)) * (tk - T),
    ])


def jac(x, u):
    """Analytic [df/dx | df/du] (3 x 5) of rhs."""
    ca, cb, T = x
    fov, tk = u
    th = T + 273.15
    k1 = K10 * np.exp(E1 / th)
    k2 = K20 * np.exp(E2 / th)
    k3 = K30 * np.exp(E3 / th)
    d1, d2, d3 = -E1 / th ** 2 * k1, -E2 / th ** 2 * k2, -E3 / th ** 2 * k3  # dk/dT
    a = 1.0 / (RHO * CP)
    b = KW * AR / (RHO * CP * VR)
    J = np.zeros((3, 5))
    J[0] = [-fov - k1 - 2 * k3 * ca, 0.0, -d1 * ca - d3 * ca * ca, CA0 - ca, 0.0]
    J[1] = [k1, -fov - k2, d1 * ca - d2 * cb, -cb, 0.0]
    J[2] = [a * (k1 * DHAB + 2 * k3 * ca * DHAD), a * k2 * DHBC,
            a * (d1 * ca * DHAB + d2 * cb * DHBC + d3 * ca * ca * DHAD) - fov - b, T0 - T, b]
    return J


def rk4(x, u, sens=None):
    """One Ts of classical RK4 with NSUB sub-steps.  sens: optional (3 x k) tangent of x and
    (2 x k) tangent of u, propagated exactly through the RK4 map (forward mode)."""
    h = TS / NSUB
    x = np.array(x, dtype=float)
    if sens is None:
        for _ in range(NSUB):
            k1 = rhs(x, u)
            k2 = rhs(x + 0.5 * h * k1, u)
            k3 = rhs(x + 0.5 * h * k2, u)
            k4 = rhs(x + h * k3, u)
            x = x + (h / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        return x
    X, Ud = sens
    X = np.array(X, dtype=float)
    for _ in range(NSUB):
        xs, Xs = x, X
        k1 = rhs(xs, u)
        J1 = jac(xs, u)
        K1 = J1[:, :3] @ Xs + J1[:, 3:] @ Ud
        xs2, Xs2 = x + 0.5 * h * k1, X + 0.5 * h * K1
        k2 = rhs(xs2, u)
        J2 = jac(xs2, u)
        K2 = J2[:, :3] @ Xs2 + J2[:, 3:] @ Ud
        xs3, Xs3 = x + 0.5 * h * k2, X + 0.5 * h * K2
        k3 = rhs(xs3, u)
        J3 = jac(xs3, u)
        K3 = J3[:, :3] @ Xs3 + J3[:, 3:] @ Ud
        xs4, Xs4 = x + h * k3, X + h * K3
        k4 = rhs(xs4, u)
        J4 = jac(xs4, u)
        K4 = J4[:, :3] @ Xs4 + J4[:, 3:] @ Ud
        x = x + (h / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        X = X + (h / 6.0) * (K1 + 2 * K2 + 2 * K3 + K4)
    return x, X


def steady_state(u=U0, x=X0_GUESS, iters=50):
    """X0 = fsolve(@(x) model(ts,x,u0), X0) (VanDeVusse_NMPC.m:78): Newton on rhs(x, u) = 0."""
    x = np.array(x, dtype=float)
    for _ in range(iters):
        f = rhs(x, u)
        dx = np.linalg.solve(jac(x, u)[:, :3], -f)
        x = x + dx
        if np.max(np.abs(dx) / np.maximum(1.0, np.abs(x))) < 1e-15:
            break
    return x


def references(x0, nit=NIT):
    """r (VanDeVusse_NMPC.m:89-90, 1-based columns) and Yref = lsim(Pref, r - x0(xc)) + x0(xc)
    (:180-185): lsim of a continuous first-order lag with a ZOH input is exact:
    y[k+1] = a y[k] + (1 - a) e[k], a = exp(-Ts/tau), y[0] = 0."""
    r = np.zeros((NY, nit))
    r[0, :] = x0[1]
    r[0, 9:] = 1.0
    r[0, 19:] = 1.0
    r[1, :] = x0[2]
    r[1, 40:] = 130.0
    e = r - x0[1:, None]
    yref = np.zeros_like(r)
    for j in range(NY):
        a = np.exp(-TS / TAU_REF[j])
        for k in range(1, nit):
            yref[j, k] = a * yref[j, k - 1] + (1.0 - a) * e[j, k - 1]
    return r, yref + x0[1:, None]


@dataclass
class NMPCResult:
    y: np.ndarray       # NY x nit
    u: np.ndarray       # NU x nit
    yopt: np.ndarray    # NY x nit (open loop)
    uopt: np.ndarray    # NU x nit
    sqp_iters: int
    bounds_ok: bool


def predict(x, U, N, Nu, want_sens=True, states=False):
    """Outputs y(k+1..k+N) (N x NY) for absolute moves U (Nu x NU, held after Nu-1) and their
    sensitivities dY/dU (N x NY x (Nu*NU), column n*Nu + l); states=True also returns the
    predicted states (N x 3) and their sensitivities (N x 3 x M)."""
    M = NU * Nu
    X = np.zeros((3, M))
    Y = np.zeros((N, NY))
    S = np.zeros((N, NY, M))
    XP = np.zeros((N, 3))
    SX = np.zeros((N, 3, M))
    for i in range(N):
        li = min(i, Nu - 1)
        u = U[li]
        if want_sens:
            Ud = np.zeros((2, M))
            for n in range(NU):
                Ud[n, n * Nu + li] = 1.0
            x, X = rk4(x, u, (X, Ud))
            S[i] = X[1:]
            SX[i] = X
        else:
            x = rk4(x, u)
        Y[i] = x[1:]
        XP[i] = x
    if states:
        return Y, S, XP, SX
    return Y, S


def cost(x, U, u_last, rvec, N, Nu, wy, wu):
    """Objective of one controller call: 1/2 the standard cost (residual form)."""
    Y, _ = predict(x, U, N, Nu, want_sens=False)
    du = np.diff(np.vstack([u_last[None, :], U]), axis=0)
    return 0.5 * float(np.sum(((Y - rvec[None, :]) * wy[None, :]) ** 2) + np.sum((du * wu[None, :]) ** 2))


def controller(x, u_last, rvec, N, Nu, delta, lam, U_init, xbounds=None, return_step=False):
    """One nlmpcmove restated (see module docstring).  xbounds = (x_min, x_max): hard state
    bounds (VanDeVusse_NMPC.m:143-146; the OV bounds of :139-142 are the same limits on states
    2:3, softened, so the hard ones dominate), linearised along the prediction in every
    Gauss-Newton subproblem.  Returns (U, iterations).

    On convergence (max |d| / s_u <= SQP_TOL) the iterate v is returned.  return_step=True
    returns clip(v + d) instead, the convention of rounds 1-3.  Which of the two nlmpcmove's
    fmincon returns is not public and no fixture pins it: parity unpinned.  The two
    differ by at most SQP_TOL s_u in one call; tests/test_nmpc.py bounds their closed-loop drift."""
    from scipy.optimize import lsq_linear

    from .toolbox_band import qp_dual_dense

    wy = np.abs(delta) / SY          # toolbox weights over ScaleFactors, squared in the cost
    wu = np.abs(lam) / SU
    U = np.array(U_init, dtype=float).reshape(Nu, NU)
    M = NU * Nu
    su = np.repeat(SU, Nu)
    it = 0
    hist = None    # Anderson history: (d, G(v)) of the previous iteration
    for it in range(1, SQP_MAX + 1):
        Y, S, XP, SX = predict(x, U, N, Nu, states=True)
        # residuals: outputs (i, j) then moves (n, l), variables v[n*Nu + l] = U[l, n]
        ry = ((Y - rvec[None, :]) * wy[None, :]).reshape(-1)
        Jy = (S * wy[None, :, None]).reshape(N * NY, M)
        du = np.diff(np.vstack([u_last[None, :], U]), axis=0)      # Nu x NU
        ru = np.zeros(M)
        Ju = np.zeros((M, M))
        for n in range(NU):
            for l in range(Nu):
                m = n * Nu + l
                ru[m] = wu[n] * du[l, n]
                Ju[m, m] = wu[n]
                if l > 0:
                    Ju[m, m - 1] = -wu[n]
        A = np.vstack([Jy, Ju])
        res = np.concatenate([ry, ru])
        v = U.T.reshape(-1)
        lo = np.repeat(LB, Nu) - v
        hi = np.repeat(UB, Nu) - v
        lo = np.minimum(lo, 0.0)   # the iterate is feasible up to rounding
        hi = np.maximum(hi, 0.0)
        d = lsq_linear(A, -res, bounds=(lo, hi), method="bvls", tol=1e-14, lsmr_tol=None).x
        if xbounds is not None:
            # linearised state rows  x_min <= x_i + SX_i d <= x_max  (i = 1..N); when the bounded
            # least-squares step violates one, the whole QP is re-solved with them (unique optimum)
            xmn, xmx = (np.asarray(b_, dtype=float) for b_ in xbounds)
            rows, rhs = [], []
            for i in range(N):
                for s in range(3):
                    if np.isfinite(xmn[s]):
                        rows.append(SX[i, s]); rhs.append(xmn[s] - XP[i, s])
                    if np.isfinite(xmx[s]):
                        rows.append(-SX[i, s]); rhs.append(XP[i, s] - xmx[s])
            if rows:
                Ac, bc = np.array(rows), np.array(rhs)
                if np.min(Ac @ d - bc) < -1e-10 * max(1.0, float(np.max(np.abs(bc)))):
                    I = np.eye(M)
                    Aall = np.vstack([I, -I, Ac])
                    ball = np.concatenate([lo, -hi, bc])
                    d, _, _ = qp_dual_dense(A, res, Aall, ball, qr=True)
        lo_b, hi_b = np.repeat(LB, Nu), np.repeat(UB, Nu)
        if np.max(np.abs(d) / su) <= SQP_TOL:
            # converged: the iterate itself is returned (not v + d, |d| <= SQP_TOL s_u), so the
            # device can run the next call's first prediction from it alongside its last trial
            # pass (nmpc_kernel.hip mpass)
            if return_step:
                U = np.clip(v + d, np.repeat(LB, Nu), np.repeat(UB, Nu)).reshape(NU, Nu).T.copy()
            break
        # Armijo backtracking on the cost along the Gauss-Newton step: pure Gauss-Newton 2-cycles
        # on the large-residual steps of this reactor (e.g. after the setpoint change)
        f0 = 0.5 * float(res @ res)
        dd = float(res @ (A @ d))      # directional derivative of the cost along d (< 0)
        g = v + d
        prev, hist = hist, (d.copy(), g.copy())
        if AA_DEPTH > 0 and prev is not None:
            df = (d - prev[0]) / su
            den = float(df @ df)
            if den > 0.0:
                gam = float(df @ (d / su)) / den
                vc = np.clip(g - gam * (g - prev[1]), lo_b, hi_b)
                Uc = vc.reshape(NU, Nu).T
                fc = cost(x, Uc, u_last, rvec, N, Nu, wy, wu)
                ok = True
                if xbounds is not None:
                    xmn, xmx = (np.asarray(b_, dtype=float) for b_ in xbounds)
                    XPc = predict(x, Uc, N, Nu, want_sens=False, states=True)[2]
                    ok = bool(np.all(XPc >= xmn[None, :]) and np.all(XPc <= xmx[None, :]))
                if ok and fc <= f0 + LS_C1 * dd:
                    v = vc
                    U = Uc.copy()
                    continue
        alpha = 1.0
        for _ in range(LS_MAX):
            va = np.clip(v + alpha * d, lo_b, hi_b)
            f1 = cost(x, va.reshape(NU, Nu).T, u_last, rvec, N, Nu, wy, wu)
            # sufficient decrease, or no increase beyond the rounding of the cost itself (the
            # Armijo test is meaningless once alpha*dd is below it)
            if f1 <= f0 + LS_C1 * alpha * dd or f1 - f0 <= LS_FLAT * f0:
                break
            alpha *= 0.5
        v = np.clip(v + alpha * d, lo_b, hi_b)
        U = v.reshape(NU, Nu).T.copy()
    return U, it


def closedloop_nmpc(r, N: int, Nu: int, delta, lam, nit: int = NIT, x0=None, u0=U0,
                    open_loop: bool = True, xbounds=(XMIN, XMAX), return_step: bool = False) -> NMPCResult:
    """[y,u,yopt,uopt] = closedloop_toolbox_nmpc(nmpcobj,model,init,r,N,Nu,delta,lambda,nit)."""
    x0 = steady_state() if x0 is None else np.asarray(x0, dtype=float)
    r = np.asarray(r, dtype=float).reshape(NY, nit)
    X = np.zeros((NX, nit))
    Y = np.zeros((NY, nit))
    U = np.zeros((NU, nit))
    X[:, 0] = x0
    Y[:, 0] = x0[1:]
    U[:, 0] = u0
    Uw = np.tile(np.asarray(u0, dtype=float), (Nu, 1))
    iters = 0
    for i in range(1, nit):
        Uw, it = controller(X[:, i - 1], U[:, i - 1], r[:, i], N, Nu, delta, lam, Uw, xbounds, return_step)
        iters += it
        U[:, i] = Uw[0]
        X[:, i] = rk4(X[:, i - 1], U[:, i])
        Y[:, i] = X[1:, i]
        Uw = np.vstack([Uw[1:], Uw[-1:]])            # warm start: shift by one move
    xmn, xmx = (np.asarray(b_, dtype=float) for b_ in (xbounds if xbounds is not None else (XMIN, XMAX)))
    ok = bool(np.all(X >= xmn[:, None] - 1e-9) and np.all(X <= xmx[:, None] + 1e-9))
    yopt = uopt = None
    if open_loop:
        Uo, it = controller(x0, np.asarray(u0, dtype=float), r[:, -1], N, Nu, delta, lam,
                            np.tile(np.asarray(u0, dtype=float), (Nu, 1)), xbounds, return_step)
        iters += it
        # MVopt: p+1 rows (moves held after Nu), padded with its last row to nit
        uo = np.array([Uo[min(k, Nu - 1)] for k in range(nit)])
        uopt = uo.T.copy()
        Xo = np.zeros((NX, nit))
        Xo[:, 0] = x0
        yopt = np.zeros((NY, nit))
        yopt[:, 0] = x0[1:]
        for i in range(1, nit):
            Xo[:, i] = rk4(Xo[:, i - 1], uopt[:, i])
            yopt[:, i] = Xo[1:, i]
    return NMPCResult(Y, U, yopt, uopt, iters, ok)
