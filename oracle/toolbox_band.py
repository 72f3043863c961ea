"""Toolbox-equivalent closed loop with measured disturbances and soft output bands — restatement
of ``closedloop_toolbox.m`` for the Shell 7x5 configuration (config 3, ``Shell7x5.m``).

Oracle; test infrastructure only.  The MPC Toolbox is closed source; this file restates the
QP the toolbox documents for a linear ``mpc`` object, specialised to what ``Shell7x5.m:112-196``
and ``MPCTuning.m:162-199`` configure:

* Model ``Pze = L*c2d([Gs Ds],Ts)*R`` with MV columns 0..nu-1 and MD columns nu.. (setmpcsignals
  MV=[1;2;3], MD=[4;5], ``Shell7x5.m:171-172``).  ``closedloop_toolbox.m:50`` calls
  ``sim(mpc,nit,r,v)`` without a plant override, so the plant IS the model.  Zero initial
  states and no unmeasured disturbance mean the default estimator sees zero innovation, so the
  toolbox's prediction equals the exact model prediction.
* Prediction y(t+k|t), k = 1..p (PredictionHorizon = max(N), ``closedloop_toolbox.m:39``):
  future MVs are u(t-1) plus the cumulative moves (blocked after ControlHorizon = max(Nu)).
  Future MDs are held at the measured v(t) (``mpcsimopt MDLookAhead 'off'``, ``Shell7x5.m:196``).
  Here that prediction is an explicit forward simulation of the model each step (``lsim``
  restated with ``scipy.signal.lfilter`` on the full input history).  It is deliberately not the
  device's incremental shift-and-extend update.
* Cost (documented toolbox form, weights over scale factors):
      sum_i sum_k (w^y_i/s^y_i)^2 (r_i(t) - y_i(t+k|t))^2 + sum_n sum_l (w^du_n/s^u_n)^2 du_n(l)^2
      + rho_eps * eps^2
  with Weights.OV = delta, Weights.MVRate = lambda (``closedloop_toolbox.m:42-43``) and
  Weights.ECR = rho_eps = 10000 (``Shell7x5.m:191``).  Band mode: every OV weight is 0
  (``Shell7x5.m:190``, kept 0 by ``GAM_fun.m:62-66`` / ``MPC_TFob.m:85-86``).
* Constraints: MV amplitude (and rate, when finite) hard.  Outputs are soft with ONE shared
  slack eps >= 0:  y_min_i - eps V^min_i s^y_i <= y_i(t+k|t) <= y_max_i + eps V^max_i s^y_i
  for every k = 1..p, with V = the MinECR/MaxECR of ``Shell7x5.m:143-152`` and s^y the OV
  ScaleFactor after ``MPCTuning.m:182-184``.
* The QP (strictly convex: lambda > 0, rho > 0) is equilibrated (unit Hessian diagonal, unit
  constraint rows: rho*eps outweighs lambda^2*du by ~9 orders of magnitude on Shell 7x5) and
  solved by a dense textbook dual active-set method (``qp_dual_dense``: everything recomputed
  each iteration, no updates, no warm start).  A primal active-set method cycles on the
  ~1.8k near-parallel output rows of the N2 = 127 search range.  Every solution must pass an
  algorithm-independent KKT check (``kkt_residual``: NNLS multipliers on the active rows).
* Open-loop first-move prediction (``closedloop_toolbox.m:85-100``): the QP at the initial
  state with reference r(:,end) and MD v(:,end) held from time 0 gives Info.Uopt, padded to
  nit.  Then ys = lsim(Pz, [uopt v]) with the actual v.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from scipy.signal import lfilter

from .matlab import step_dtf
from .toolbox_gpc import CLResult, constraint_rows


@dataclass
class BandScenario:
    """Candidate-independent part of the band-mode closed loop."""

    plant: list            # my x (nu+nd) DTF (plant == model, closedloop_toolbox.m:50)
    nu: int
    du_min: np.ndarray
    du_max: np.ndarray
    u_min: np.ndarray
    u_max: np.ndarray
    y_min: np.ndarray      # OV Min/Max (scaled by L, MPCTuning.m:180-181)
    y_max: np.ndarray
    ecr_min: np.ndarray    # OV MinECR / MaxECR
    ecr_max: np.ndarray
    sy: np.ndarray         # OV ScaleFactor
    su: np.ndarray         # MV ScaleFactor
    rho: float = 1e4       # Weights.ECR
    weights_squared: bool = True

    @property
    def my(self):
        return len(self.plant)

    @property
    def nin(self):
        return len(self.plant[0])

    @property
    def nd(self):
        return self.nin - self.nu

    def ba(self):
        return [[self.plant[i][j].zinv_form() for j in range(self.nin)] for i in range(self.my)]


def simulate(ba, U, T):
    """Outputs y(0..T-1) of the my x nin model for the input history U (nin x >= T)."""
    my, nin = len(ba), len(ba[0])
    Y = np.zeros((my, T))
    for i in range(my):
        for j in range(nin):
            b, a = ba[i][j]
            if np.any(b):
                Y[i] += lfilter(b, a, U[j, :T])
    return Y


def step_table(sc: BandScenario, n: int):
    """s_ij(0..n-1), unit-step responses of every entry (MatG.m:51 restated)."""
    return np.array([[step_dtf(sc.plant[i][j], n) for j in range(sc.nin)] for i in range(sc.my)])


def dyn_matrix(S, nu, N2, Nu):
    """G[(i,k), (n,l)] = s_in(k + 1 - l) for k = 0..N2-1 (toolbox window t+1..t+N2), moves held
    after l: the MatG.m:64-67 layout with d = 0, columns ordered n*Nu + l."""
    my = S.shape[0]
    G = np.zeros((my * N2, nu * Nu))
    for i in range(my):
        for k in range(N2):
            for n in range(nu):
                for l in range(Nu):
                    if k + 1 - l >= 0:
                        G[i * N2 + k, n * Nu + l] = S[i, n, k + 1 - l]
    return G


def qp_primal_active_set_x0(W, c, Ain, bin_, x0, tol=1e-12, maxit=2000):
    """min 1/2 ||W x + c||^2 s.t. Ain x >= bin from the feasible point x0: the primal
    active-set method of toolbox_gpc.qp_primal_active_set (null-space steps by lstsq, never the
    normal equations) with a vectorised ratio test.  Returns (x, iterations, working set)."""
    M = W.shape[1]
    x = np.array(x0, dtype=float)
    s = Ain @ x - bin_
    if np.any(s < -1e-9 * max(1.0, np.abs(bin_).max())):
        raise ValueError("QP start point infeasible (%g)" % s.min())
    W_ = []
    for i in np.nonzero(s <= tol)[0]:
        cand = W_ + [int(i)]
        if np.linalg.matrix_rank(Ain[cand]) == len(cand):
            W_ = cand
    rownorm = np.max(np.abs(Ain), axis=1)
    for it in range(1, maxit + 1):
        q = len(W_)
        res = W @ x + c
        if q:
            _, _, Vt = np.linalg.svd(Ain[W_])
            Z = Vt[q:].T
        else:
            Z = np.eye(M)
        p = Z @ np.linalg.lstsq(W @ Z, -res, rcond=None)[0] if Z.shape[1] else np.zeros(M)
        Ap = Ain @ p
        s = Ain @ x - bin_
        thr = 1e-12 * np.max(np.abs(p)) * rownorm
        cand = Ap < -thr
        if W_:
            cand[W_] = False
        alpha, block = 1.0, None
        if np.any(cand):
            ratios = np.full(Ain.shape[0], np.inf)
            ratios[cand] = np.maximum(s[cand], 0.0) / (-Ap[cand])
            i = int(np.argmin(ratios))
            if ratios[i] < 1.0:
                alpha, block = float(ratios[i]), i
        x = x + alpha * p
        if block is not None:
            W_.append(block)
            continue
        if q == 0:
            return x, it, W_
        grad = W.T @ (W @ x + c)
        mu = np.linalg.lstsq(Ain[W_].T, grad, rcond=None)[0]
        # absolute test against the (equilibrated) gradient: on Shell 7x5 the multipliers of the
        # rows that hold eps span ~1e8 while a wrong working set shows as mu ~ -1e-1, which any
        # test relative to max|mu| accepts
        if np.all(mu >= -1e-10 * max(1.0, np.max(np.abs(grad)))):
            return x, it, W_
        W_.pop(int(np.argmin(mu)))
    raise RuntimeError("primal active set did not converge")


def qp_dual_dense(W, c, A, b, tol=1e-12, maxit=5000, qr=False):
    """min 1/2 ||W x + c||^2 s.t. A x >= b by the textbook dual method of Goldfarb & Idnani
    (1983), recomputed densely at every iteration: in the coordinates w = L'x (H = W'W = LL')
    the Hessian is I, the primal direction is the projection of n_p onto null(N_A) and the dual
    direction solves N_A' r = n_p, both from a fresh QR of the active rows (never N H^-1 N',
    which squares their conditioning at the near-dependent vertices of the output bands); after
    every addition the iterate is re-solved exactly on the active set.  No factor updates and no
    warm start: the device's J-form / Householder / warm-started variant shares none of this
    arithmetic.  The dual objective increases monotonically, so the ~1.8k near-parallel output
    rows of the N2 = 127 range cannot make it cycle.  Returns (x, iterations, active set).
    qr=True: the factor comes from a QR of W (H = R'R, L = R') instead of a Cholesky of W'W --
    for least-squares problems whose W'W is too ill-conditioned to form (the NMPC's, cond ~1e15)."""
    import scipy.linalg as sla

    if qr:
        Qw, Rw = np.linalg.qr(W)
        L = Rw.T
        gw = Qw.T @ c
    else:
        H = W.T @ W
        g = W.T @ c
        L = np.linalg.cholesky(H)
        gw = sla.solve_triangular(L, g, lower=True)
    Aw = sla.solve_triangular(L, A.T, lower=True).T          # rows of A L^-T
    w = -gw
    act, u = [], np.zeros(0)
    it = 0

    def factor():
        Q, R = np.linalg.qr(Aw[act].T, mode="complete")
        q = len(act)
        return Q[:, :q], Q[:, q:], R[:q, :q]

    while True:
        s = Aw @ w - b
        if act:
            s[act] = np.inf
        p = int(np.argmin(s))
        if not s[p] < -tol * max(1.0, abs(b[p])):
            return sla.solve_triangular(L.T, w, lower=False), it, act
        n = Aw[p]
        up = np.concatenate([u, [0.0]])
        while True:
            it += 1
            if it > maxit:
                raise RuntimeError("dual active set did not converge")
            if act:
                Q1, Q2, R = factor()
                z = Q2 @ (Q2.T @ n)
                r = sla.solve_triangular(R, Q1.T @ n, lower=False)
            else:
                z, r = n.copy(), np.zeros(0)
            zn = float(z @ n)
            t2 = -(float(n @ w) - b[p]) / zn if zn > 1e-20 * float(n @ n) else np.inf
            pos = np.nonzero(r > 0)[0]
            t1, k = np.inf, -1
            if pos.size:
                ratios = up[pos] / r[pos]
                j = int(np.argmin(ratios))
                t1, k = float(ratios[j]), int(pos[j])
            t = min(t1, t2)
            if not np.isfinite(t):
                raise RuntimeError("QP infeasible")
            if np.isfinite(t2):
                w = w + t * z
            up[:-1] -= t * r
            up[-1] += t
            if t2 <= t1:
                act.append(p)
                # exact re-solve on the active set: w = -gw + Q1 R^-T (b_A + N_A gw)
                Q1, _, R = factor()
                y = sla.solve_triangular(R, b[act] + Aw[act] @ gw, lower=False, trans="T")
                w = -gw + Q1 @ y
                u = np.maximum(sla.solve_triangular(R, y, lower=False), 0.0)
                break
            del act[k]
            up = np.delete(up, k)


def kkt_residual(W, c, A, b, x, tol=1e-9):
    """Algorithm-independent optimality measure of x: NNLS multipliers on the rows active at x,
    relative stationarity residual (0 at a KKT point) and the most negative slack."""
    from scipy.optimize import nnls

    grad = W.T @ (W @ x + c)
    s = A @ x - b
    act = np.abs(s) <= tol * np.maximum(1.0, np.abs(b))
    gn = max(1.0, float(np.linalg.norm(grad)))
    if not act.any():
        return float(np.linalg.norm(grad)) / gn, float(s.min(initial=np.inf))
    # many near-parallel active band rows (the cold QP where the disturbance enters) need more
    # than scipy's default 3n Lawson-Hanson iterations
    _, rn = nnls(A[act].T, grad, maxiter=max(1000, 50 * int(act.sum())))
    return rn / gn, float(s.min())


def band_qp(sc: BandScenario, G, f, rvec, u_prev, N2, Nu, q, wl, pin=None, with_obj=False):
    """One toolbox QP: returns (x = [dU; eps], iterations).  f: free response (my*N2),
    q: per-output tracking weight, wl: per-MV move weight (already squared / scaled).
    pin: {n: value} fixes MV n's first move du_n(0) (two extra rows), for replay checks of a
    move taken elsewhere; with_obj: also return the objective 1/2 |W x + c|^2."""
    my, nu = sc.my, sc.nu
    M = nu * Nu
    rows, cvec = [], []
    for i in range(my):
        if q[i] > 0:
            sq = np.sqrt(q[i])
            blk = np.zeros((N2, M + 1))
            blk[:, :M] = sq * G[i * N2:(i + 1) * N2]
            rows.append(blk)
            cvec.append(sq * (f[i * N2:(i + 1) * N2] - rvec[i]))
    Wl = np.zeros((M + 1, M + 1))
    Wl[np.arange(M), np.arange(M)] = np.sqrt(np.repeat(wl, Nu))
    Wl[M, M] = np.sqrt(sc.rho)
    rows.append(Wl)
    cvec.append(np.zeros(M + 1))
    W = np.vstack(rows)
    c = np.concatenate(cvec)
    Ab, bb = constraint_rows(nu, Nu, sc.du_min, sc.du_max, sc.u_min, sc.u_max, u_prev)
    A = [np.hstack([Ab, np.zeros((Ab.shape[0], 1))])]
    b = [bb]
    e = np.zeros((1, M + 1)); e[0, M] = 1.0
    A.append(e); b.append(np.zeros(1))
    for n, val in (pin or {}).items():
        e = np.zeros((2, M + 1))
        e[0, n * Nu], e[1, n * Nu] = 1.0, -1.0
        A.append(e); b.append(np.array([val, -val]))
    for i in range(my):
        Gi = G[i * N2:(i + 1) * N2]
        fi = f[i * N2:(i + 1) * N2]
        if np.isfinite(sc.y_max[i]):
            A.append(np.hstack([-Gi, np.full((N2, 1), sc.ecr_max[i] * sc.sy[i])]))
            b.append(fi - sc.y_max[i])
        if np.isfinite(sc.y_min[i]):
            A.append(np.hstack([Gi, np.full((N2, 1), sc.ecr_min[i] * sc.sy[i])]))
            b.append(sc.y_min[i] - fi)
    A = np.vstack(A)
    b = np.concatenate(b)
    # feasible start: dU = 0 (u_prev within its bounds), eps = the smallest slack that covers
    # every soft row violated at dU = 0
    x0 = np.zeros(M + 1)
    viol = b - A @ x0
    need = (viol > 0) & (A[:, M] > 0)
    # hard rows (MV bounds, eps >= 0, ECR-0 outputs) hold at dU = 0 up to the rounding of u_prev
    # (and, in replay_moves, up to the device QP's feasibility tolerance 1e-10); pinned rows
    # need not
    hard = ~(A[:, M] > 0)
    if pin:
        hard[Ab.shape[0] + 1:Ab.shape[0] + 1 + 2 * len(pin)] = False   # the pinned rows follow eps >= 0
    if np.any((viol > 1e-9 * np.maximum(1.0, np.abs(b))) & hard):
        raise NotImplementedError("hard output constraint violated by the free response")
    if np.any(need):
        x0[M] = np.max(viol[need] / A[need, M]) * (1 + 1e-12)
    # equilibrate: rho*eps dominates the gradient by ~9 orders of magnitude over lambda^2*du on
    # Shell 7x5, which makes any multiplier-sign test relative to max|mu| accept wrong working
    # sets.  Solve in y = D^-1 x with D = diag(H)^-1/2 and unit-norm constraint rows.
    dsc = 1.0 / np.sqrt(np.sum(W * W, axis=0))
    As = A * dsc[None, :]
    rn = np.linalg.norm(As, axis=1)
    rn[rn == 0] = 1.0
    Ws, As, bs = W * dsc[None, :], As / rn[:, None], b / rn
    y, it, _ = qp_dual_dense(Ws, c, As, bs)
    res, smin = kkt_residual(Ws, c, As, bs, y)
    if res > 1e-8 or smin < -1e-9:
        raise RuntimeError("oracle QP failed its KKT check (residual %.2e, slack %.2e)" % (res, smin))
    if with_obj:
        x = y * dsc
        return x, it, 0.5 * float(np.sum((W @ x + c) ** 2))
    return y * dsc, it


def closedloop_band(sc: BandScenario, r, v, N2: int, Nu: int, delta, lam, nit: int,
                    open_loop: bool = True, trace=None) -> CLResult:
    """[y,u,t,ys,uopt] = closedloop_toolbox(mpc,r,v,N,Nu,delta,lambda,nit) restated for the
    band-mode / measured-disturbance configuration.  r: my x nit, v: nd x nit."""
    my, nu, nd, nin = sc.my, sc.nu, sc.nd, sc.nin
    r = np.asarray(r, dtype=float).reshape(my, nit)
    v = np.asarray(v, dtype=float).reshape(nd, nit)
    delta = np.abs(np.asarray(delta, dtype=float))
    lam = np.abs(np.asarray(lam, dtype=float))
    wq = (delta / sc.sy) ** 2 if sc.weights_squared else delta / sc.sy
    wl = (lam / sc.su) ** 2 if sc.weights_squared else lam / sc.su
    ba = sc.ba()
    S = step_table(sc, N2 + 2)
    G = dyn_matrix(S, nu, N2, Nu)
    M = nu * Nu
    horizon = nit + N2 + 1

    def free(U, t, u_hold, v_hold):
        """Model prediction y(t+1..t+N2) with MVs held at u_hold from t, MDs at v_hold after t."""
        Uf = np.zeros((nin, t + N2 + 1))
        Uf[:, :t] = U[:, :t]
        Uf[:nu, t:] = u_hold[:, None]
        Uf[nu:, t:] = v_hold[:, None]
        Y = simulate(ba, Uf, t + N2 + 1)
        return Y[:, t + 1:].reshape(-1)

    ys = uopt = None
    iters = 0
    if open_loop:
        U0 = np.zeros((nin, 1))
        f0 = free(U0, 0, np.zeros(nu), v[:, -1])
        x0, it0 = band_qp(sc, G, f0, r[:, -1], np.zeros(nu), N2, Nu, wq, wl)
        Uopt = np.zeros((N2 + 1, nu))
        for i in range(N2 + 1):
            for n in range(nu):
                Uopt[i, n] = x0[n * Nu: n * Nu + min(i, Nu - 1) + 1].sum()
        uo = Uopt[:nit] if N2 + 1 > nit else np.vstack([Uopt, np.repeat(Uopt[-1:], nit - (N2 + 1), axis=0)])
        uopt = uo.T.copy()
        ys = simulate(ba, np.vstack([uopt, v]), nit)

    U = np.zeros((nin, horizon))
    U[nu:, :nit] = v
    Y = np.zeros((my, nit))
    u_prev = np.zeros(nu)
    DU = np.zeros((nu, nit))
    EPS = np.zeros(nit)
    for t in range(nit):
        Y[:, t] = simulate(ba, U, t + 1)[:, t]
        f = free(U, t, u_prev, v[:, t])
        if trace is not None:
            trace.append(f.copy())
        x, it = band_qp(sc, G, f, r[:, t], u_prev, N2, Nu, wq, wl)
        iters += it
        du = np.array([x[n * Nu] for n in range(nu)])
        DU[:, t] = du
        EPS[t] = x[M]
        u_prev = u_prev + du
        U[:nu, t] = u_prev
    res = CLResult(Y, U[:nu, :nit].copy(), ys, uopt, iters, DU)
    res.eps = EPS
    return res


def pinned_gap(sc: BandScenario, r, v, N2: int, Nu: int, delta, lam, U, t: int):
    """Replay check of the move an applied MV trajectory U (nu x nit) took at step t, judged by
    the QP's objective instead of the moves: the toolbox QP at the state U reached, solved free
    and with the first moves pinned to U's (du_n(0) = U[n, t] - U[n, t-1]).  Returns (J_free,
    J_pinned, du_oracle).  At steps where the soft-band slack dominates the cost by orders of
    magnitude the optimum is flat along the moves: the pinned QP then reaches the free optimum
    to ~1e-12 relative although the moves differ at 1e-6."""
    my, nu, nd, nin = sc.my, sc.nu, sc.nd, sc.nin
    nit = U.shape[1]
    r = np.asarray(r, dtype=float).reshape(my, nit)
    v = np.asarray(v, dtype=float).reshape(nd, nit)
    delta = np.abs(np.asarray(delta, dtype=float))
    lam = np.abs(np.asarray(lam, dtype=float))
    wq = (delta / sc.sy) ** 2 if sc.weights_squared else delta / sc.sy
    wl = (lam / sc.su) ** 2 if sc.weights_squared else lam / sc.su
    ba = sc.ba()
    G = dyn_matrix(step_table(sc, N2 + 2), nu, N2, Nu)
    u_prev = U[:, t - 1] if t > 0 else np.zeros(nu)
    Uf = np.zeros((nin, t + N2 + 1))
    Uf[:nu, :t] = U[:, :t]
    Uf[nu:, :t] = v[:, :t]
    Uf[:nu, t:] = u_prev[:, None]
    Uf[nu:, t:] = v[:, t][:, None]
    f = simulate(ba, Uf, t + N2 + 1)[:, t + 1:].reshape(-1)
    x, _, J0 = band_qp(sc, G, f, r[:, t], u_prev, N2, Nu, wq, wl, with_obj=True)
    pin = {n: float(U[n, t] - u_prev[n]) for n in range(nu)}
    _, _, J1 = band_qp(sc, G, f, r[:, t], u_prev, N2, Nu, wq, wl, pin=pin, with_obj=True)
    return J0, J1, np.array([x[n * Nu] for n in range(nu)])


def replay_moves(sc: BandScenario, r, v, N2: int, Nu: int, delta, lam, U, T=None):
    """Per-step optimality check of an applied MV trajectory U (nu x nit, e.g. the device's):
    at every step t the state is rebuilt from U[:, :t] and v, and the toolbox QP is solved there.
    Returns (du_oracle, du_applied), both nu x T.  A trajectory that diverges from the oracle's
    free run (unstable or switching closed loops amplify rounding) must still take the QP's
    optimal move at the state it is actually in."""
    my, nu, nd, nin = sc.my, sc.nu, sc.nd, sc.nin
    nit = U.shape[1]
    T = nit if T is None else T
    r = np.asarray(r, dtype=float).reshape(my, nit)
    v = np.asarray(v, dtype=float).reshape(nd, nit)
    delta = np.abs(np.asarray(delta, dtype=float))
    lam = np.abs(np.asarray(lam, dtype=float))
    wq = (delta / sc.sy) ** 2 if sc.weights_squared else delta / sc.sy
    wl = (lam / sc.su) ** 2 if sc.weights_squared else lam / sc.su
    ba = sc.ba()
    G = dyn_matrix(step_table(sc, N2 + 2), nu, N2, Nu)
    Uall = np.zeros((nin, nit + N2 + 1))
    Uall[:nu, :nit] = U
    Uall[nu:, :nit] = v
    du_o = np.zeros((nu, T))
    du_a = np.zeros((nu, T))
    for t in range(T):
        u_prev = U[:, t - 1] if t > 0 else np.zeros(nu)
        Uf = np.zeros((nin, t + N2 + 1))
        Uf[:, :t] = Uall[:, :t]
        Uf[:nu, t:] = u_prev[:, None]
        Uf[nu:, t:] = v[:, t][:, None]
        f = simulate(ba, Uf, t + N2 + 1)[:, t + 1:].reshape(-1)
        x, _ = band_qp(sc, G, f, r[:, t], u_prev, N2, Nu, wq, wl)
        du_o[:, t] = [x[n * Nu] for n in range(nu)]
        du_a[:, t] = U[:, t] - u_prev
    return du_o, du_a
