"""Toolbox-equivalent constrained GPC closed loop — restatement of ``closedloop_toolbox.m``.

Oracle; test infrastructure only.  SURVEY §8 rows A1/A2 (semantics) composed with the DTC-GPC
primitives A3-A8 (arithmetic):

* ``closedloop_toolbox.m:36-43`` sets PredictionHorizon = max(N), ControlHorizon = max(Nu),
  Weights.OV = delta, Weights.MVRate = lambda.  The toolbox cost is
      sum_{j=1..p} || delta .* (y(t+j|t) - r(t)) ||^2 + sum_{l=0..Nu-1} || lambda .* du(t+l) ||^2
  (weights enter SQUARED; reference held flat over the horizon — mpcsimopt RefLookAhead 'off',
  Shell3x3.m:154), subject to the MV rate and amplitude bounds (Shell3x3.m:120-142 scaled by
  MPCTuning.m:170-178).
* In the nominal tuning setting the toolbox's state estimator sees zero innovation, so its
  prediction equals the exact model prediction.  That prediction is computed here the way the
  reference's own GPC computes it: free response ``f = Hp*up + S*Yd`` from the Diophantine F
  polynomials (diophantine.m, DTC_GPC_WW.m:83-86) and the past-control matrix
  (deltaUFree.m + cell2mat2.m, DTC_GPC_WW.m:92-93), forced response from MatG.m.
  window='toolbox' predicts t+1..t+N2 (toolbox), window='gpc' predicts t+dmin+1..t+dmin+N2
  (MatG/diophantine N1 = d+1), weights_squared=False gives the DTC_GPC_WW.m:67-76 weighting.
* The per-step QP  min 1/2 dU'(G'QG + Lambda) dU + dU'G'Q(f - w)  is solved to optimality by a
  textbook primal active-set method (Nocedal & Wright Alg. 16.3) on its least-squares form
  ||[Q^1/2 G; Lambda^1/2] dU + [Q^1/2 (f-w); 0]||^2 (never forming the ill-conditioned normal
  equations) — deliberately a different algorithm from the device's dual (Goldfarb-Idnani)
  method; the strictly convex QP has a unique minimiser, so both must agree to rounding.
* Open-loop first-move prediction (closedloop_toolbox.m:85-100): the QP at the initial state
  with reference r(:,end) gives Info.Uopt (p+1 rows, held after the control horizon), padded
  with its last row to nit (:94-98); ys = lsim(Pz, [uopt v]) (:100).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .dtcgpc import ba_mimo, blkdiag, cell2mat2, delta_u_free, descomp_mpc, diophantine, mat_g


@dataclass
class Scenario:
    """Everything closedloop_toolbox needs that does not depend on the candidate."""

    plant: list            # my x (nu+nd) DTF — the simulated plant (sim's default: the model)
    model: list            # my x (nu+nd) DTF — controller's prediction model (mpcobj.Model.Plant)
    nu: int                # number of MVs
    du_min: np.ndarray
    du_max: np.ndarray
    u_min: np.ndarray
    u_max: np.ndarray
    window: str = "toolbox"          # 'toolbox' (t+1..t+N2) or 'gpc' (t+dmin+1..)
    weights_squared: bool = True     # toolbox weights enter squared
    round_roots: bool = False        # BA_MIMO verbatim rounding (DTC-faithful) vs exact LCM
    # derived
    B: list = field(default=None)
    A: list = field(default=None)
    na: np.ndarray = field(default=None)
    nb: np.ndarray = field(default=None)
    dp: np.ndarray = field(default=None)

    def __post_init__(self):
        Bn, An, d = descomp_mpc(self.model)
        self.dp = d
        self.B, self.A, self.na, self.nb = ba_mimo(Bn, An, round_roots=self.round_roots)
        for i in range(self.my):
            for j in range(self.nu):
                b, _ = self.plant[i][j].zinv_form()
                if b[0] != 0:
                    raise ValueError("MV direct feedthrough: algebraic loop")

    @property
    def my(self):
        return len(self.model)

    @property
    def nin(self):
        return len(self.model[0])

    @property
    def nd(self):
        return self.nin - self.nu

    @property
    def dmin(self):
        return self.dp[:, : self.nu].min(axis=1)


def prediction_tables(sc: Scenario, N2: int, Nu: int):
    """G (MatG), S (blkdiag F), Hp (cell2mat2(deltaUFree)), duM for one (N2, Nu)."""
    my, nu = sc.my, sc.nu
    dwin = np.zeros(my, dtype=int) if sc.window == "toolbox" else sc.dmin
    dmat = np.repeat(dwin[:, None], nu, axis=1)
    mv_model = [row[:nu] for row in sc.model]
    G, _ = mat_g(mv_model, [N2] * my, [Nu] * nu, dmat)
    En, F = [], []
    for i in range(my):
        Ei, Fi = diophantine(sc.A[i], N2, int(dwin[i]))
        En.append(Ei)
        F.append(Fi)
    S = blkdiag(*[F[i][:N2, :] for i in range(my)])
    Bmv = [row[:nu] for row in sc.B]
    uG = delta_u_free(Bmv, En, [N2] * my, sc.dp[:, :nu])
    Hp = cell2mat2(uG)
    duM = np.array([max(uG[m][n].shape[1] for m in range(my)) for n in range(nu)])
    return G, S, Hp, duM


def constraint_rows(nu: int, Nu: int, du_min, du_max, u_min, u_max, u_prev):
    """Rows (Aineq, bineq) of Aineq x >= bineq for x = [du_1(0..Nu-1), du_2(..), ...]:
    rate bounds on every move and amplitude bounds u(t-1) + cumsum(du) in [umin, umax]."""
    M = nu * Nu
    rows, rhs = [], []
    for n in range(nu):
        for l in range(Nu):
            e = np.zeros(M)
            e[n * Nu + l] = 1.0
            pre = np.zeros(M)
            pre[n * Nu: n * Nu + l + 1] = 1.0
            if np.isfinite(du_min[n]):
                rows.append(e); rhs.append(du_min[n])
            if np.isfinite(du_max[n]):
                rows.append(-e); rhs.append(-du_max[n])
            if np.isfinite(u_min[n]):
                rows.append(pre); rhs.append(u_min[n] - u_prev[n])
            if np.isfinite(u_max[n]):
                rows.append(-pre); rhs.append(-(u_max[n] - u_prev[n]))
    if not rows:
        return np.zeros((0, M)), np.zeros(0)
    return np.array(rows), np.array(rhs)


def qp_primal_active_set(W, c, Ain, bin_, tol=1e-12, maxit=1000):
    """min 1/2 ||W x + c||^2  s.t. Ain x >= bin, from the feasible start x = 0 — a textbook
    primal active-set method (Nocedal & Wright Alg. 16.3) that never forms the normal equations:
    the equality-constrained subproblem on the working set is solved by the null-space method,
    p = Z y, y = lstsq(W Z, -(W x + c)) (SVD), Z an orthonormal basis of null(Ain[W]).
    H = W'W, g = W'c is the toolbox QP min 1/2 dU'H dU + g'dU.  Normal equations would lose
    ~cond(H)*eps (~1e-5 at cond 1e11, reached on the config-2 grid); see DESIGN.md §Numerics.
    Returns (x, iterations, working_set, multipliers)."""
    M = W.shape[1]
    x = np.zeros(M)
    s = Ain @ x - bin_ if Ain.size else np.zeros(0)
    if Ain.size and np.any(s < -1e-9):
        raise ValueError("QP start point infeasible (%g)" % s.min())
    W_ = []
    for i in np.nonzero(s <= tol)[0]:  # independent initial working set
        cand = W_ + [int(i)]
        if np.linalg.matrix_rank(Ain[cand]) == len(cand):
            W_ = cand
    it = 0
    while it < maxit:
        it += 1
        q = len(W_)
        res = W @ x + c
        if q:
            AW = Ain[W_]
            _, sv, Vt = np.linalg.svd(AW)
            Z = Vt[q:].T
        else:
            Z = np.eye(M)
        if Z.shape[1]:
            y = np.linalg.lstsq(W @ Z, -res, rcond=None)[0]
            p = Z @ y
        else:
            p = np.zeros(M)
        alpha, block = 1.0, None
        if Ain.size:
            Ap = Ain @ p
            s = Ain @ x - bin_
            # only a constraint the step really moves toward can block it; a rounding-level
            # A_i p < 0 would admit a constraint dependent on the working set (degenerate cycling)
            thr = 1e-12 * np.max(np.abs(p)) * np.max(np.abs(Ain), axis=1)
            for i in range(Ain.shape[0]):
                if i in W_ or Ap[i] >= -thr[i]:
                    continue
                a = max(s[i], 0.0) / (-Ap[i])
                if a < alpha:
                    alpha, block = a, i
        x = x + alpha * p
        if block is not None:
            W_.append(block)
            continue
        # full step: x minimises on the working set; multipliers from W'(Wx + c) = AW' mu
        if q == 0:
            return x, it, W_, np.zeros(0)
        grad = W.T @ (W @ x + c)
        mu = np.linalg.lstsq(Ain[W_].T, grad, rcond=None)[0]
        # scale-relative optimality test: the multipliers scale with the objective, which can be
        # ~1e-9 on the config-2 grid (an absolute tolerance accepts wrong working sets there)
        if np.all(mu >= -1e-9 * np.max(np.abs(mu))):
            return x, it, W_, mu
        W_.pop(int(np.argmin(mu)))
    raise RuntimeError("primal active set did not converge")


@dataclass
class CLResult:
    y: np.ndarray
    u: np.ndarray
    ys: np.ndarray | None
    uopt: np.ndarray | None
    qp_iters: int
    du_hist: np.ndarray


class _Plant:
    """Incremental simulation of an my x nin matrix of DTF entries (lsim restated)."""

    def __init__(self, P):
        self.P = P
        self.my = len(P)
        self.nin = len(P[0])
        self.ba = [[P[i][j].zinv_form() for j in range(self.nin)] for i in range(self.my)]

    def simulate(self, U, T):
        """Outputs y(0..T-1) for inputs U (nin x T) — direct form per entry."""
        Y = np.zeros((self.my, T))
        for i in range(self.my):
            for j in range(self.nin):
                b, a = self.ba[i][j]
                ye = np.zeros(T)
                for t in range(T):
                    acc = 0.0
                    for l in range(len(b)):
                        if t - l >= 0 and b[l] != 0:
                            acc += b[l] * U[j, t - l]
                    for l in range(1, len(a)):
                        if t - l >= 0:
                            acc -= a[l] * ye[t - l]
                    ye[t] = acc
                Y[i] += ye
        return Y

    def output_at(self, U, t, ystate):
        """y(t) for each entry from inputs U[:, :t+1] (entries strictly proper in MVs).
        ystate[i][j] is the entry's output history list (appended to)."""
        y = np.zeros(self.my)
        for i in range(self.my):
            for j in range(self.nin):
                b, a = self.ba[i][j]
                hist = ystate[i][j]
                acc = 0.0
                for l in range(len(b)):
                    if t - l >= 0 and b[l] != 0:
                        acc += b[l] * U[j, t - l]
                for l in range(1, len(a)):
                    if t - l >= 0:
                        acc -= a[l] * hist[t - l]
                hist.append(acc)
                y[i] += acc
        return y


def closedloop_toolbox(sc: Scenario, r, v, N2: int, Nu: int, delta, lam, nit: int,
                       open_loop: bool = True, full_history: bool = False) -> CLResult:
    """[y,u,t,ys,uopt] = closedloop_toolbox(mpc,r,v,N,Nu,delta,lambda,nit) restated.

    r: my x nit reference (row signals, as the callers pass Xsp), v: nd x nit (may be empty).
    Returns row-signal arrays (my x nit, nu x nit) like col2row at closedloop_toolbox.m:103-107.
    full_history: the plant output of step t is re-simulated over the whole input history with
    lsim (scipy lfilter per entry), the structure of DTC_GPC_WW.m:130-136 / OptimalPredictor2.m:
    28-37 -- O(nit^2) per simulation, the reference-structured CPU baseline.
    """
    my, nu, nd = sc.my, sc.nu, sc.nd
    r = np.asarray(r, dtype=float).reshape(my, nit)
    v = np.zeros((nd, nit)) if nd == 0 else np.asarray(v, dtype=float).reshape(nd, nit)
    if nd:
        raise NotImplementedError("measured disturbances: round-2 scope (Shell 7x5)")
    delta = np.abs(np.asarray(delta, dtype=float))
    lam = np.abs(np.asarray(lam, dtype=float))
    G, S, Hp, duM = prediction_tables(sc, N2, Nu)
    wq = delta ** 2 if sc.weights_squared else delta
    wl = lam ** 2 if sc.weights_squared else lam
    qdiag = np.repeat(wq, N2)
    # weighted least-squares form of the toolbox cost: ||Q^1/2 (G dU + f - w)||^2 + ||Lambda^1/2 dU||^2
    sq = np.sqrt(qdiag)
    Wls = np.vstack([sq[:, None] * G, np.diag(np.sqrt(np.repeat(wl, Nu)))])
    na = sc.na
    M = nu * Nu
    plant = _Plant(sc.plant)

    def solve(yhist, up, u_prev, rvec):
        Yd = np.concatenate([yhist[i] for i in range(my)])
        f = Hp @ up + S @ Yd
        w = np.repeat(rvec, N2)
        cvec = np.concatenate([sq * (f - w), np.zeros(M)])
        Ain, bin_ = constraint_rows(nu, Nu, sc.du_min, sc.du_max, sc.u_min, sc.u_max, u_prev)
        x, it, _, _ = qp_primal_active_set(Wls, cvec, Ain, bin_)
        return x, it

    ys = uopt = None
    if open_loop:
        # closedloop_toolbox.m:85-91: initial state, yo = y(0) = 0, reference r(:,end)
        yh0 = [np.zeros(na[i] + 1) for i in range(my)]
        x0, _ = solve(yh0, np.zeros(duM.sum()), np.zeros(nu), r[:, -1])
        p = N2
        Uopt = np.zeros((p + 1, nu))
        for i in range(p + 1):
            for n in range(nu):
                Uopt[i, n] = x0[n * Nu: n * Nu + min(i, Nu - 1) + 1].sum()
        if p + 1 > nit:
            uo = Uopt[:nit]
        else:
            uo = np.vstack([Uopt, np.repeat(Uopt[-1:], nit - (p + 1), axis=0)])
        uopt = uo.T.copy()
        ys = plant.simulate(np.vstack([uopt, v]), nit)

    U = np.zeros((nu + nd, nit))
    Y = np.zeros((my, nit))
    ystate = [[[] for _ in range(sc.nin)] for _ in range(my)]
    yhist = [np.zeros(na[i] + 1) for i in range(my)]
    up = np.zeros(duM.sum())
    offs = np.concatenate([[0], np.cumsum(duM)])
    u_prev = np.zeros(nu)
    iters = 0
    DU = np.zeros((nu, nit))
    if full_history:
        from scipy.signal import lfilter

    for t in range(nit):
        if full_history:   # y = lsim(P, u(1:k)) every step (DTC_GPC_WW.m:130-131)
            yt = np.array([sum(lfilter(*plant.ba[i][j], U[j, :t + 1])[t] for j in range(sc.nin))
                           for i in range(my)])
        else:
            yt = plant.output_at(U, t, ystate)
        Y[:, t] = yt
        for i in range(my):
            yhist[i] = np.concatenate([[yt[i]], yhist[i][:-1]])
        x, it = solve(yhist, up, u_prev, r[:, t])
        iters += it
        du = np.array([x[n * Nu] for n in range(nu)])
        DU[:, t] = du
        u_prev = u_prev + du
        U[:nu, t] = u_prev
        for n in range(nu):
            seg = up[offs[n]: offs[n + 1]]
            up[offs[n]: offs[n + 1]] = np.concatenate([[du[n]], seg[:-1]])
    return CLResult(Y, U[:nu].copy(), ys, uopt, iters, DU)
