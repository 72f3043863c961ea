"""The tuning loop around the batched closed-loop engine: MPCTuning's Par, the VNS horizon search,
the GAM weight search and their alternation, and the Tuning_Parameters record.

  de2bi / bits_of            Communications-toolbox de2bi as MPCTuning.m:285 / VNS2.m:210-215 use it
  TuningPar                  Par of MPCTuning.m:307-340 (bit weights, initial horizons, bounds, ...)
  vns2(par, evaluate, fv)    VNS2.m:1-292, control flow kept line by line (orders {1, 3} only, the
                             ii increment sits inside the tt loop, first improvement, restarts)
  vns2_batched(...)          the same search, every neighbour evaluation served from batches
                             scored on the GPU (speculative replay, identical decisions)
  gam_fgoalattain(...)       GAM_fun.m + MPC_TFob.m:61-67: goal attainment on J1 (restated)
  mpc_tfob(...)              MPC_TFob.m:28-143: GAM / VNS alternation and its quirks
  save_tuning_parameters     MPCTuning.m:374-381 record (MAT v5 via scipy.io.savemat, or JSON)

The evaluators are callables, so the search logic is the same whether a neighbour is scored by
the HIP engine (mpct.engine, the product path) or by a checker in tests.
"""
from __future__ import annotations

import functools
import json
import math
from dataclasses import dataclass, field

import numpy as np

from .objectives import precon


# --------------------------------------------------------------------------------------------
def de2bi(x: int, n: int) -> list:
    """de2bi(x, n): n bits, least significant first (MATLAB's default 'right-msb' ordering)."""
    return [(int(x) >> k) & 1 for k in range(n)]


def bits_of(x: int, n: int) -> list:
    """flip(de2bi(x, n)): most significant bit first, the layout of Xv1 / Xv2 rows."""
    return de2bi(x, n)[::-1]


def bit_weights(nbp: int, nbc: int) -> np.ndarray:
    """Fc of MPCTuning.m:270-278: [2^(nbp-1) .. 1, 2^(nbc-1) .. 1]."""
    return np.array([2 ** i for i in range(nbp - 1, -1, -1)] + [2 ** i for i in range(nbc - 1, -1, -1)],
                    dtype=np.int64)


@dataclass
class TuningPar:
    """MPCTuning.m:264-340.  my outputs, ny MVs (the reference's Par.ny / Par.nu naming is
    swapped, MPCTuning.m:307-308; here my = outputs, ny = inputs)."""

    my: int
    ny: int
    nbp: int = 7
    nbc: int = 4
    dmin: np.ndarray = None         # minimal delay per output (MPCTuning.m:257-262)
    w: np.ndarray = None            # GAM weights (Pareto), Shell3x3.m:161
    q0: np.ndarray = None           # initial OV weights (mpcobj.Weights.OV)
    w0: np.ndarray = None           # initial MV-rate weights (mpcobj.Weights.MVRate)
    nit: int = 500
    Fc: np.ndarray = field(default=None)
    N: np.ndarray = field(default=None)
    Nu: np.ndarray = field(default=None)
    Xv1: list = field(default=None)
    Xv2: list = field(default=None)
    delta: np.ndarray = field(default=None)
    lam: np.ndarray = field(default=None)
    x0: np.ndarray = field(default=None)
    lb1: np.ndarray = field(default=None)
    ov_zero: np.ndarray = field(default=None)   # OV weights the user set to 0 (band mode)

    def __post_init__(self):
        if self.nbp < self.nbc:            # MPCTuning.m:138-140
            self.nbp = self.nbc
        self.Fc = bit_weights(self.nbp, self.nbc)
        Hp, Hc = 2 ** self.nbp - 1, 2 ** self.nbc - 1     # MPCTuning.m:283-285
        self.Xv1 = bits_of(Hp, self.nbp)
        self.Xv2 = [bits_of(Hc, self.nbc) for _ in range(self.ny)]   # MPC_TFob.m:46-50
        self.N = np.full(self.my, Hp, dtype=np.int64)                # MPCTuning.m:288
        self.Nu = np.full(self.ny, 2, dtype=np.int64)                # MPCTuning.m:289
        self.delta = np.ones(self.my)                                # MPCTuning.m:265-266
        self.lam = np.ones(self.ny)
        q0 = np.ones(self.my) if self.q0 is None else np.asarray(self.q0, dtype=float)
        w0 = np.ones(self.ny) if self.w0 is None else np.asarray(self.w0, dtype=float)
        self.ov_zero = q0 == 0
        self.x0 = np.concatenate([q0, w0])                           # MPCTuning.m:300
        self.lb1 = np.full(self.my + self.ny, 1e-5)                  # MPCTuning.m:302
        self.dmin = np.zeros(self.my, dtype=np.int64) if self.dmin is None else np.asarray(self.dmin)
        self.w = np.ones(self.my) if self.w is None else np.asarray(self.w, dtype=float)


# --------------------------------------------------------------------------------------------
def vns2(par: TuningPar, evaluate, fv: float):
    """VNS2.m:1-292 with the MATLAB control flow kept line by line.

    evaluate(N, Nu) -> F (VNS2.m:147-195 for the neighbour, max(N)/max(Nu) horizons).
    fv is the global Fv (best cost so far, MPCTuning.m:292).  Returns
    (N, Nu, Xv1, Xv2, Fvns, fv, n_evals).  A failed simulation (NaN F) never improves.
    """
    my, ny = par.my, par.ny
    Fc = [int(v) for v in par.Fc]
    nbp = par.nbp
    Fc1, Fc2 = Fc[:nbp], Fc[nbp:]
    Nt1, Nt2 = len(Fc1), len(Fc2)
    Xv1 = list(par.Xv1)
    Xv2 = [list(r) for r in par.Xv2]
    N = [int(v) for v in par.N]
    Nu = [int(v) for v in par.Nu]
    Nu1 = list(Nu)
    dmin = [int(v) for v in par.dmin]
    dot = lambda c, x: sum(a * b for a, b in zip(c, x))          # noqa: E731
    n_evals = 0

    ii = 1
    while ii <= 3:                                   # VNS2.m:89
        Order = ii
        tt = 1
        m = 1
        Hpc = my
        H = 1
        while tt <= 2:                               # VNS2.m:98 (ii advances inside: orders 1, 3)
            while H <= Hpc:
                if tt == 1:
                    Nt, X3, Fc3 = Nt1, [None] + list(Xv1), Fc1
                else:
                    Nt, X3, Fc3 = Nt2, [None] + list(Xv2[H - 1]), Fc2
                Ix = [None, Nt]                      # 1-based like the reference
                for i in range(2, Order + 1):
                    Ix.append(Ix[i - 1] - 1)
                while Ix[1] >= 1 and tt != 0:        # VNS2.m:114
                    for t in range(1, Order):        # static indices (VNS2.m:116-120)
                        if 0 < Ix[t] <= Nt:
                            X3[Ix[t]] = 1 - X3[Ix[t]]
                    while Ix[-1] >= 1:               # VNS2.m:122
                        X3[Ix[-1]] = 1 - X3[Ix[-1]]
                        if tt == 1:
                            N[:] = [dot(Fc3, X3[1:])] * my
                        else:
                            Nu[H - 1] = dot(Fc3, X3[1:])
                            Nu1[H - 1] = dot(Fc2, Xv2[H - 1])
                        if (not precon(N, Nu) or not precon(N, Nu1) or any(n <= d for n, d in zip(N, dmin))
                                or any(u <= 1 for u in Nu)):      # VNS2.m:135
                            X3[Ix[-1]] = 1 - X3[Ix[-1]]
                            if tt == 1:
                                N[:] = [dot(Fc3, X3[1:])] * my
                            else:
                                Nu[H - 1] = dot(Fc3, X3[1:])
                        else:
                            F = evaluate(tuple(N), tuple(Nu))
                            n_evals += 1
                            if F < fv:                            # VNS2.m:198
                                fv = F
                                Ix[1] = Nt
                                for i in range(2, Order + 1):
                                    Ix[i] = Ix[i - 1] - 1
                                Ix[-1] = -1
                                Ix[1] = -1
                                Xv1 = bits_of(N[0], len(Fc1))     # VNS2.m:210-215
                                Xv2 = [bits_of(Nu[i], len(Fc2)) for i in range(ny)]
                            else:                                 # discard the neighbour
                                X3[Ix[-1]] = 1 - X3[Ix[-1]]
                                if tt == 1:
                                    N[:] = [dot(Fc3, X3[1:])] * my
                                else:
                                    Nu[H - 1] = dot(Fc3, X3[1:])
                        Ix[-1] -= 1                               # VNS2.m:223
                    X3 = [None] + (list(Xv1) if tt == 1 else list(Xv2[H - 1]))
                    if Order == 1 and Ix[1] < 0:                  # VNS2.m:233-239
                        Ix[1] = Nt
                        pos = [1]
                    else:
                        pos = [2]
                    while pos and pos[0] != 1:                    # VNS2.m:241-251
                        pos = [k for k in range(1, len(Ix)) if Ix[k] == 0]
                        if pos and pos[0] != 1:
                            p0 = pos[0]
                            Ix[p0 - 1] -= 1
                            Ix[p0] = Ix[p0 - 1] - 1
                        pos = [k for k in range(1, len(Ix)) if Ix[k] == 0]
                    if not pos and Ix[1] != -1:                   # VNS2.m:255-259
                        neg = [k for k in range(1, len(Ix)) if Ix[k] < 0]
                        if neg:
                            for j in range(neg[0], Order + 1):
                                Ix[j] = Ix[j - 1] - 1
                if tt == 0:
                    H = Hpc
                H += 1
            H = 1
            tt += 1
            if m <= 1 or tt == 1:                    # VNS2.m:276-281
                Hpc = my
            if tt == 2:
                Hpc = ny
            ii += 1
    N = [dot(Fc1, Xv1)] * my                         # VNS2.m:285-289
    Nu = [dot(Fc2, Xv2[i]) for i in range(ny)]
    return np.array(N), np.array(Nu), Xv1, Xv2, fv, fv, n_evals


class StaleRows:
    """VNS2.m:148-165: a square plant's VNS runs one closed loop per output i inside try/catch and
    copies row i of Xy / Xu / Xyma / Xuma from simulation i only when it succeeds (:157-160).  A
    failed simulation leaves row i as the last successful evaluation set it, so the neighbour's F
    (:172-195) mixes rows of different neighbours.  Row i enters F only through
    T_i = j21_i + j22_i + Jnu_i, so the state is the last T per row.  The rows are never
    initialised: MATLAB zero-fills rows below an assigned one (T_i0 = sum_{t >= inK} Yref_i(t)^2:
    Xy = Xyma = Xuma = 0).
    While only row 1 exists (every earlier simulation of outputs 2..my failed), :173
    Xy - Yref broadcasts the 1 x K row against the my x K Yref (implicit expansion), and
    F = my j21_1 + sum_i sum_{t >= inK} (y_1 - Yref_i)^2 + N(1) + Jnu_1: the evaluator supplies
    that quantity without N(1) as a callable ``bcast`` of row 1's simulation (evaluated lazily;
    objectives.vns_row1_broadcast).  With 1 < rows < my the expansion fails and :173 throws,
    which ends the reference's run; here that neighbour scores NaN (never taken), as it does with
    one row when no ``bcast`` is given.
    score(N1, terms, ok[, bcast]) -> F with terms = T of this neighbour's simulations and ok =
    which of them succeeded; call reset() at the start of every VNS2 pass."""

    def __init__(self, init_terms):
        self.init = np.asarray(init_terms, dtype=float)
        self.reset()

    def reset(self):
        self.last = self.init.copy()
        self.nrows = 0
        self.row1 = None  # bcast of the simulation that last set row 1

    def score(self, N1, terms, ok, bcast=None):
        terms = np.asarray(terms, dtype=float)
        ok = np.asarray(ok, dtype=bool)
        self.last[ok] = terms[ok]
        if ok[0]:
            self.row1 = bcast  # evaluated below only while row 1 is the only row (memoized per
            # neighbour by its producer, batch_vns_rows, so a cache hit does not re-simulate)
        if ok.any():
            self.nrows = max(self.nrows, int(np.nonzero(ok)[0].max()) + 1)
        if self.nrows < self.last.size:
            if self.nrows == 1 and self.row1 is not None:
                if callable(self.row1):
                    self.row1 = float(self.row1())
                return self.row1 + N1
            return math.nan
        return float(self.last.sum()) + N1


class _Miss(Exception):
    pass


def vns2_batched(par: TuningPar, batch_evaluate, fv: float, max_batch: int = 512, stale=None):
    """vns2 with every neighbour scored in GPU batches and the SAME decisions as the sequential
    search.  A speculative pass replays the search from the start with the scores known so far;
    unknown neighbours are taken as non-improving and collected, then scored together in one
    batch (batch_evaluate(list of (N, Nu)) -> list of F, or with ``stale`` (StaleRows) a list of
    (terms, ok) per neighbour, F then following VNS2.m's stale-row semantics in evaluation order).
    Replays repeat until a pass needs nothing unknown; every decision of the final pass was taken
    on real scores (and real stale-row state), and speculated neighbours never change the search
    state (a rejected neighbour is reverted), so the result equals the sequential search's.
    Returns vns2's tuple plus the number of batches."""
    cache = {}
    n_batches = 0
    while True:
        pending = []
        if stale is not None:
            stale.reset()

        def spec(N, Nu):
            key = (N, Nu)
            if key in cache:
                if stale is not None:
                    return stale.score(N[0], *cache[key])
                return cache[key]
            if key not in pending and len(pending) < max_batch:
                pending.append(key)
            return math.inf

        out = vns2(par, spec, fv)
        if not pending:
            return out + (n_batches,)
        scores = batch_evaluate(pending)
        n_batches += 1
        for key, F in zip(pending, scores):
            if stale is not None:
                cache[key] = F
            else:
                cache[key] = float(F) if np.isfinite(F) else math.nan


# --------------------------------------------------------------------------------------------
def gam_fgoalattain(par: TuningPar, batch_j1, goal: float = 1e-3, diff_min_change: float = 0.5,
                    max_iter: int = 400, ftol: float = 1e-3, speculate: bool = False,
                    max_fun_evals: int | None = None, memo: dict | None = None):
    """GAM step of MPC_TFob.m:61-67: fgoalattain(@GAM_fun, x0, goal=0.001, weight=w, lb=1e-5,
    EqualityGoalCount = numel(w)) -- restated as the goal-attainment problem
        min gamma  s.t.  |J1_i(x) - goal| <= w_i * gamma,  x >= lb1
    solved by SLSQP with forward-difference Jacobians whose step is at least DiffMinChange
    (MPCTuning.m:88-91: 'DiffMinChange', 0.5); each Jacobian is ONE batch of my+ny+1 closed
    loops.  batch_j1(X rows) -> J1 rows (GAM_fun.m:55-116 for each row).  MATLAB's SQP internals
    are not public: parity with fgoalattain's iterate sequence is unpinned; the goal-attainment
    formulation and options are the reference's.  Returns (x, attainfactor, J1(x), n_batches,
    last_eval): last_eval is the J1 of the LAST point the search evaluated, in evaluation order
    (a Jacobian batch evaluates x, then x + h_k e_k for k = 0..n-1, as MATLAB's forward
    differences do) -- the value GAM_fun.m:114 leaves in the global F that MPC_TFob.m:104 reads.
    speculate: every new point the search asks for (a line-search trial) is scored in one batch
    together with its n forward-difference points, so an accepted step's Jacobian costs no further
    engine call.  Measured on the Van de Vusse run it saves nothing: SLSQP's line
    search on these finite-difference Jacobians backtracks on most iterations, and a batch of n + 1
    closed loops waits for its slowest one (91 s against 88 s unbatched, same endpoint).  Scoring
    the backtracking steps ahead as well needs SLSQP's trial points bit for bit, which its caller
    cannot reproduce; points matched to 13 digits moved the search to another endpoint.  Off by
    default.  Points are cached by their exact value.
    max_fun_evals: fgoalattain's MaxFunctionEvaluations, which MPCTuning.m:88-91 leaves at its
    default of 100 * numel(x0).  MATLAB counts every call of the objective, line-search trials and
    forward-difference points alike; here every distinct point the search asks for.  The search
    stops after the iteration that reaches the budget and returns that iterate (MATLAB's exitflag
    0).  memo: a point cache that outlives the call (mpc_tfob keeps one per (max N, max Nu), so a
    GAM round that repeats an earlier one from the same start costs no engine call); the values
    and the evaluation-order bookkeeping are the same as without it."""
    from scipy.optimize import minimize

    my, ny = par.my, par.ny
    n = my + ny
    w = np.asarray(par.w, dtype=float)
    if max_fun_evals is None:
        max_fun_evals = 100 * n
    cache = memo if memo is not None else {}
    nb = [0]
    last = [None]
    last_eval = [None]

    def fd_points(x):
        h = np.maximum(diff_min_change, np.sqrt(np.finfo(float).eps) * np.abs(x))
        return [x] + [x + h[k] * np.eye(n)[k] for k in range(n)], h

    asked = set()   # points the search itself has requested (MATLAB evaluates each once)

    def key(x):
        return tuple(np.asarray(x, dtype=float).tolist())

    def evals(X, spec=()):
        keys = [key(x) for x in X]
        todo = [i for i, k in enumerate(keys) if k not in cache]
        if todo:
            extra, ek = [], set()
            for p in spec:
                k = key(p)
                if k not in cache and k not in ek and k not in keys:
                    extra.append(p)
                    ek.add(k)
            J = batch_j1(np.array([X[i] for i in todo] + extra))
            nb[0] += 1
            for i, j in zip(todo, J):
                cache[keys[i]] = np.asarray(j, dtype=float)
            for p, j in zip(extra, J[len(todo):]):
                cache[key(p)] = np.asarray(j, dtype=float)
        new = [k for k in keys if k not in asked]
        if new:   # the search's own last request (a re-request of a known point is no evaluation)
            last_eval[0] = cache[new[-1]]
            asked.update(new)
        return [cache[k] for k in keys]

    def jac_F(x):
        pts, h = fd_points(x)
        vals = evals(pts)
        F0 = vals[0]
        Jm = np.stack([(vals[k + 1] - F0) / h[k] for k in range(n)], axis=1)   # my x n
        return F0, Jm

    best = [np.inf, None]   # best attainment factor over the iterates / line-search points

    def F(x):
        v = evals([x], spec=fd_points(x)[0][1:] if speculate and key(x) not in cache else ())[0]
        last[0] = v
        a = float(np.max(np.abs(v - goal) / w))
        if a < best[0]:
            best[0], best[1] = a, np.array(x, dtype=float)
        return v

    x0 = np.maximum(np.asarray(par.x0, dtype=float), par.lb1)
    F0 = F(x0)
    g0 = float(np.max(np.abs(F0 - goal) / w))
    z0 = np.concatenate([x0, [g0]])
    cons = [
        {"type": "ineq", "fun": lambda z: w * z[-1] - (F(z[:-1]) - goal),
         "jac": lambda z: np.hstack([-jac_F(z[:-1])[1], w[:, None]])},
        {"type": "ineq", "fun": lambda z: w * z[-1] + (F(z[:-1]) - goal),
         "jac": lambda z: np.hstack([jac_F(z[:-1])[1], w[:, None]])},
    ]
    bounds = [(lb, None) for lb in par.lb1] + [(None, None)]

    class _Budget(Exception):
        pass

    iterate = [z0]

    def budget(zk):
        iterate[0] = np.array(zk, dtype=float)
        if len(asked) >= max_fun_evals:
            raise _Budget

    try:
        res = minimize(lambda z: z[-1], z0, jac=lambda z: np.eye(n + 1)[-1], method="SLSQP",
                       constraints=cons, bounds=bounds, callback=budget,
                       options={"maxiter": max_iter, "ftol": ftol})
        zf = res.x
    except _Budget:
        zf = iterate[0]
    x = np.maximum(zf[:-1], par.lb1)
    final_eval = last_eval[0]   # the search's own last evaluation, before the report below
    Fx = F(x)
    attain = float(np.max(np.abs(Fx - goal) / w))
    if best[1] is not None and best[0] < attain:
        # SLSQP on finite-difference Jacobians of closed-loop costs can end on a point worse than
        # one it visited (seen on the NMPC: 2.75 -> 13.0); fgoalattain's SQP descends on its merit
        # function, so the best attainment factor found is returned instead
        x = np.maximum(best[1], par.lb1)
        Fx = F(x)
        attain = float(np.max(np.abs(Fx - goal) / w))
    return x, attain, Fx, nb[0], final_eval


# --------------------------------------------------------------------------------------------
def mpc_tfob(par: TuningPar, batch_j1, batch_vns, fv: float = 1e30, log=None, gam_max_iter: int = 400,
             fgam_from: str = "last_eval", stale=None, gam_speculate: bool = False,
             gam_max_fun_evals: int | None = None):
    """MPC_TFob.m:28-143: alternate GAM (weights) and VNS (horizons) until a GAM round does not
    improve.  Quirks kept: Fgam = round(sum(F), 2) where F is the global GAM_fun.m:114 set on its
    LAST call (MPC_TFob.m:104), i.e. the J1 of fgoalattain's last evaluated point, not of the
    returned XOt (fgam_from="returned" takes the returned point instead); OV weights the user set
    to 0 stay 0 (:83-93); the returned delta/lambda are the LAST GAM result, not the best
    (:134-135); VNS2's stale rows on a failed simulation (``stale``, see StaleRows).
    Returns (N, Nu, lam, delta, Fvns, Fvf, fv)."""
    my = par.my
    Fva, Fvf = 10e8, 1e15
    hi = 0
    delta = lam = None
    Fvns = fv
    memo = {}
    while True:
        x, attain, Fx, ncalls, Flast = gam_fgoalattain(
            par, batch_j1, max_iter=gam_max_iter, speculate=gam_speculate, max_fun_evals=gam_max_fun_evals,
            memo=memo.setdefault((int(np.max(par.N)), int(np.max(par.Nu))), {}))
        x = x.copy()
        x[:my][par.ov_zero] = 0.0
        par.x0 = x
        delta = np.abs(x[:my])
        lam = np.abs(x[my:])
        Fgam = round(float(np.sum(Flast if fgam_from == "last_eval" and Flast is not None else Fx)), 2)
        if log:
            log("Fgam=%g; Delta=%s; Lambda=%s; GAM engine calls=%d" % (Fgam, delta, lam, ncalls))
        if Fgam >= Fvf:
            hi += 1
        else:
            Fvf = Fgam
            par.lam, par.delta = lam, delta

        def bv(keys, _d=par.delta, _l=par.lam):
            return batch_vns(keys, _d, _l)

        N, Nu, Xv1, Xv2, Fvns, fv, _, _ = vns2_batched(par, bv, fv, stale=stale)
        if Fvns < Fva:
            Fva = Fvns
            par.N, par.Nu, par.Xv1, par.Xv2 = N, Nu, Xv1, Xv2
        if log:
            log("Fvns=%g; N=%s; Nu=%s" % (Fvns, par.N, par.Nu))
        if hi > 0:
            break
    par.lam, par.delta = lam, delta
    return par.N, par.Nu, par.lam, par.delta, Fvns, Fvf, fv


# --------------------------------------------------------------------------------------------
def scale_record(L, R, nu: int) -> dict:
    """Tuning_Parameters.scale as MPCTuning.m:154-160 builds it: L, R (diagonal CondMin scalings),
    Ru = R(1:ny,1:ny) for the MVs, Rv = R(ny+1:end,ny+1:end) for the measured disturbances (empty
    when there are none); the drivers' resume path reads all four (Shell3x3.m:180-183)."""
    L = np.diag(np.asarray(L, dtype=float).ravel()) if np.ndim(L) < 2 else np.asarray(L, dtype=float)
    R = np.diag(np.asarray(R, dtype=float).ravel()) if np.ndim(R) < 2 else np.asarray(R, dtype=float)
    return {"L": L, "R": R, "Ru": R[:nu, :nu], "Rv": R[nu:, nu:]}


def matlab_datenum(t) -> float:
    """MATLAB datenum of a datetime (days since year 0; datenum(1970,1,1) = 719529)."""
    import datetime

    epoch = datetime.datetime(1970, 1, 1)
    return 719529.0 + (t - epoch).total_seconds() / 86400.0


def save_tuning_parameters(path: str, N, Nu, delta, lam, scale: dict | None = None, date=None):
    """MPCTuning.m:374-381 Tuning_Parameters {N, Nu, delta, lambda, scale.{L,R,Ru,Rv}, date}.
    ``scale``: scale_record(L, R, nu) (a dict holding only L and R is completed with Ru, Rv from
    R's leading nu x nu block: MPCTuning.m:156-157).  ``date``: MATLAB's datetime object cannot be
    written outside MATLAB, so it is stored as its datenum (double; datetime(date,
    'ConvertFrom','datenum') restores it) plus date_str.  The mpc object (Tuning_Parameters.mpcobj)
    is MATLAB-only: the MATLAB host attaches it (matlab/mpct_tuning_record.m).  '.mat' -> MAT v5 via
    scipy, anything else -> JSON.  The drivers' tuning=false path reads N / Nu / delta / lambda /
    scale.{L,R,Ru,Rv} back (Shell3x3.m:176-183)."""
    import datetime

    now = date or datetime.datetime.now()
    Nu_ = np.asarray(Nu, dtype=float).reshape(1, -1)
    rec = {"N": int(np.max(N)), "Nu": Nu_,
           "delta": np.asarray(delta, dtype=float).reshape(1, -1),
           "lambda": np.asarray(lam, dtype=float).reshape(1, -1),
           "date": matlab_datenum(now), "date_str": now.strftime("%d-%b-%Y %H:%M:%S")}
    if scale is not None:
        sc = {k: np.asarray(v, dtype=float) for k, v in scale.items()}
        if "R" in sc and ("Ru" not in sc or "Rv" not in sc):
            sc = scale_record(sc["L"], sc["R"], Nu_.size)
        rec["scale"] = sc
    if path.endswith(".mat"):
        from scipy.io import savemat

        savemat(path, {"Tuning_Parameters": rec})
    else:
        def conv(v):
            if isinstance(v, dict):
                return {k: conv(x) for k, x in v.items()}
            if isinstance(v, np.ndarray):
                return v.tolist()
            return v

        with open(path, "w") as f:
            json.dump({"Tuning_Parameters": conv(rec)}, f, indent=1)
    return rec


# --------------------------------------------------------------------------------------------
def engine_evaluators(sc, r, par: TuningPar, device: int = -1, vns_refs=None, mdv=None):
    """Batched evaluators over the HIP engine (one eval_batch call per batch):
      batch_j1(X rows)                 -> J1 rows  (GAM_fun.m:55-116 with Par.N / Par.Nu, which
                                          closedloop_toolbox reduces with max, :36-40)
      batch_vns(keys, delta, lambda)   -> F per (N, Nu) neighbour (VNS2.m:147-195: my step
                                          simulations for square plants, one simulation with Xsp
                                          for non-square ones, F = sum(j21 + j22) + N(1) + sum(Jnu)).
    mdv = Par.mdv (nd x nit, already scaled by Rv, MPCTuning.m:191) reaches every simulation
    (GAM_fun.m:81, VNS2.m:153,168).  Only fatal statuses (objectives.FATAL_STATUS: the reference's
    sim would have thrown) score NaN; iteration caps keep their finite cost."""
    from .engine import eval_batch
    from .objectives import failed, vns_objective, vns_row1_broadcast

    my, ny = par.my, par.ny
    v = None if mdv is None or np.size(mdv) == 0 else np.asarray(mdv, dtype=float)[None]

    def batch_j1(X):
        X = np.atleast_2d(np.asarray(X, dtype=float))
        C = X.shape[0]
        delta = np.abs(X[:, :my]).copy()
        delta[:, par.ov_zero] = 0.0                   # GAM_fun.m:62-72
        lam = np.abs(X[:, my:my + ny])
        N2 = np.full(C, int(np.max(par.N)), dtype=np.int32)
        Nu = np.full(C, int(np.max(par.Nu)), dtype=np.int32)
        res = eval_batch(sc, N2, Nu, delta, lam, np.asarray(r)[None], v=v, device=device)
        J1 = res.J1.copy()
        J1[failed(res.status)] = np.nan
        return J1

    def vns_terms(keys, delta, lam):
        C = len(keys)
        N2 = np.array([max(k[0]) for k in keys], dtype=np.int32)
        Nu = np.array([max(k[1]) for k in keys], dtype=np.int32)
        d = np.tile(np.asarray(delta, dtype=float), (C, 1))
        l = np.tile(np.asarray(lam, dtype=float), (C, 1))
        F, j21, j22, jnu, res = vns_objective(sc, N2, Nu, d, l, device=device, refs=vns_refs, mdv=mdv)
        return F, j21, j22, jnu, failed(res.status).reshape(C, -1)

    def batch_vns(keys, delta, lam):
        F, j21, j22, jnu, bad = vns_terms(keys, delta, lam)
        return np.where(bad.any(axis=1), np.nan, F)

    def batch_vns_rows(keys, delta, lam):
        """Square plants: per neighbour (T, ok, bcast) with T_i = j21_i + j22_i + Jnu_i of
        simulation i, ok_i = simulation i succeeded and bcast the row-1 broadcast F term (lazy),
        for StaleRows (VNS2.m:151-173)."""
        F, j21, j22, jnu, bad = vns_terms(keys, delta, lam)
        T = j21 + j22 + jnu

        def bcast(key):
            # evaluated at most once per neighbour: the callable rides in vns2_batched's cache entry,
            # so every later score of that neighbour (cache hits, replays) reuses the value
            @functools.lru_cache(maxsize=1)
            def term():
                return vns_row1_broadcast(sc, max(key[0]), max(key[1]), delta, lam, device=device,
                                          refs=vns_refs, mdv=mdv)
            return term
        return [(T[k], ~bad[k], bcast(keys[k])) for k in range(len(keys))]

    batch_vns.rows = batch_vns_rows if my == ny else None
    return batch_j1, batch_vns


def stale_rows_for(yref, inK: int = 10) -> StaleRows:
    """VNS2's row state before its first simulation: zero rows score T_i0 = sum_{t >= inK}
    Yref_i(t)^2 (Xy = Xyma = Xuma = 0: j21 = 0, Jnu = 0/0 -> 0, VNS2.m:172-191)."""
    Y = np.asarray(yref, dtype=float)
    return StaleRows((Y[:, inK - 1:] ** 2).sum(1))


def mpc_tuning(sc, r, my: int, ny: int, w, nbp: int = 7, nbc: int = 4, dmin=None, q0=None, w0=None,
               device: int = -1, log=None, save_path: str | None = None, scale: dict | None = None,
               gam_max_iter: int = 400, lineal: bool = True, mdv=None, fgam_from: str = "last_eval",
               stale_rows: bool = True, gam_speculate: bool = False, gam_max_fun_evals: int | None = None):
    """MPCTuning.m:93-381 on an already scaled scenario (mpct.scenarios builds Pze = L*Pz*R, the
    scaled bounds, L*Xsp and L*Yref from the committed L, R -- MPCTuning.m:154-189).  Returns
    (N, Nu, delta, lambda, Fob = [Fvns, Fgam]) and optionally writes Tuning_Parameters.
    lineal = False: a nonlinear (NMPC) scenario (MPCTuning.m:202-250): VNS simulates the driver's
    setpoint one output at a time instead of unit steps (VNS2.m:67-71,148-155).
    fgam_from / stale_rows: the MPC_TFob.m:104 and VNS2.m:151-163 quirks (mpc_tfob, StaleRows);
    "returned" / False give the round-2 behaviour (Fgam at the returned point, failed -> NaN).
    gam_max_fun_evals: fgoalattain's MaxFunctionEvaluations (None: its default 100 * (my + ny),
    which MPCTuning.m:88-91 keeps; gam_fgoalattain)."""
    par = TuningPar(my=my, ny=ny, nbp=nbp, nbc=nbc, dmin=dmin, w=w, q0=q0, w0=w0, nit=sc.nit)
    if sc.n2_max < 2 ** par.nbp - 1 or sc.nu_max < 2 ** par.nbc - 1:
        raise ValueError("scenario horizons (n2_max=%d, nu_max=%d) must cover the bit ranges "
                         "(%d, %d)" % (sc.n2_max, sc.nu_max, 2 ** par.nbp - 1, 2 ** par.nbc - 1))
    vns_refs = None
    if not lineal:
        from .objectives import vns_refs_nonlinear

        # square: Xsp.*sel one output at a time (VNS2.m:148-155); non-square: Xsp whole (:168)
        vns_refs = vns_refs_nonlinear(r) if my == ny else np.asarray(r, dtype=float)[None]
    batch_j1, batch_vns = engine_evaluators(sc, r, par, device=device, vns_refs=vns_refs, mdv=mdv)
    stale = None
    if stale_rows and batch_vns.rows is not None:   # square plants (VNS2.m:148-165)
        stale = stale_rows_for(sc.yref)
        batch_vns = batch_vns.rows
    N, Nu, lam, delta, Fvns, Fgam, _ = mpc_tfob(par, batch_j1, batch_vns, fv=1e30, log=log,
                                                  gam_max_iter=gam_max_iter, fgam_from=fgam_from, stale=stale,
                                                  gam_speculate=gam_speculate, gam_max_fun_evals=gam_max_fun_evals)
    if save_path:
        save_tuning_parameters(save_path, N, Nu, delta, lam, scale=scale)
    return N, Nu, delta, lam, np.array([Fvns, Fgam])
