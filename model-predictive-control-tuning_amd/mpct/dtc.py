"""DTC-GPC setup on the host: the robustness filter design of mimofilter.m /
filtro_siso.m and the WoodBerry configuration of DTC_GPC_WW.m.  The closed loop itself runs on
the GPU engine in DTC mode (mpct_scenario_desc.dtc = 1): the free response is driven by the
predictor yp = Gz*u + Fr*(y - Pz*u) (OptimalPredictor2.m:24-40), kept as recursions instead of
the reference's full-history lsim."""
from __future__ import annotations

import numpy as np

from .lti import Tf, c2d, carima, descomp


def _solve_mldivide(A, B):
    """A\\B as MATLAB evaluates it: square -> LU; underdetermined -> the basic solution of a
    column-pivoted QR (rank(A) nonzeros), which filtro_siso.m:85 hits when the delay is 0."""
    import scipy.linalg as sla

    if A.shape[0] == A.shape[1]:
        return sla.solve(A, B)
    Q, R, piv = sla.qr(A, mode="economic", pivoting=True)
    tol = max(A.shape) * np.finfo(float).eps * abs(R[0, 0])
    r = int(np.sum(np.abs(np.diag(R)) > tol))
    x = np.zeros(A.shape[1])
    x[piv[:r]] = sla.solve_triangular(R[:r, :r], (Q.T @ B)[:r])
    return x


def robust_filter(den, d: int, alfa: float = 0.7, raio: float = 0.8):
    """filtro_siso.m:12-96 for a fast model with denominator den (z, descending) and dead time d:
    Fr = Nr(z) / (z - alfa)^nk with Nr chosen so that the poles |p| >= raio of the model are
    cancelled in the predictor error dynamics (Sylvester system).  Returns Tf(Nr, Dr, 0)."""
    poles = np.roots(np.asarray(den, dtype=float)) if len(den) > 1 else np.zeros(0)
    bad = [p for p in poles if abs(p) >= raio]
    if not bad:
        return Tf.make([1.0], [1.0], 0)
    pd = 2 if d == 0 else 0
    nk = len(bad) + pd
    px = np.real(np.poly(np.concatenate([[1.0], bad])))        # (z - 1) * prod (z - p_bad)
    Dr = np.array([1.0])
    for _ in range(nk):
        Dr = np.convolve(Dr, [1.0, -alfa])
    order = (Dr.size - 1) + d
    A = np.zeros((order + 1, order + 1 + pd))
    for c, col in enumerate(range(order + 1 - d, order + 1 + pd)):  # shifted copies of px
        rows = np.arange(c, min(order + 1, c + px.size))
        A[rows, col] = px[: rows.size]
    for c, row in enumerate(range(d, order + 1)):                   # the Nr block
        A[row, c] = 1.0
    B = np.zeros(order + 1)
    B[0] = 1.0
    B[1:Dr.size] = Dr[1:]
    X = _solve_mldivide(A, B)
    return Tf.make(X[: order + 1 - d], Dr, 0)


def mimofilter(P, alfa: float = 0.7, raio: float = 0.8):
    """mimofilter.m:16-50: one filter per output, designed on the product of the row's nonzero
    entries (poles of H_i = prod_j P_ij) with dead time dmin_i.  P: my x nu of Tf."""
    filters = []
    for row in P:
        dmin = min(t.delay for t in row)
        den = np.array([1.0])
        any_nz = False
        for t in row:
            if np.sum(t.num) != 0:
                den = np.convolve(den, np.asarray(t.den, dtype=float))
                any_nz = True
        filters.append(robust_filter(den, dmin, alfa, raio) if any_nz else Tf.make([1.0], [1.0], 0))
    return filters


# --------------------------------------------------------------------------------------------
WB_K = np.array([[12.8, -18.9], [6.6, -19.4]])     # DTC_GPC_WW.m:23-28 (Wood & Berry)
WB_TAU = np.array([[16.7, 21.0], [10.9, 14.4]])
WB_L = np.array([[1.0, 2.0], [2.0, 1.0]])
WB_QK = np.array([3.8, 4.9])                       # DTC_GPC_WW.m:29-30 disturbance path Pq
WB_QTAU = np.array([14.9, 13.2])
WB_QL = np.array([8.1, 3.4])


def woodberry_dtc(n2_max: int = 30, nu_max: int = 10, nit: int = 200, deltak: float = 0.0,
                  deltaL: float = 0.0, alfa: float = 0.7, raio: float = 0.8, filt: bool = True):
    """DTC_GPC_WW.m:18-124 configuration (config 1) on the engine, CondMin-free (L = R = I):
    Ts = 1, real plant P (gain/delay mismatch deltak, deltaL), nominal model Pn, disturbance
    path Pq; unconstrained; Q = diag(delta), W = diag(lambda) unsquared; BA_MIMO's rounded LCM.
    Returns (Scenario, r [2 x nit], q [1 x nit])."""
    from .engine import Scenario

    Ts = 1.0
    P = [[c2d([WB_K[i, j] * (1 + deltak)], [WB_TAU[i, j], 1.0], Ts, WB_L[i, j] + deltaL) for j in range(2)]
         for i in range(2)]
    Pn = [[c2d([WB_K[i, j]], [WB_TAU[i, j], 1.0], Ts, WB_L[i, j]) for j in range(2)] for i in range(2)]
    Pq = [[c2d([WB_QK[i]], [WB_QTAU[i], 1.0], Ts, WB_QL[i])] for i in range(2)]
    filters = mimofilter(Pn, alfa, raio) if filt else None
    r = np.zeros((2, nit))
    r[0, 10:] = 0.8                                  # DTC_GPC_WW.m:117-119
    r[1, 60:] = 0.5
    q = np.zeros((1, nit))
    q[0, 140:] = -0.25                               # DTC_GPC_WW.m:123-124
    inf = np.full(2, np.inf)
    sc = Scenario(P, Pn, nu=2, du_min=-inf, du_max=inf, u_min=-inf, u_max=inf, yref=r,
                  n2_max=n2_max, nu_max=nu_max, Ts=Ts, window="gpc", weights_squared=False,
                  exact_carima=False, dtc=True, filters=filters, dist=Pq)
    return sc, r, q


# --------------------------------------------------------------------------------------------
def woodberry_mc_plants(draws: int, seed: int = 20250307, gain_spread: float = 0.2, max_dshift: int = 2,
                        Ts: float = 1.0):
    """SURVEY §8d config 4 plant-mismatch draws modelled on DTC_GPC_WW.m:18-19 (deltak, deltaL):
    each entry's gain x (1 + U(-gain_spread, gain_spread)) and delay + U{0..max_dshift} * Ts,
    numpy default_rng(seed).  Returns a list of 2x2 plants (mpct.lti.Tf)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(draws):
        g = 1.0 + rng.uniform(-gain_spread, gain_spread, (2, 2))
        dl = rng.integers(0, max_dshift + 1, (2, 2))
        out.append([[c2d([WB_K[i, j] * g[i, j]], [WB_TAU[i, j], 1.0], Ts, WB_L[i, j] + dl[i, j] * Ts)
                     for j in range(2)] for i in range(2)])
    return out


def config4_candidates(C: int = 10000, seed: int = 20250307, p_max: int = 30, m_max: int = 10):
    """SURVEY §8d config 4 candidate grid: p in 3..p_max, m in 1..min(p, m_max), then log10 lambda
    and log10 delta ~ U(-3, 1), numpy default_rng(seed) in that order.  Returns (N2, Nu, delta,
    lambda) in the engine's candidate layout (one p / m for both loops: the toolbox-style max)."""
    rng = np.random.default_rng(seed)
    N2 = rng.integers(3, p_max + 1, C).astype(np.int32)
    Nu = np.array([rng.integers(1, min(int(p), m_max) + 1) for p in N2], dtype=np.int32)
    lam = 10.0 ** rng.uniform(-3, 1, (C, 2))
    delta = 10.0 ** rng.uniform(-3, 1, (C, 2))
    return N2, Nu, delta, lam


def woodberry_mc(draws: int = 32, n2_max: int = 30, nu_max: int = 10, nit: int = 200, seed: int = 20250307,
                 alfa: float = 0.7, raio: float = 0.8):
    """Config 4 scenario: the DTC-GPC of woodberry_dtc evaluated over `draws` mismatched plants
    (variant k runs with reference row k).  Returns (Scenario, refs [draws, 2, nit],
    v [draws, 1, nit], plants)."""
    from .engine import Scenario

    base, r, q = woodberry_dtc(n2_max=2, nu_max=1, nit=nit)        # for r, q and the model
    plants = woodberry_mc_plants(draws, seed)
    Pn = base.model
    Pq = [[c2d([WB_QK[i]], [WB_QTAU[i], 1.0], 1.0, WB_QL[i])] for i in range(2)]
    inf = np.full(2, np.inf)
    sc = Scenario(plants[0], Pn, nu=2, du_min=-inf, du_max=inf, u_min=-inf, u_max=inf, yref=r,
                  n2_max=n2_max, nu_max=nu_max, Ts=1.0, window="gpc", weights_squared=False,
                  exact_carima=False, dtc=True, filters=mimofilter(Pn, alfa, raio), dist=Pq,
                  plant_variants=plants)
    base.close()
    refs = np.broadcast_to(r, (draws, 2, nit)).copy()
    v = np.broadcast_to(q, (draws, 1, nit)).copy()
    return sc, refs, v, plants


def robust_scores(J1, C: int, draws: int):
    """Per-candidate robustness scores over the draws: (mean, worst) of sum_i J1_i, where J1 is
    the engine's (C*draws, my) cost array in simulation order (candidate-major)."""
    J = np.asarray(J1).reshape(C, draws, -1).sum(axis=2)
    return J.mean(axis=1), J.max(axis=1)
