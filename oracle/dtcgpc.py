"""Restated DTC-GPC primitives (reference ``DTC-GPC/*.m``) — oracle, test infrastructure only.

Indexing: Python lists of lists stand in for MATLAB cells ``{i,j}``; all horizons/rows are
1-based in the docstrings (as in the .m files) and 0-based in code.
"""
from __future__ import annotations

import numpy as np

from .matlab import DTF, conv, lsim_dtf, mround, poly, roots, step_dtf


# ---------------------------------------------------------------------------------------------
def descomp_mpc(P):
    """descompMPC.m:19-43.  ``P`` is an my x nin matrix of DTF (tfdata 'v' form).

    Returns (B, A, d): cells of numerator / denominator rows and the delay matrix, after the
    two adjustments of descompMPC.m:35-41:
      * if B{i,j}(1) ~= 0: d(i,j) = d(i,j)-1 and B{i,j} = [0 B{i,j}]   (keep u(k-1) causal)
      * if dcgain(P(i,j)) == 0: d(i,j) = max(d(i,:))   (zero entry takes the row's max delay)
    """
    my = len(P)
    nin = len(P[0])
    B = [[None] * nin for _ in range(my)]
    A = [[None] * nin for _ in range(my)]
    d = np.zeros((my, nin), dtype=int)
    for i in range(my):
        for j in range(nin):
            B[i][j] = np.array(P[i][j].num, dtype=float)
            A[i][j] = np.array(P[i][j].den, dtype=float)
            d[i, j] = P[i][j].iodelay
    for i in range(my):
        for j in range(nin):
            if B[i][j][0] != 0:  # Q = inf default -> condition u < Q(1) always true
                d[i, j] -= 1
                B[i][j] = np.concatenate([[0.0], B[i][j]])
            if P[i][j].dcgain() == 0:
                d[i, j] = d[i, :].max()
    return B, A, d


# ---------------------------------------------------------------------------------------------
def ba_mimo(Bn, An, round_roots: bool = True):
    """BA_MIMO.m:20-71.  Least-common-multiple denominator per output row and the matching
    numerators.

    round_roots=True is the reference verbatim: LCM poles are ``unique(round(roots(prod),4))``
    (BA_MIMO.m:38-40) and B{i,j} = Bn{i,j} * poly(LCM roots not in round(roots(An{i,j}),4))
    (BA_MIMO.m:48-60), including its index-skipping removal loop.  This perturbs the model by
    ~1e-5 (a deliberate model change in the reference).

    round_roots=False is the exact-model variant used for toolbox-equivalent semantics
    (SURVEY §7 "two modes"): the LCM is the product of the DISTINCT denominator polynomials of
    the row (duplicates detected by coefficient equality), so the CARIMA model equals the plant
    up to rounding.  Returns (B, A, na, nb) with A a list (A{i,i}).
    """
    p = len(An)
    m = len(An[0])
    Bn = [[np.array(Bn[i][j], dtype=float) for j in range(m)] for i in range(p)]
    for i in range(p):
        for j in range(m):
            if Bn[i][j][0] == 0:  # BA_MIMO.m:21-23 strip ONE leading zero
                Bn[i][j] = Bn[i][j][1:]
    A = [None] * p
    B = [[None] * m for _ in range(p)]
    if round_roots:
        for i in range(p):
            aux = An[i][0]
            for j in range(1, m):
                aux = conv(aux, An[i][j])
            A[i] = aux
            if p != 1:
                au1 = mround(roots(aux), 4)
                pol = np.unique(au1)
                A[i] = np.real(poly(pol))
        for i in range(p):
            for j in range(m):
                aux = Bn[i][j]
                rA = list(mround(roots(A[i]), 4))
                rAn = list(mround(roots(An[i][j]), 4))
                kk = 0
                while kk < len(rA):
                    for jj in range(len(rAn)):
                        # MATLAB: if rA(kk)==rAn(jj), rA = rA(rA ~= rA(kk)) — index may now be
                        # out of range for the next jj (MATLAB would error); keep the same order.
                        if rA[kk] == rAn[jj]:
                            v = rA[kk]
                            rA = [x for x in rA if x != v]
                            if kk >= len(rA):
                                break
                    kk += 1
                pA = np.real(poly(np.array(rA))) if rA else np.ones(1)
                B[i][j] = conv(aux, pA)
    else:
        for i in range(p):
            uniq = []
            for j in range(m):
                dj = np.asarray(An[i][j], dtype=float)
                if not any(len(dj) == len(u) and np.array_equal(dj, u) for u in uniq):
                    uniq.append(dj)
            A[i] = np.ones(1)
            for u in uniq:
                A[i] = conv(A[i], u)
            for j in range(m):
                aux = Bn[i][j]
                dj = np.asarray(An[i][j], dtype=float)
                for u in uniq:
                    if not (len(dj) == len(u) and np.array_equal(dj, u)):
                        aux = conv(aux, u)
                B[i][j] = aux
    na = np.array([len(A[i]) - 1 for i in range(p)])
    nb = np.array([[len(B[i][j]) - 1 for j in range(m)] for i in range(p)])
    return B, A, na, nb


# ---------------------------------------------------------------------------------------------
def diophantine(A, N: int, d: int):
    """diophantine.m:23-79 (Normey-Rico & Camacho).  A~ = conv(A,[1 -1]); F rows for the window
    N1 = d+1 .. N2 = d+N; E rows N1..N2 (each a length-N2 row, E_j left-aligned)."""
    AD = conv(A, [1.0, -1.0])
    nAD = len(AD)
    N1 = d + 1
    N2 = d + N
    f = np.zeros((N2 + 1, nAD - 1))
    f[0, 0] = 1.0
    for j in range(N2):
        for i in range(nAD - 2):
            f[j + 1, i] = f[j, i + 1] - f[j, 0] * AD[i + 1]
        f[j + 1, nAD - 2] = -f[j, 0] * AD[nAD - 1]
    F = f[N1: N2 + 1, :]
    E = np.zeros((N2, N2))
    e = [1.0]
    E[0, 0] = 1.0
    for i in range(2, N2 + 1):
        e.append(f[i - 1, 0])
        E[i - 1, :i] = e
    E = E[N1 - 1: N2, :]
    return E, F


def diophantine_mimo(A, N, dmin):
    """diophantineMIMO.m:15-21 — per output on A{i,i}.  Returns (E, En, F) lists."""
    E, En, F = [], [], []
    for i in range(len(A)):
        En1, Fn = diophantine(A[i], int(N[i]), int(dmin[i]))
        E.append(En1[-1, :])
        F.append(Fn)
        En.append(En1)
    return E, En, F


# ---------------------------------------------------------------------------------------------
def mat_g(P, N, Nu, d):
    """MatG.m:38-74.  Dynamic matrix from step responses:
    G{i,j}(k:end, k) = g(dmin(i)+2 : dmin(i)+N(i)-k+2), g = step(P(i,j), (N(i)+dmin(i))*Ts).

    Row r (0-based) of block i therefore predicts y_i(t + dmin(i) + 1 + r); column c is
    Delta u_j(t + c).  Passing d == 0 gives the toolbox window t+1..t+N.  Returns (MG, MGc)."""
    s = len(P)
    e = len(P[0]) if s else 0
    d = np.atleast_2d(np.asarray(d))
    dmin = d.ravel() if e == 1 else d.min(axis=1)
    H = [[None] * e for _ in range(s)]
    for i in range(s):
        for j in range(e):
            g = step_dtf(P[i][j], int(N[i] + dmin[i]) + 1)
            G = np.zeros((int(N[i]), int(Nu[j])))
            for k in range(1, int(Nu[j]) + 1):
                lo = int(dmin[i]) + 2
                hi = int(dmin[i]) + int(N[i]) - k + 2
                G[k - 1:, k - 1] = g[lo - 1: hi]
            H[i][j] = G
    MG = np.block(H)
    return MG, H


# ---------------------------------------------------------------------------------------------
def delta_u_free(B, En, N, dp):
    """deltaUFree.m:13-62.  uG{m,n}(i,:) = last cp coefficients of conv(En{m}(i,:), B{m,n})
    after removing ALL zero coefficients (deltaUFree.m:40-45: the loop keeps aux(j) ~= 0 for
    every j, not only trailing ones), cp = dp(m,n) + length(B{m,n}) - 1, left-padded with zeros
    when shorter.  Column order: Delta u(t-1), Delta u(t-2), ..., Delta u(t-cp)."""
    ny = len(B)
    nu = len(B[0])
    uG = [[None] * nu for _ in range(ny)]
    for m in range(ny):
        for n in range(nu):
            cp = int(dp[m][n]) + len(B[m][n]) - 1
            if cp < 1:
                cp = 1
            uG1 = np.zeros((int(N[m]), cp))
            for i in range(int(N[m])):
                aux = conv(En[m][i, :], B[m][n])
                BE = [a for a in aux if a != 0]
                lBE = len(BE)
                if lBE < cp:
                    uG1[i, :] = np.concatenate([np.zeros(cp - lBE), BE])
                else:
                    uG1[i, :] = BE[lBE - cp:]
            uG[m][n] = uG1
    return uG


def cell2mat2(Bc):
    """cell2mat2.m:25-58 — left-aligned block assembly; block column width = max rows' widths,
    block row height = max columns' heights."""
    m = len(Bc)
    n = len(Bc[0])
    f1 = np.array([[Bc[i][j].shape[0] for j in range(n)] for i in range(m)])
    c1 = np.array([[Bc[i][j].shape[1] for j in range(n)] for i in range(m)])
    c1m = np.concatenate([[0], c1.max(axis=0)])
    f1m = np.concatenate([[0], f1.max(axis=1)])
    n1 = max(c1[i].sum() for i in range(m))
    m1 = f1.max(axis=1).sum()
    A = np.zeros((m1, max(n1, c1m.sum())))
    for i in range(m):
        for j in range(n):
            r0 = f1m[: i + 1].sum()
            c0 = c1m[: j + 1].sum()
            A[r0: r0 + f1[i, j], c0: c0 + c1[i, j]] = Bc[i][j]
    return A[:, : c1m.sum()]


def blkdiag(*mats):
    rows = sum(a.shape[0] for a in mats)
    cols = sum(a.shape[1] for a in mats)
    out = np.zeros((rows, cols))
    r = c = 0
    for a in mats:
        out[r: r + a.shape[0], c: c + a.shape[1]] = a
        r += a.shape[0]
        c += a.shape[1]
    return out


# ---------------------------------------------------------------------------------------------
# DTC-GPC robustness filter and predictor (config 1)
# ---------------------------------------------------------------------------------------------
def _mldivide(A, B):
    """MATLAB A\\B: square -> LU solve; rectangular underdetermined -> the basic solution of a
    column-pivoted QR (at most rank(A) nonzeros), as mldivide returns it."""
    import scipy.linalg as sla

    A = np.asarray(A, dtype=float)
    B = np.asarray(B, dtype=float)
    if A.shape[0] == A.shape[1]:
        return np.linalg.solve(A, B)
    Q, R, piv = sla.qr(A, mode="economic", pivoting=True)
    r = int(np.sum(np.abs(np.diag(R)) > max(A.shape) * np.finfo(float).eps * abs(R[0, 0])))
    x = np.zeros(A.shape[1])
    x[piv[:r]] = sla.solve_triangular(R[:r, :r], (Q.T @ B)[:r])
    return x


def filtro_siso(num, den, d: int, alfa: float, raio: float, kn: int = 2):
    """filtro_siso.m:12-96.  Robustness filter Fr(z) = Nr(z)/Dr(z) for the fast model
    num/den (z, descending powers) with dead time d: the unwanted poles |p| >= raio are
    cancelled (Sylvester system A X = B, :52-83) and Dr = (z - alfa)^nk (:42-45).  kn is unused
    by the reference.  Returns (Nr, Dr); (1, 1) when no pole is unwanted (:89-93)."""
    polos = roots(den)
    p_ind = [p for p in polos if abs(p) >= raio]            # :27
    nm = len(p_ind)
    nk = nm
    pd = 0
    if d == 0:                                               # :31-35
        pd = 2
        nk += pd
    px = np.real(poly([1.0] + list(p_ind)))                  # :37-39
    Dr = np.array([1.0])
    for _ in range(nk):
        Dr = conv(Dr, [1.0, -alfa])
    ordem = (len(Dr) - 1) + d                                # :46
    lpx = len(px)
    A = np.zeros((ordem + 1, ordem + 1 + pd))
    ip = 1
    for j in range(ordem + 2 - d, ordem + 2 + pd):           # :52-65 (1-based columns)
        pn = 1
        for i in range(ip, ordem + 2):
            if pn <= lpx:
                A[i - 1, j - 1] = px[pn - 1]
                pn += 1
        ip += 1
    j = 1
    for i in range(d + 1, ordem + 2):                        # :67-70
        A[i - 1, j - 1] = 1.0
        j += 1
    B = np.zeros(ordem + 1)
    B[0] = 1.0
    B[1:len(Dr)] = Dr[1:]
    X = _mldivide(A, B)
    Nr = X[:ordem + 1 - d]
    if nm == 0:
        return np.array([1.0]), np.array([1.0])
    return np.asarray(Nr, dtype=float), Dr


def mimofilter(Pd, alfa: float = 0.7, raio: float = 0.8, kn: int = 2):
    """mimofilter.m:16-50: one filter per output on the product of the row's nonzero entries
    (H(i) = prod_j G(i,j), delay dmin(i)).  Pd: my x n DTF.  Returns a list of (Nr, Dr)."""
    my = len(Pd)
    Fr = []
    for i in range(my):
        dmin_i = min(Pd[i][j].iodelay for j in range(len(Pd[i])))
        num, den = np.array([1.0]), np.array([1.0])
        for j in range(len(Pd[i])):
            if np.sum(Pd[i][j].num) != 0:
                num = conv(num, np.trim_zeros(Pd[i][j].num, "f"))
                den = conv(den, Pd[i][j].den)
        if np.sum(num) == 0:
            Fr.append((np.array([1.0]), np.array([1.0])))
        else:
            Fr.append(filtro_siso(num, den, int(dmin_i), alfa, raio, kn))
    return Fr


def optimal_predictor2(Fr, Pz, Gz, u, y, k: int):
    """OptimalPredictor2.m:24-40, full history (the reference structure, O(k) per call):
    yp = Gz*u + Fr*(y - Pz*u) over samples 1..k."""
    from .matlab import lsim_mimo

    U = np.asarray(u)[:, :k]
    ypz = lsim_mimo(Pz, U)
    ygz = lsim_mimo(Gz, U)
    eM = np.asarray(y)[:, :k] - ypz
    yfr = np.zeros_like(eM)
    for i, (Nr, Dr) in enumerate(Fr):
        yfr[i] = lsim_dtf(DTF(Nr, Dr, 0), eM[i])
    return ygz + yfr


def woodberry_models(deltak: float = 0.0, deltaL: float = 0.0, Ts: float = 1.0):
    """DTC_GPC_WW.m:18-41 models, CondMin-free variant L = R = I (CondMin's fmincon result is
    not unique and no WoodBerry tuning file is committed): real plant P (gain / delay
    mismatch deltak, deltaL), nominal Pn, disturbance path Pq -- all discretised ZOH (lsim of
    the continuous plant with 'zoh' input is exactly this)."""
    from .matlab import c2d_zoh

    K = np.array([[12.8, -18.9], [6.6, -19.4]])
    tau = np.array([[16.7, 21.0], [10.9, 14.4]])
    L = np.array([[1.0, 2.0], [2.0, 1.0]])
    P = [[c2d_zoh([K[i, j] * (1 + deltak)], [tau[i, j], 1.0], Ts, L[i, j] + deltaL) for j in range(2)]
         for i in range(2)]
    Pn = [[c2d_zoh([K[i, j]], [tau[i, j], 1.0], Ts, L[i, j]) for j in range(2)] for i in range(2)]
    Pq = [[c2d_zoh([3.8], [14.9, 1.0], Ts, 8.1)], [c2d_zoh([4.9], [13.2, 1.0], Ts, 3.4)]]
    return P, Pn, Pq


def woodberry_mc_draws(draws: int, seed: int = 20250307, gain_spread: float = 0.2, max_dshift: int = 2,
                       Ts: float = 1.0):
    """SURVEY §8d config 4 plant-mismatch draws, modelled on DTC_GPC_WW.m:18-19 (P = Pn with the
    gain scaled by 1 + deltak and the delay shifted by deltaL), one draw per entry: gain x
    (1 + U(-gain_spread, gain_spread)), delay + U{0..max_dshift}*Ts, numpy default_rng(seed),
    drawn per plant in the order (gain 2x2, delay shift 2x2).  Returns [draws] 2x2 DTF plants."""
    from .matlab import c2d_zoh

    K = np.array([[12.8, -18.9], [6.6, -19.4]])
    tau = np.array([[16.7, 21.0], [10.9, 14.4]])
    L = np.array([[1.0, 2.0], [2.0, 1.0]])
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(draws):
        g = 1.0 + rng.uniform(-gain_spread, gain_spread, (2, 2))
        dl = rng.integers(0, max_dshift + 1, (2, 2))
        out.append([[c2d_zoh([K[i, j] * g[i, j]], [tau[i, j], 1.0], Ts, L[i, j] + dl[i, j] * Ts)
                     for j in range(2)] for i in range(2)])
    return out


def dtc_gpc_ww(p=(3, 3), m=(3, 3), lam=(1.0, 1.0), delta=(1.0, 1.0), nit: int = 200, deltak: float = 0.0,
               deltaL: float = 0.0, alfa: float = 0.7, raio: float = 0.8, disturbance: bool = True,
               filt: bool = True, plant=None):
    """DTC_GPC_WW.m:59-164 (config 1), reference structure: every step re-simulates the whole
    history with lsim (plant, disturbance path and the three predictor models), O(nit^2).
    L = R = I.  ``plant``: a 2x2 DTF real plant replacing P of DTC_GPC_WW.m:18-19 (one
    Monte-Carlo draw of config 4, woodberry_mc_draws); the model stays nominal.
    Returns dict(y, u, yp, r, q)."""
    P, Pn, Pq = woodberry_models(deltak, deltaL)
    if plant is not None:
        P = plant
    my = ny = 2
    Pnz = Pn
    Bp, Ap, dp = descomp_mpc(Pnz)
    dmin = np.array([dp[i, :].min() for i in range(my)])
    Gnz = [[DTF(Pnz[i][j].num, Pnz[i][j].den, Pnz[i][j].iodelay - dmin[i]) for j in range(ny)]
           for i in range(my)]
    dnz = dp - dmin[:, None]
    p = list(p)
    m = list(m)
    W = np.diag(np.concatenate([lam[i] * np.ones(m[i]) for i in range(ny)]))   # :67-71
    Q = np.diag(np.concatenate([delta[i] * np.ones(p[i]) for i in range(my)]))  # :72-76
    B, A, na, nb = ba_mimo(Bp, Ap)                           # :79
    E, En, F = diophantine_mimo(A, p, [0, 0])                # :80
    S = blkdiag(*[F[i][: p[i], :] for i in range(my)])
    H, _ = mat_g(Pnz, p, m, dp)                              # :89
    uG = delta_u_free(B, En, p, dnz)                         # :91
    Hp = cell2mat2(uG)
    duM = (nb + dnz).max(axis=0)                             # :93
    up = np.zeros(int(duM.sum()))
    S1 = H.T @ Q @ H + W
    S1 = (S1 + S1.T) / 2
    K = np.linalg.solve(S1, H.T @ Q)                         # :98-100
    Km = np.stack([K[int(sum(m[:i]))] for i in range(ny)])
    Fr = mimofilter(Pnz, alfa, raio) if filt else [(np.array([1.0]), np.array([1.0]))] * my
    r = np.zeros((my, nit))
    r[0, 10:] = 0.8                                          # :117-119 (1-based 11, 61)
    r[1, 60:] = 0.5
    q = np.zeros((1, nit))
    if disturbance:
        q[0, 140:] = -0.25                                   # :123-124
    u = np.zeros((ny, nit))
    ue = np.zeros((ny, nit))
    y = np.zeros((my, nit))
    yp = np.zeros((my, nit))
    from .matlab import lsim_mimo

    for k in range(4, nit + 1):                              # :126 (1-based k)
        yq = lsim_mimo(Pq, q[:, :k])
        yk = lsim_mimo(P, u[:, :k]) + yq
        y[:, :k] = yk
        ye = yk
        ypk = optimal_predictor2(Fr, Pnz, Gnz, ue, ye, k)
        yp[:, :k] = ypk
        Yd = np.concatenate([ypk[j, k - 1 - np.arange(na[j] + 1)] for j in range(my)])
        Ref = np.concatenate([np.full(p[i], r[i, k - 1]) for i in range(my)])
        yf = Hp @ up + S @ Yd
        dU = Km @ (Ref - yf)
        off = 0
        for i in range(ny):
            blk = up[off: off + duM[i]].copy()
            up[off: off + duM[i]] = np.concatenate([[dU[i]], blk[:-1]])
            off += duM[i]
        ue[:, k - 1] = (ue[:, k - 2] if k > 1 else 0.0) + dU
        u[:, k - 1] = ue[:, k - 1]
    return dict(y=y, u=u, yp=yp, r=r, q=q, Fr=Fr, Km=Km, S=S, Hp=Hp, dmin=dmin, duM=duM)
