"""Host-side LTI model handling for scenario construction (product code).

The MATLAB host gets these from the Control System Toolbox (c2d, tfdata, dcgain) and from the
reference's own descompMPC.m / BA_MIMO.m; this module provides the same for the Python host.
Everything here runs once per scenario on the CPU and feeds the C ABI descriptor.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
from scipy.linalg import expm


@dataclass(frozen=True)
class Tf:
    """SISO discrete tf  z^-delay num(z)/den(z)  in tfdata('v') form (equal lengths)."""

    num: tuple
    den: tuple
    delay: int = 0

    @staticmethod
    def make(num, den, delay=0) -> "Tf":
        num = np.atleast_1d(np.asarray(num, dtype=float))
        den = np.atleast_1d(np.asarray(den, dtype=float))
        n = max(num.size, den.size)
        num = np.pad(num, (n - num.size, 0))
        den = np.pad(den, (n - den.size, 0))
        return Tf(tuple(num.tolist()), tuple(den.tolist()), int(delay))

    def scale(self, k: float) -> "Tf":
        return Tf(tuple((np.asarray(self.num) * k).tolist()), self.den, self.delay)

    @property
    def dcgain(self) -> float:
        s = float(np.sum(self.den))
        return float(np.sum(self.num)) / s if s != 0.0 else float("inf")

    def impulse_form(self):
        """(b, a) in z^-1 powers, delay folded into b: y(t) = b*u(t-.) - a[1:]*y(t-.)."""
        den = np.asarray(self.den)
        b = np.concatenate([np.zeros(self.delay), np.asarray(self.num)]) / den[0]
        return b, den / den[0]


def c2d(num, den, Ts: float, delay: float = 0.0) -> Tf:
    """ZOH discretisation of num(s)/den(s) e^{-delay s} with a fractional delay
    (Control System Toolbox c2d(sys,Ts,'zoh') as called at Shell3x3.m:65).

    delay = D*Ts + theta: x+ = Phi x + G0 u[t-D] + G1 u[t-D-1]; MATLAB reports theta > 0 as
    iodelay D+1 with a full-degree numerator and theta == 0 as iodelay D."""
    den = np.trim_zeros(np.asarray(den, dtype=float), "f")
    num = np.asarray(num, dtype=float)
    n = den.size - 1
    den_n = den / den[0]
    num_n = np.pad(num / den[0], (max(0, n - num.size), 0))[-n:]
    A = np.zeros((n, n))
    A[0] = -den_n[1:]
    A[1:, :-1] = np.eye(n - 1)
    B = np.zeros((n, 1))
    B[0, 0] = 1.0
    Cm = num_n[None, :]

    def zoh(T):
        Maug = np.zeros((n + 1, n + 1))
        Maug[:n, :n] = A * T
        Maug[:n, n:] = B * T
        E = expm(Maug)
        return E[:n, :n], E[:n, n:]

    D = int(np.floor(delay / Ts + 1e-12))
    theta = delay - D * Ts
    if abs(theta) < 1e-12 * max(1.0, Ts):
        theta = 0.0
    Phi = expm(A * Ts)
    _, G0 = zoh(Ts - theta)
    cp = np.real(np.poly(Phi))

    def numer(Gam):
        return np.real(np.poly(Phi - Gam @ Cm)) - cp

    if theta == 0.0:
        return Tf.make(numer(G0), cp, D)
    _, I1 = zoh(theta)
    G1 = expm(A * (Ts - theta)) @ I1
    numz = np.append(numer(G0)[1:], 0.0) + numer(G1)
    return Tf.make(numz, cp, D + 1)


def lsim(tf: Tf, u) -> np.ndarray:
    """Discrete simulation from rest (lsim of a discrete tf)."""
    from scipy.signal import lfilter

    b, a = tf.impulse_form()
    return lfilter(b, a, np.asarray(u, dtype=float))


def descomp(P):
    """descompMPC.m:19-43 on an my x nin list of Tf: (B, A, d) with the B(1)~=0 -> d-1, [0 B]
    adjustment and the zero-dcgain -> max row delay rule."""
    my, nin = len(P), len(P[0])
    B = [[np.asarray(P[i][j].num, dtype=float) for j in range(nin)] for i in range(my)]
    A = [[np.asarray(P[i][j].den, dtype=float) for j in range(nin)] for i in range(my)]
    d = np.array([[P[i][j].delay for j in range(nin)] for i in range(my)], dtype=int)
    for i in range(my):
        for j in range(nin):
            if B[i][j][0] != 0.0:
                d[i, j] -= 1
                B[i][j] = np.concatenate([[0.0], B[i][j]])
            if P[i][j].dcgain == 0.0:
                d[i, j] = d[i].max()
    return B, A, d


def _mround4(x):
    return np.sign(x) * np.floor(np.abs(x) * 1e4 + 0.5) / 1e4


def _poly_matlab(r):
    c = np.zeros(len(r) + 1, dtype=complex)
    c[0] = 1.0
    for j, e in enumerate(r):
        c[1: j + 2] = c[1: j + 2] - e * c[: j + 1]
    return c.real


def carima(Bn, An, exact: bool = True):
    """CARIMA numerators/denominators per output row (BA_MIMO.m:20-71).

    exact=True: least common multiple built from the DISTINCT denominator polynomials of the row
    (toolbox-equivalent: the model equals the plant).  exact=False: BA_MIMO verbatim, LCM poles
    = unique(round(roots(.),4)) — a ~1e-5 model change the reference's GPC makes.
    Returns (B, A, na, nb)."""
    my, nin = len(An), len(An[0])
    Bs = [[(b[1:] if b[0] == 0.0 else b) for b in row] for row in Bn]
    A, B = [], [[None] * nin for _ in range(my)]
    for i in range(my):
        if exact:
            uniq = []
            for j in range(nin):
                if not any(np.array_equal(An[i][j], u) for u in uniq):
                    uniq.append(np.asarray(An[i][j], dtype=float))
            Ai = np.ones(1)
            for u in uniq:
                Ai = np.convolve(Ai, u)
            A.append(Ai)
            for j in range(nin):
                b = Bs[i][j]
                for u in uniq:
                    if not np.array_equal(An[i][j], u):
                        b = np.convolve(b, u)
                B[i][j] = b
        else:
            prod = np.ones(1)
            for j in range(nin):
                prod = np.convolve(prod, An[i][j])
            Ai = prod if my == 1 else _poly_matlab(np.unique(_mround4(np.roots(prod))))
            A.append(Ai)
            for j in range(nin):
                rA = list(_mround4(np.roots(Ai)))
                rAn = list(_mround4(np.roots(An[i][j])))
                kk = 0
                while kk < len(rA):
                    for x in rAn:
                        if kk < len(rA) and rA[kk] == x:
                            v = rA[kk]
                            rA = [q for q in rA if q != v]
                    kk += 1
                B[i][j] = np.convolve(Bs[i][j], _poly_matlab(rA) if rA else np.ones(1))
    na = np.array([a.size - 1 for a in A])
    nb = np.array([[B[i][j].size - 1 for j in range(nin)] for i in range(my)])
    return B, A, na, nb
