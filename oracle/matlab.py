"""Restated MATLAB builtins used by the reference's hot path (oracle; test infrastructure only).

Every function names the reference call sites it stands in for.  Discrete transfer functions
are represented as :class:`DTF` (one SISO entry: z-domain ``num``/``den`` exactly as ``tfdata``
returns them, plus the integer ``iodelay``), which is the representation the reference's
``descompMPC.m:19`` reads.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import scipy.linalg as sla


@dataclass
class DTF:
    """One SISO discrete transfer function ``z^-iodelay * num(z)/den(z)`` (tfdata 'v' form).

    ``num`` and ``den`` are coefficient lists in descending powers of z with ``len(num) ==
    len(den)`` (MATLAB pads the numerator with leading zeros), ``den[0] == 1``.
    """

    num: np.ndarray
    den: np.ndarray
    iodelay: int = 0

    def __post_init__(self):
        self.num = np.asarray(self.num, dtype=float).ravel()
        self.den = np.asarray(self.den, dtype=float).ravel()
        n = max(len(self.num), len(self.den))
        self.num = np.concatenate([np.zeros(n - len(self.num)), self.num])
        self.den = np.concatenate([np.zeros(n - len(self.den)), self.den])

    def dcgain(self) -> float:
        s = self.den.sum()
        return float(self.num.sum() / s) if s != 0 else float("inf")

    def zinv_form(self):
        """Return (b, a) in powers of z^-1 with the delay folded into b's leading zeros:
        y(t) = sum_l b[l] u(t-l) - sum_{l>=1} a[l] y(t-l)."""
        # num(z)/den(z) with equal degree n: divide by z^n -> coefficients are already z^-1 powers
        b = np.concatenate([np.zeros(self.iodelay), self.num]) / self.den[0]
        a = self.den / self.den[0]
        return b, a

    def scaled(self, k: float) -> "DTF":
        return DTF(self.num * k, self.den.copy(), self.iodelay)


# ---------------------------------------------------------------------------------------------
# round(x, 4) — MATLAB rounds half away from zero (used at BA_MIMO.m:38,48-49)
# ---------------------------------------------------------------------------------------------
def mround(x, n: int = 4):
    x = np.asarray(x)
    s = 10.0 ** n
    if np.iscomplexobj(x):
        return mround(x.real, n) + 1j * mround(x.imag, n)
    return np.sign(x) * np.floor(np.abs(x) * s + 0.5) / s


def conv(a, b):
    """MATLAB conv (full) — DTC-GPC/diophantine.m:35, deltaUFree.m:35, BA_MIMO.m:32,60."""
    return np.convolve(np.asarray(a, dtype=float), np.asarray(b, dtype=float))


def roots(c):
    """MATLAB roots (roots.m): strip leading zeros, turn trailing zeros into roots at the
    origin, and take the eigenvalues of the companion matrix of what is left.  Stands in for
    BA_MIMO.m:38,48-49 and filtro_siso.m:26 (pole)."""
    c = np.asarray(c, dtype=float).ravel()
    nz = np.nonzero(c)[0]
    if nz.size == 0:
        return np.zeros(0)
    n_zero = len(c) - 1 - nz[-1]
    c = c[nz[0]: nz[-1] + 1]
    n = len(c) - 1
    if n < 1:
        r = np.zeros(0)
    else:
        a = np.diag(np.ones(n - 1), -1)
        a[0, :] = -c[1:] / c[0]
        r = np.linalg.eigvals(a)
        if np.all(np.abs(r.imag) == 0):
            r = r.real
    return np.concatenate([r, np.zeros(n_zero)])


def poly(r):
    """MATLAB poly from a root vector, same accumulation order as poly.m:
    c(2:(j+1)) = c(2:(j+1)) - e(j).*c(1:j).  Real output when roots come in conjugate pairs."""
    e = np.asarray(r).ravel()
    n = len(e)
    c = np.zeros(n + 1, dtype=complex)
    c[0] = 1.0
    for j in range(n):
        c[1:j + 2] = c[1:j + 2] - e[j] * c[0:j + 1]
    if np.all(np.abs(c.imag) <= 0) or np.allclose(np.sort_complex(e), np.sort_complex(np.conj(e))):
        return c.real.copy()
    return c


def de2bi(x: int, n: int):
    """Communications-toolbox de2bi, least-significant bit first (MPCTuning.m:285, VNS2.m:210)."""
    return [(int(x) >> k) & 1 for k in range(n)]


# ---------------------------------------------------------------------------------------------
# c2d(sys, Ts, 'zoh') for a continuous SISO tf with an input/output delay
# (Shell3x3.m:65, Shell7x5.m:95, WoodBerry.m:62, DTC_GPC_WW.m:41, Shell3x3.m:77 Pref)
# ---------------------------------------------------------------------------------------------
def _tf2ss(num, den):
    """Controllable canonical realisation of a strictly proper num/den (descending powers)."""
    num = np.asarray(num, dtype=float).ravel()
    den = np.asarray(den, dtype=float).ravel()
    den = np.trim_zeros(den, "f")
    num = np.trim_zeros(num, "f") if np.any(num) else np.zeros(1)
    n = len(den) - 1
    a0 = den[0]
    den = den / a0
    num = num / a0
    if len(num) > n:
        raise ValueError("c2d restatement handles strictly proper continuous systems only")
    num = np.concatenate([np.zeros(n - len(num)), num])
    A = np.zeros((n, n))
    A[0, :] = -den[1:]
    if n > 1:
        A[1:, :-1] = np.eye(n - 1)
    B = np.zeros((n, 1))
    B[0, 0] = 1.0
    C = num.reshape(1, n)
    return A, B, C


def _zoh_int(A, B, T):
    """(e^{A T}, int_0^T e^{A s} ds B) via the augmented exponential."""
    n = A.shape[0]
    M = np.zeros((n + 1, n + 1))
    M[:n, :n] = A
    M[:n, n:] = B
    E = sla.expm(M * T)
    return E[:n, :n], E[:n, n:]


def c2d_zoh(num, den, Ts: float, delay: float = 0.0) -> DTF:
    """Exact ZOH discretisation of ``num(s)/den(s) * exp(-delay*s)``.

    With delay = D*Ts + theta (0 <= theta < Ts), the input seen by the plant over sample n is
    u[n-D-1] on [0, theta) and u[n-D] on [theta, Ts).  Hence
        x[n+1] = Phi x[n] + G0 u[n-D] + G1 u[n-D-1],
        G0 = int_0^{Ts-theta} e^{As}ds B,  G1 = e^{A(Ts-theta)} int_0^{theta} e^{As}ds B.
    MATLAB reports theta == 0 as iodelay D with num [0 C G0 ...], and theta > 0 as
    iodelay D+1 with a numerator of full degree (the fixtures' iodelay [7 7 7;5 4 4;5 6 0]).
    """
    A, B, C = _tf2ss(num, den)
    n = A.shape[0]
    D = int(np.floor(delay / Ts + 1e-12))
    theta = delay - D * Ts
    if abs(theta) < 1e-12 * max(1.0, Ts):
        theta = 0.0
    _, G0 = _zoh_int(A, B, Ts - theta)
    Phi = sla.expm(A * Ts)
    if theta > 0:
        _, I1 = _zoh_int(A, B, theta)
        G1 = sla.expm(A * (Ts - theta)) @ I1
    else:
        G1 = np.zeros_like(G0)
    cp = np.real(np.poly(Phi)) if n > 0 else np.ones(1)

    def _num_of(Gam):
        # C (zI-Phi)^-1 Gam = [det(zI - Phi + Gam C) - det(zI - Phi)] / det(zI - Phi)
        return np.real(np.poly(Phi - Gam @ C)) - cp

    N0 = _num_of(G0)  # length n+1, leading coefficient 0
    if theta > 0:
        N1 = _num_of(G1)
        # z^{-(D+1)} [z N0(z) + N1(z)] / cp(z): numerator of degree n
        numz = N0[1:] + 0.0
        numz = np.concatenate([numz, [0.0]]) + N1
        return DTF(numz, cp, D + 1)
    return DTF(N0, cp, D)


def c2d_fopdt(K: float, tau: float, Ts: float, delay: float) -> DTF:
    """Closed form of :func:`c2d_zoh` for K/(tau s + 1) e^{-delay s} (every Shell / WoodBerry
    entry).  Used as an independent check of the general path."""
    a = np.exp(-Ts / tau)
    D = int(np.floor(delay / Ts + 1e-12))
    theta = delay - D * Ts
    if abs(theta) < 1e-12:
        return DTF([0.0, K * (1 - a)], [1.0, -a], D)
    m = np.exp(-(Ts - theta) / tau)
    return DTF([K * (1 - m), K * (m - a)], [1.0, -a], D + 1)


# ---------------------------------------------------------------------------------------------
# Discrete simulation: step / lsim (MatG.m:51, OptimalPredictor2.m:28-37, closedloop_toolbox.m:100)
# ---------------------------------------------------------------------------------------------
def lsim_dtf(sys: DTF, u) -> np.ndarray:
    """Full-history discrete simulation from rest (lsim of a discrete tf): direct form
    y(t) = sum_l b[l] u(t-l) - sum_{l>=1} a[l] y(t-l)."""
    b, a = sys.zinv_form()
    u = np.asarray(u, dtype=float).ravel()
    T = len(u)
    y = np.zeros(T)
    for t in range(T):
        acc = 0.0
        for l in range(len(b)):
            if t - l >= 0:
                acc += b[l] * u[t - l]
        for l in range(1, len(a)):
            if t - l >= 0:
                acc -= a[l] * y[t - l]
        y[t] = acc
    return y


def step_dtf(sys: DTF, nsamples: int) -> np.ndarray:
    """step(sys, (nsamples-1)*Ts): samples s(0..nsamples-1) of the unit-step response."""
    return lsim_dtf(sys, np.ones(nsamples))


def lsim_mimo(P, U) -> np.ndarray:
    """lsim of an my x nin matrix of DTF entries; U is nin x T; returns my x T."""
    U = np.atleast_2d(np.asarray(U, dtype=float))
    my = len(P)
    T = U.shape[1]
    Y = np.zeros((my, T))
    for i in range(my):
        for j in range(len(P[i])):
            if np.any(P[i][j].num):
                Y[i] += lsim_dtf(P[i][j], U[j])
    return Y


def lsim_continuous_fopdt_diag(K, tau, delay, Ts, U):
    """lsim of a diagonal first-order-plus-delay reference model with ZOH (Shell3x3.m:99)."""
    U = np.atleast_2d(np.asarray(U, dtype=float))
    Y = np.zeros_like(U)
    for i in range(U.shape[0]):
        Y[i] = lsim_dtf(c2d_fopdt(K[i], tau[i], Ts, delay[i]), U[i])
    return Y
