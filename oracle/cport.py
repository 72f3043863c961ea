"""ctypes wrapper of oracle/cgpc.c (the C restatement) — test infrastructure / CPU baseline only.

The tables handed to C are built HERE from the numpy oracle's own restatements (step responses
via matlab.step_dtf, Diophantine via dtcgpc.diophantine, past controls via dtcgpc.delta_u_free),
never from the product library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .dtcgpc import delta_u_free, diophantine
from .matlab import step_dtf

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libcgpc.so")

_ip = C.POINTER(C.c_int)
_dp = C.POINTER(C.c_double)


class CgScen(C.Structure):
    _fields_ = [("my", C.c_int), ("nu", C.c_int), ("nin", C.c_int), ("nit", C.c_int),
                ("n2max", C.c_int), ("tlen", C.c_int), ("nx", C.c_int), ("wsq", C.c_int),
                ("ink0", C.c_int),
                ("n1", _ip), ("step", _dp), ("phi", _dp), ("yoff", _ip), ("nyhi", _ip),
                ("upoff", _ip), ("dum", _ip),
                ("ne", C.c_int), ("pl_maxb", C.c_int), ("pl_maxa", C.c_int),
                ("pl_nb", _ip), ("pl_na", _ip), ("pl_b", _dp), ("pl_a", _dp),
                ("bnd", _dp), ("yref", _dp)]


def build():
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)


def _load():
    if not os.path.exists(_SO):
        build()
    lib = C.CDLL(_SO)
    lib.cgpc_eval.restype = C.c_int
    lib.cgpc_eval.argtypes = [C.POINTER(CgScen), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 10
    return lib


def oracle_tables(sc, n2max: int, nit: int, yref, ink=10):
    """Candidate-independent tables of the oracle Scenario ``sc`` (toolbox_gpc.Scenario)."""
    my, nu = sc.my, sc.nu
    dwin = np.zeros(my, dtype=int) if sc.window == "toolbox" else sc.dmin.astype(int)
    n1 = (dwin + 1).astype(np.int32)
    tlen = int(n1.max()) + n2max
    step = np.zeros((my, nu, tlen))
    for i in range(my):
        for n in range(nu):
            step[i, n] = step_dtf(sc.model[i][n], tlen)
    nyhi = (sc.na + 1).astype(np.int32)
    yoff = np.concatenate([[0], np.cumsum(nyhi)[:-1]]).astype(np.int32)
    nyh = int(nyhi.sum())
    En, F = [], []
    for i in range(my):
        Ei, Fi = diophantine(sc.A[i], n2max, int(dwin[i]))
        En.append(Ei)
        F.append(Fi)
    uG = delta_u_free([row[:nu] for row in sc.B], En, [n2max] * my, sc.dp[:, :nu])
    dum = np.array([max(uG[m][n].shape[1] for m in range(my)) for n in range(nu)], dtype=np.int32)
    upoff = (nyh + np.concatenate([[0], np.cumsum(dum)[:-1]])).astype(np.int32)
    nx = nyh + int(dum.sum())
    phi = np.zeros((my * n2max, nx))
    for i in range(my):
        phi[i * n2max:(i + 1) * n2max, yoff[i]:yoff[i] + nyhi[i]] = F[i]
        for n in range(nu):
            w = uG[i][n].shape[1]
            phi[i * n2max:(i + 1) * n2max, upoff[n]:upoff[n] + w] = uG[i][n]
    ne = my * sc.nin
    ba = [sc.plant[i][j].zinv_form() for i in range(my) for j in range(sc.nin)]
    pl_nb = np.array([len(b) for b, _ in ba], dtype=np.int32)
    pl_na = np.array([len(a) for _, a in ba], dtype=np.int32)
    mb, ma = int(pl_nb.max()), int(pl_na.max())
    pl_b = np.zeros((ne, mb))
    pl_a = np.zeros((ne, ma))
    for e, (b, a) in enumerate(ba):
        pl_b[e, :len(b)] = b
        pl_a[e, :len(a)] = a
    bnd = np.stack([sc.du_min, sc.du_max, sc.u_min, sc.u_max]).astype(float)
    return dict(my=my, nu=nu, nin=sc.nin, nit=nit, n2max=n2max, tlen=tlen, nx=nx,
                wsq=int(sc.weights_squared), ink0=ink - 1, n1=n1, step=step, phi=phi, yoff=yoff,
                nyhi=nyhi, upoff=upoff, dum=dum, ne=ne, pl_maxb=mb, pl_maxa=ma, pl_nb=pl_nb,
                pl_na=pl_na, pl_b=pl_b, pl_a=pl_a, bnd=bnd, yref=np.ascontiguousarray(yref, dtype=float))


class CPort:
    def __init__(self, sc, n2max, nit, yref, ink=10):
        self.lib = _load()
        t = oracle_tables(sc, n2max, nit, yref, ink)
        self.t = {k: (np.ascontiguousarray(v) if isinstance(v, np.ndarray) else v) for k, v in t.items()}
        s = CgScen()
        for k in ("my", "nu", "nin", "nit", "n2max", "tlen", "nx", "wsq", "ink0", "ne", "pl_maxb", "pl_maxa"):
            setattr(s, k, int(self.t[k]))
        for k in ("n1", "yoff", "nyhi", "upoff", "dum", "pl_nb", "pl_na"):
            self.t[k] = np.ascontiguousarray(self.t[k], dtype=np.int32)
            setattr(s, k, self.t[k].ctypes.data_as(_ip))
        for k in ("step", "phi", "pl_b", "pl_a", "bnd", "yref"):
            self.t[k] = np.ascontiguousarray(self.t[k], dtype=float)
            setattr(s, k, self.t[k].ctypes.data_as(_dp))
        self.s = s

    def eval(self, N2, Nu, delta, lam, refs, open_loop=False, want_traj=False, threads=0):
        my, nu, nit = self.s.my, self.s.nu, self.s.nit
        N2 = np.ascontiguousarray(np.atleast_1d(N2), dtype=np.int32)
        Cn = N2.size
        Nu = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(Nu), (Cn,)), dtype=np.int32)
        delta = np.ascontiguousarray(np.asarray(delta, float).reshape(Cn, my))
        lam = np.ascontiguousarray(np.asarray(lam, float).reshape(Cn, nu))
        refs = np.ascontiguousarray(np.asarray(refs, float).reshape(-1, my, nit))
        nref = refs.shape[0]
        S = Cn * nref
        out = dict(J1=np.zeros((S, my)), j21=np.zeros((S, my)), j22=np.zeros((S, my)),
                   Jnu=np.zeros((S, nu)), status=np.zeros(S, dtype=np.int32),
                   qp_iters=np.zeros(S, dtype=np.int64))
        tr = [None] * 4
        if want_traj:
            out["y"] = np.zeros((S, my, nit))
            out["u"] = np.zeros((S, nu, nit))
            out["ys"] = np.zeros((S, my, nit))
            out["uopt"] = np.zeros((S, nu, nit))
            tr = [out[k].ctypes.data for k in ("y", "u", "ys", "uopt")]
        self.lib.cgpc_eval(C.byref(self.s), Cn, N2.ctypes.data, Nu.ctypes.data, delta.ctypes.data,
                           lam.ctypes.data, nref, refs.ctypes.data, int(open_loop), int(threads),
                           out["J1"].ctypes.data, out["j21"].ctypes.data, out["j22"].ctypes.data,
                           out["Jnu"].ctypes.data, out["status"].ctypes.data, out["qp_iters"].ctypes.data,
                           *tr)
        return out
