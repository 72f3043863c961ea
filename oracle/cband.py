"""ctypes wrapper of oracle/cband.c (the C restatement of oracle/toolbox_band.py) — test
infrastructure only: it scores config-3 (Shell 7x5 band-mode) grids and replays device
trajectories step by step.  Its tables are built HERE from the oracle's own BandScenario
(``DTF.zinv_form`` of every plant entry), never from the product library."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libcband.so")

_ip = C.POINTER(C.c_int)
_dp = C.POINTER(C.c_double)


class CbScen(C.Structure):
    _fields_ = [("my", C.c_int), ("nu", C.c_int), ("nd", C.c_int), ("nit", C.c_int),
                ("wsq", C.c_int), ("ink0", C.c_int), ("maxb", C.c_int), ("maxa", C.c_int),
                ("nb", _ip), ("na", _ip), ("b", _dp), ("a", _dp), ("bnd", _dp),
                ("ymin", _dp), ("ymax", _dp), ("ecrmin", _dp), ("ecrmax", _dp), ("sy", _dp),
                ("su", _dp), ("rho", C.c_double), ("yref", _dp), ("qp_warm", C.c_int)]


def _load():
    if not os.path.exists(_SO):
        subprocess.run(["make", "-C", _HERE, "-s", "libcband.so"], check=True)
    lib = C.CDLL(_SO)
    lib.cband_eval.restype = C.c_int
    lib.cband_eval.argtypes = [C.POINTER(CbScen), C.c_int64] + [C.c_void_p] * 4 + [
        C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 10
    lib.cband_replay.restype = C.c_int
    lib.cband_replay.argtypes = [C.POINTER(CbScen), C.c_int64] + [C.c_void_p] * 7 + [
        C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.cband_replay_gap.restype = C.c_int
    lib.cband_replay_gap.argtypes = [C.POINTER(CbScen), C.c_int64] + [C.c_void_p] * 7 + [
        C.c_int, C.c_int] + [C.c_void_p] * 4
    return lib


class CBand:
    """C port of ``toolbox_band.closedloop_band`` / ``replay_moves`` for one BandScenario."""

    def __init__(self, sc, nit, yref, ink=10, warm=False):
        """warm: the second, equally valid QP path (each step's dual method warm-started from the
        previous step's final active set; cband.c cb_scen.qp_warm) -- the C-vs-C floor."""
        self.lib = _load()
        my, nu, nin = sc.my, sc.nu, sc.nin
        ba = [sc.plant[i][j].zinv_form() for i in range(my) for j in range(nin)]
        for e, (b, a) in enumerate(ba):
            if e % nin < nu and len(b) and b[0] != 0.0:
                raise ValueError("MV feed-through: the toolbox needs a strictly proper MV channel")
        nb = np.array([len(b) for b, _ in ba], np.int32)
        na = np.array([len(a) for _, a in ba], np.int32)
        B = np.zeros((len(ba), max(1, nb.max())))
        A = np.zeros((len(ba), na.max()))
        for e, (b, a) in enumerate(ba):
            B[e, :len(b)] = b
            A[e, :len(a)] = a
        self.t = dict(nb=nb, na=na, b=B, a=A,
                      bnd=np.ascontiguousarray(np.stack([sc.du_min, sc.du_max, sc.u_min, sc.u_max]), float),
                      ymin=np.ascontiguousarray(sc.y_min, float), ymax=np.ascontiguousarray(sc.y_max, float),
                      ecrmin=np.ascontiguousarray(sc.ecr_min, float), ecrmax=np.ascontiguousarray(sc.ecr_max, float),
                      sy=np.ascontiguousarray(sc.sy, float), su=np.ascontiguousarray(sc.su, float),
                      yref=np.ascontiguousarray(np.asarray(yref, float).reshape(my, nit)))
        s = CbScen()
        s.my, s.nu, s.nd, s.nit = my, nu, nin - nu, int(nit)
        s.wsq, s.ink0 = int(sc.weights_squared), int(ink) - 1
        s.maxb, s.maxa = B.shape[1], A.shape[1]
        for k in ("nb", "na"):
            setattr(s, k, self.t[k].ctypes.data_as(_ip))
        for k in ("b", "a", "bnd", "ymin", "ymax", "ecrmin", "ecrmax", "sy", "su", "yref"):
            setattr(s, k, self.t[k].ctypes.data_as(_dp))
        s.rho = float(sc.rho)
        s.qp_warm = int(bool(warm))
        self.s = s
        self.my, self.nu, self.nd, self.nit = my, nu, nin - nu, int(nit)

    def _cands(self, N2, Nu, delta, lam):
        N2 = np.ascontiguousarray(np.atleast_1d(N2), np.int32)
        n = N2.size
        Nu = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(Nu), (n,)), np.int32)
        delta = np.ascontiguousarray(np.asarray(delta, float).reshape(n, self.my))
        lam = np.ascontiguousarray(np.asarray(lam, float).reshape(n, self.nu))
        return N2, Nu, delta, lam

    def eval(self, N2, Nu, delta, lam, refs, v, open_loop=False, want_traj=False, threads=0):
        """Score candidates x reference sets: refs (nref, my, nit), v (nref, nd, nit)."""
        N2, Nu, delta, lam = self._cands(N2, Nu, delta, lam)
        my, nu, nit = self.my, self.nu, self.nit
        refs = np.ascontiguousarray(np.asarray(refs, float).reshape(-1, my, nit))
        nref = refs.shape[0]
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(v, float).reshape(-1, self.nd, nit),
                                                 (nref, self.nd, nit)))
        S = N2.size * nref
        out = dict(J1=np.zeros((S, my)), j21=np.zeros((S, my)), j22=np.zeros((S, my)),
                   Jnu=np.zeros((S, nu)), status=np.zeros(S, np.int32), qp_iters=np.zeros(S, np.int64))
        tr = [None] * 4
        if want_traj:
            for k, d in (("y", my), ("u", nu), ("ys", my), ("uopt", nu)):
                out[k] = np.zeros((S, d, nit))
            tr = [out[k].ctypes.data for k in ("y", "u", "ys", "uopt")]
        self.lib.cband_eval(C.byref(self.s), N2.size, N2.ctypes.data, Nu.ctypes.data, delta.ctypes.data,
                            lam.ctypes.data, nref, refs.ctypes.data, v.ctypes.data, int(open_loop), int(threads),
                            out["J1"].ctypes.data, out["j21"].ctypes.data, out["j22"].ctypes.data,
                            out["Jnu"].ctypes.data, out["status"].ctypes.data, out["qp_iters"].ctypes.data, *tr)
        return out

    def replay(self, N2, Nu, delta, lam, r, v, U, T=None, threads=0):
        """Oracle first moves (C, nu, T) at the states the applied trajectories U (C, nu, nit)
        reached, and the applied moves; statuses."""
        N2, Nu, delta, lam = self._cands(N2, Nu, delta, lam)
        nit = self.nit
        T = nit if T is None else int(T)
        U = np.ascontiguousarray(np.asarray(U, float).reshape(N2.size, self.nu, nit))
        r = np.ascontiguousarray(np.asarray(r, float).reshape(self.my, nit))
        v = np.ascontiguousarray(np.asarray(v, float).reshape(self.nd, nit))
        du_o = np.zeros((N2.size, self.nu, T))
        st = np.zeros(N2.size, np.int32)
        rc = self.lib.cband_replay(C.byref(self.s), N2.size, N2.ctypes.data, Nu.ctypes.data, delta.ctypes.data,
                                   lam.ctypes.data, r.ctypes.data, v.ctypes.data, U.ctypes.data, T, int(threads),
                                   du_o.ctypes.data, st.ctypes.data)
        if rc != 0:
            raise ValueError("cband_replay: bad T")
        du_a = np.diff(np.concatenate([np.zeros((N2.size, self.nu, 1)), U], axis=2), axis=2)[:, :, :T]
        return du_o, du_a, st

    def replay_gap(self, N2, Nu, delta, lam, r, v, U, T=None, threads=0):
        """replay() plus toolbox_band.pinned_gap at every step: (du_o (C, nu, T), du_a, J_free
        (C, T), J_pinned (C, T), status).  J_pinned is NaN where the pinned QP failed."""
        N2, Nu, delta, lam = self._cands(N2, Nu, delta, lam)
        nit = self.nit
        T = nit if T is None else int(T)
        U = np.ascontiguousarray(np.asarray(U, float).reshape(N2.size, self.nu, nit))
        r = np.ascontiguousarray(np.asarray(r, float).reshape(self.my, nit))
        v = np.ascontiguousarray(np.asarray(v, float).reshape(self.nd, nit))
        du_o = np.zeros((N2.size, self.nu, T))
        J0 = np.zeros((N2.size, T))
        J1 = np.zeros((N2.size, T))
        st = np.zeros(N2.size, np.int32)
        rc = self.lib.cband_replay_gap(C.byref(self.s), N2.size, N2.ctypes.data, Nu.ctypes.data, delta.ctypes.data,
                                       lam.ctypes.data, r.ctypes.data, v.ctypes.data, U.ctypes.data, T, int(threads),
                                       du_o.ctypes.data, J0.ctypes.data, J1.ctypes.data, st.ctypes.data)
        if rc != 0:
            raise ValueError("cband_replay_gap: bad T")
        du_a = np.diff(np.concatenate([np.zeros((N2.size, self.nu, 1)), U], axis=2), axis=2)[:, :, :T]
        return du_o, du_a, J0, J1, st
