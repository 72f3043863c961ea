"""Python host mirror of the reference's closed-loop seam, over the libmpct C ABI.

  Scenario            mpct_scenario_create: plant/model/CARIMA tables + bounds + Yref
  eval_batch          mpct_eval_batch (host arrays): C candidates x nref reference sets
  eval_batch_device   mpct_eval_batch_device (torch CUDA tensors, enqueued on a stream)
  closedloop_toolbox  drop-in for closedloop_toolbox.m:1 (one candidate, full trajectories)

No CPU fallback: every numerical result comes from the HIP kernel.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .lti import Tf, carima, descomp


def _dp(a):
    return a.ctypes.data_as(_lib.c_double_p)


def _ip(a):
    return a.ctypes.data_as(_lib.c_int32_p)


class MpctError(RuntimeError):
    pass


class Scenario:
    """Candidate-independent description of one tuning problem (MPCTuning's Par minus N/Nu/
    delta/lambda).  ``plant``/``model`` are my x (nu+nd) lists of :class:`Tf` (scaled, discrete:
    MPCTuning.m:162 Pze = L*Pz*R).  ``window``: 'toolbox' predicts t+1..t+N2 (PredictionHorizon
    semantics, closedloop_toolbox.m:38), 'gpc' predicts t+dmin+1..t+dmin+N2 (MatG.m / DTC_GPC_WW).
    ``exact_carima``: exact LCM (toolbox-equivalent) vs BA_MIMO's rounded roots.
    ``bands``: the toolbox MPC with measured disturbances and soft output bands (Shell7x5.m,
    WoodBerry.m; ABI mdband): dict(y_min, y_max, ecr_min, ecr_max, y_scale=None, u_scale=None,
    rho=1e4) of OV Min/Max, MinECR/MaxECR, ScaleFactors and Weights.ECR.  Scenarios with measured
    disturbances (nd > 0) always use that kernel (unbounded outputs when bands is None).
    ``host_carima``: False passes no CARIMA tables and lets the library derive them from the model
    (exact LCM, what the MATLAB MEX host does; toolbox window only)."""

    def __init__(self, plant, model, nu, du_min, du_max, u_min, u_max, yref, n2_max, nu_max,
                 Ts=1.0, window="toolbox", weights_squared=True, exact_carima=True, vns_ink=10,
                 dtc=False, filters=None, dist=None, plant_variants=None, bands=None, host_carima=True):
        self.lib = _lib.load()
        self.plant, self.model = plant, model
        self.my, self.nin = len(model), len(model[0])
        self.nu = int(nu)
        self.nd = self.nin - self.nu
        self.yref = np.ascontiguousarray(np.asarray(yref, dtype=float).reshape(self.my, -1))
        self.nit = self.yref.shape[1]
        self.n2_max, self.nu_max, self.Ts = int(n2_max), int(nu_max), float(Ts)
        self.window, self.weights_squared, self.vns_ink = window, bool(weights_squared), int(vns_ink)
        Bn, An, dp = descomp(model)
        B, A, na, nb = carima(Bn, An, exact=exact_carima)
        self.dp, self.na, self.nb = dp, na, nb
        self.dmin = dp[:, : self.nu].min(axis=1)
        n1 = np.ones(self.my, dtype=np.int32) if window == "toolbox" else (self.dmin + 1).astype(np.int32)
        # DTC-GPC (DTC_GPC_WW.m): GPC window, deltaUFree on the delays net of dmin (dnz)
        self.dtc = bool(dtc)
        self.nq = len(dist[0]) if dist else 0
        self.dist, self.filters = dist, filters
        if self.dtc and window != "gpc":
            raise ValueError("DTC mode uses the GPC window (MatG/diophantine N1 = dmin+1)")
        dp_desc = (dp - self.dmin[:, None]) if self.dtc else dp
        keep = []  # keep every buffer alive for the descriptor's lifetime

        def dtf_array(P):
            arr = (_lib.MpctDtf * (self.my * self.nin))()
            for i in range(self.my):
                for j in range(self.nin):
                    t = P[i][j]
                    num = np.ascontiguousarray(t.num, dtype=float)
                    den = np.ascontiguousarray(t.den, dtype=float)
                    keep.extend([num, den])
                    arr[i * self.nin + j] = _lib.MpctDtf(len(num), _dp(num), _dp(den), int(t.delay))
            keep.append(arr)
            return arr

        A_cat = np.ascontiguousarray(np.concatenate([np.asarray(a, dtype=float) / a[0] for a in A]))
        B_cat = np.ascontiguousarray(np.concatenate(
            [np.asarray(B[i][j], dtype=float) / A[i][0] for i in range(self.my) for j in range(self.nin)]))
        na32 = np.ascontiguousarray(na, dtype=np.int32)
        nb32 = np.ascontiguousarray(nb.ravel(), dtype=np.int32)
        dp32 = np.ascontiguousarray(dp_desc.ravel(), dtype=np.int32)
        bnds = [np.ascontiguousarray(np.broadcast_to(np.asarray(b, dtype=float), (self.nu,)))
                for b in (du_min, du_max, u_min, u_max)]
        self.bounds = bnds
        keep += [A_cat, B_cat, na32, nb32, dp32, n1, self.yref] + bnds
        d = _lib.MpctScenarioDesc()
        d.abi_version = _lib.ABI_VERSION
        d.my, d.nu, d.nd, d.nit = self.my, self.nu, self.nd, self.nit
        d.n2_max, d.nu_max = self.n2_max, self.nu_max
        d.weights_squared = int(self.weights_squared)
        d.vns_ink = self.vns_ink
        d.n1 = _ip(n1)
        d.plant = dtf_array(plant)
        d.model = dtf_array(model)
        if host_carima or self.dtc or not exact_carima:
            d.na, d.carima_A, d.nb, d.carima_B, d.dp = _ip(na32), _dp(A_cat), _ip(nb32), _dp(B_cat), _ip(dp32)
        d.du_min, d.du_max, d.u_min, d.u_max = (_dp(b) for b in bnds)
        d.yref = _dp(self.yref)
        d.dtc = int(self.dtc)
        d.nq = self.nq
        if filters is not None:
            farr = (_lib.MpctDtf * self.my)()
            for i, t in enumerate(filters):
                num = np.ascontiguousarray(t.num, dtype=float)
                den = np.ascontiguousarray(t.den, dtype=float)
                keep.extend([num, den])
                farr[i] = _lib.MpctDtf(len(num), _dp(num), _dp(den), int(t.delay))
            keep.append(farr)
            d.filter = farr
        if self.nq:
            darr = (_lib.MpctDtf * (self.my * self.nq))()
            for i in range(self.my):
                for j in range(self.nq):
                    t = dist[i][j]
                    num = np.ascontiguousarray(t.num, dtype=float)
                    den = np.ascontiguousarray(t.den, dtype=float)
                    keep.extend([num, den])
                    darr[i * self.nq + j] = _lib.MpctDtf(len(num), _dp(num), _dp(den), int(t.delay))
            keep.append(darr)
            d.dist = darr
        self.nplant = len(plant_variants) if plant_variants else 1
        if plant_variants and len(plant_variants) > 1:
            n = self.my * self.nin
            varr = (_lib.MpctDtf * (len(plant_variants) * n))()
            for v, Pv in enumerate(plant_variants):
                for i in range(self.my):
                    for j in range(self.nin):
                        t = Pv[i][j]
                        num = np.ascontiguousarray(t.num, dtype=float)
                        den = np.ascontiguousarray(t.den, dtype=float)
                        keep.extend([num, den])
                        varr[v * n + i * self.nin + j] = _lib.MpctDtf(len(num), _dp(num), _dp(den), int(t.delay))
            keep.append(varr)
            d.nplant = len(plant_variants)
            d.plant_var = varr
        self.mdband = bands is not None or self.nd > 0
        if self.mdband:
            if window != "toolbox" or self.dtc:
                raise ValueError("the MD / output-band kernel predicts over the toolbox window (no DTC)")
            b = dict(bands or {})
            inf = np.full(self.my, np.inf)

            def vec(key, default, n):
                v = b.get(key)
                return np.ascontiguousarray(np.broadcast_to(np.asarray(default if v is None else v, dtype=float), (n,)))

            self.bands = {k: vec(k, dflt, n) for k, dflt, n in (
                ("y_min", -inf, self.my), ("y_max", inf, self.my), ("ecr_min", 1.0, self.my),
                ("ecr_max", 1.0, self.my), ("y_scale", 1.0, self.my), ("u_scale", 1.0, self.nu))}
            self.rho = float(b.get("rho", 1e4))
            keep.extend(self.bands.values())
            d.mdband = 1
            d.y_min, d.y_max = _dp(self.bands["y_min"]), _dp(self.bands["y_max"])
            d.ecr_min, d.ecr_max = _dp(self.bands["ecr_min"]), _dp(self.bands["ecr_max"])
            d.y_scale, d.u_scale = _dp(self.bands["y_scale"]), _dp(self.bands["u_scale"])
            d.rho_ecr = self.rho
        h = C.c_void_p()
        rc = self.lib.mpct_scenario_create(C.byref(d), C.byref(h))
        if rc != 0:
            raise MpctError("mpct_scenario_create failed (%d): %s" % (rc, _lib.last_error()))
        self._h = h
        self._keep = keep
        self.n1 = n1

    @property
    def handle(self):
        return self._h

    def table(self, which: int) -> np.ndarray:
        n = self.lib.mpct_scenario_table(self._h, which, None, 0)
        if n < 0:
            raise MpctError(_lib.last_error())
        buf = np.zeros(n)
        self.lib.mpct_scenario_table(self._h, which, _dp(buf), n)
        return buf

    def dims(self) -> dict:
        """mpct_scenario_table(2): the ABI-6 dims table, every entry named."""
        k = ["my", "nu", "nd", "n2_max", "nu_max", "tlen", "nx", "nyh", "nup", "nit", "nq"]
        t = self.table(2)
        if t.size != len(k):
            raise MpctError("dims table has %d entries, expected %d" % (t.size, len(k)))
        return dict(zip(k, t.astype(int).tolist()))

    def lds_bytes(self, N2=None, Nu=None, costs_only=False) -> int:
        """LDS per workgroup with the open-loop leg / trajectories (or, costs_only, of the
        cost-only instance GAM_fun.m:81 calls launch)."""
        if costs_only:
            return int(self.lib.mpct_lds_bytes_opts(self._h, None, N2 or self.n2_max, Nu or self.nu_max))
        return int(self.lib.mpct_lds_bytes(self._h, N2 or self.n2_max, Nu or self.nu_max))

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mpct_scenario_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class EvalResult:
    J1: np.ndarray          # (S, my)
    j21: np.ndarray         # (S, my)
    j22: np.ndarray         # (S, my)
    Jnu: np.ndarray         # (S, nu)
    status: np.ndarray      # (S,)
    qp_iters: np.ndarray    # (S,)
    y: np.ndarray | None = None      # (S, my, nit)
    u: np.ndarray | None = None      # (S, nu, nit)
    ys: np.ndarray | None = None
    uopt: np.ndarray | None = None
    nref: int = 1
    extra: dict = field(default_factory=dict)


def _opts(open_loop, want_traj, device=-1, max_qp_iter=0, feas_tol=0.0):
    return _lib.MpctOpts(int(open_loop), int(want_traj), int(max_qp_iter), int(device), float(feas_tol))


def eval_batch(sc: Scenario, N2, Nu, delta, lam, refs, v=None, open_loop=False, want_traj=False,
               device=-1, max_qp_iter=0, feas_tol=0.0) -> EvalResult:
    """Score C candidates against nref reference sets (host arrays in, host arrays out)."""
    N2 = np.ascontiguousarray(np.atleast_1d(N2), dtype=np.int32)
    Cn = N2.size
    Nu = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(Nu), (Cn,)), dtype=np.int32)
    delta = np.ascontiguousarray(np.asarray(delta, dtype=float).reshape(Cn, sc.my))
    lam = np.ascontiguousarray(np.asarray(lam, dtype=float).reshape(Cn, sc.nu))
    refs = np.ascontiguousarray(np.asarray(refs, dtype=float).reshape(-1, sc.my, sc.nit))
    nref = refs.shape[0]
    S = Cn * nref
    vv = None
    if sc.nd + sc.nq:
        vv = np.ascontiguousarray(np.broadcast_to(np.asarray(v, dtype=float).reshape(-1, sc.nd + sc.nq, sc.nit),
                                                  (nref, sc.nd + sc.nq, sc.nit)))
    res = EvalResult(J1=np.zeros((S, sc.my)), j21=np.zeros((S, sc.my)), j22=np.zeros((S, sc.my)),
                     Jnu=np.zeros((S, sc.nu)), status=np.zeros(S, dtype=np.int32),
                     qp_iters=np.zeros(S, dtype=np.int64), nref=nref)
    r = _lib.MpctResult()
    r.J1, r.j21, r.j22, r.Jnu = _dp(res.J1), _dp(res.j21), _dp(res.j22), _dp(res.Jnu)
    r.status = _ip(res.status)
    r.qp_iters = res.qp_iters.ctypes.data_as(_lib.c_int64_p)
    if want_traj:
        res.y = np.zeros((S, sc.my, sc.nit))
        res.u = np.zeros((S, sc.nu, sc.nit))
        r.y, r.u = _dp(res.y), _dp(res.u)
        if open_loop:
            res.ys = np.zeros((S, sc.my, sc.nit))
            res.uopt = np.zeros((S, sc.nu, sc.nit))
            r.ys, r.uopt = _dp(res.ys), _dp(res.uopt)
    o = _opts(open_loop, want_traj, device, max_qp_iter, feas_tol)
    rc = sc.lib.mpct_eval_batch(sc.handle, Cn, N2.ctypes.data, Nu.ctypes.data, delta.ctypes.data,
                                lam.ctypes.data, nref, refs.ctypes.data,
                                vv.ctypes.data if vv is not None else None, C.byref(o), C.byref(r))
    if rc != 0:
        raise MpctError("mpct_eval_batch failed (%d): %s" % (rc, _lib.last_error()))
    return res


def eval_batch_device(sc: Scenario, N2, Nu, delta, lam, refs, out: dict, v=None, open_loop=False,
                      device=-1, stream=None):
    """Device-pointer entry: every argument is a CUDA (HIP) torch tensor already in HBM; results
    are written into the tensors of ``out`` (keys J1, j21, j22, Jnu, status, qp_iters).  The
    launch is enqueued on ``stream`` (torch stream; default: current) and not synchronised."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream()
    Cn = N2.numel()
    nref = refs.shape[0]
    r = _lib.MpctResult()

    def ptr(t, ty):
        return C.cast(C.c_void_p(t.data_ptr()), ty) if t is not None else None

    r.J1 = ptr(out.get("J1"), _lib.c_double_p)
    r.j21 = ptr(out.get("j21"), _lib.c_double_p)
    r.j22 = ptr(out.get("j22"), _lib.c_double_p)
    r.Jnu = ptr(out.get("Jnu"), _lib.c_double_p)
    r.status = ptr(out.get("status"), _lib.c_int32_p)
    r.qp_iters = ptr(out.get("qp_iters"), _lib.c_int64_p)
    o = _opts(open_loop, False, device)
    rc = sc.lib.mpct_eval_batch_device(
        sc.handle, Cn, C.c_void_p(N2.data_ptr()), C.c_void_p(Nu.data_ptr()), C.c_void_p(delta.data_ptr()),
        C.c_void_p(lam.data_ptr()), nref, C.c_void_p(refs.data_ptr()),
        C.c_void_p(v.data_ptr()) if v is not None else None, C.byref(o), C.byref(r),
        C.c_void_p(stream.cuda_stream))
    if rc != 0:
        raise MpctError("mpct_eval_batch_device failed (%d): %s" % (rc, _lib.last_error()))


def closedloop_toolbox(sc: Scenario, r, v, N, Nu, delta, lam, nit=None):
    """[y,u,t,ys,uopt] = closedloop_toolbox(mpc_toolbox,r,v,N,Nu,delta,lambda,nit)
    (closedloop_toolbox.m:1).  N, Nu may be vectors (max taken, :38-40).  Row signals out."""
    nit = sc.nit if nit is None else int(nit)
    if nit != sc.nit:
        raise ValueError("scenario was built for nit=%d" % sc.nit)
    N2 = int(np.max(N))
    nuh = int(np.max(Nu))
    res = eval_batch(sc, [N2], [nuh], np.reshape(delta, (1, -1)), np.reshape(lam, (1, -1)),
                     np.asarray(r, dtype=float)[None], v=None if v is None or np.size(v) == 0 else np.asarray(v)[None],
                     open_loop=True, want_traj=True)
    t = np.arange(nit) * sc.Ts
    return res.y[0], res.u[0], t, res.ys[0], res.uopt[0]


def kernel_instance(sc: Scenario, open_loop=False, want_traj=False) -> str:
    """mpct_kernel_instance: the kernel instance eval_batch launches for these options."""
    buf = C.create_string_buffer(128)
    n = sc.lib.mpct_kernel_instance(sc.handle, C.byref(_opts(open_loop, want_traj)), buf, len(buf))
    if n < 0:
        raise MpctError(_lib.last_error())
    return buf.value.decode()


def shard_candidates(C_: int, ndev: int, k: int) -> np.ndarray:
    """mpct_shard_candidates: the candidates of device slot k (k, k+ndev, ... < C)."""
    lib = _lib.load()
    n = lib.mpct_shard_candidates(int(C_), int(ndev), int(k), None, 0)
    if n < 0:
        raise MpctError(_lib.last_error())
    idx = np.zeros(n, dtype=np.int64)
    lib.mpct_shard_candidates(int(C_), int(ndev), int(k), idx.ctypes.data_as(_lib.c_int64_p), n)
    return idx


def eval_batch_multi(sc: Scenario, devices, N2, Nu, delta, lam, refs, v=None, open_loop=False,
                     want_traj=False, max_qp_iter=0, feas_tol=0.0) -> EvalResult:
    """mpct_eval_batch_multi: one call scores the candidates on every GPU of ``devices`` at once
    (strided shards, one host thread, context and stream per list entry, results in the caller's
    order; a device may be listed more than once)."""
    devs = np.ascontiguousarray(np.atleast_1d(devices), dtype=np.int32)
    N2 = np.ascontiguousarray(np.atleast_1d(N2), dtype=np.int32)
    Cn = N2.size
    Nu = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(Nu), (Cn,)), dtype=np.int32)
    delta = np.ascontiguousarray(np.asarray(delta, dtype=float).reshape(Cn, sc.my))
    lam = np.ascontiguousarray(np.asarray(lam, dtype=float).reshape(Cn, sc.nu))
    refs = np.ascontiguousarray(np.asarray(refs, dtype=float).reshape(-1, sc.my, sc.nit))
    nref = refs.shape[0]
    S = Cn * nref
    vv = None
    if sc.nd + sc.nq:
        vv = np.ascontiguousarray(np.broadcast_to(np.asarray(v, dtype=float).reshape(-1, sc.nd + sc.nq, sc.nit),
                                                  (nref, sc.nd + sc.nq, sc.nit)))
    res = EvalResult(J1=np.zeros((S, sc.my)), j21=np.zeros((S, sc.my)), j22=np.zeros((S, sc.my)),
                     Jnu=np.zeros((S, sc.nu)), status=np.zeros(S, dtype=np.int32),
                     qp_iters=np.zeros(S, dtype=np.int64), nref=nref)
    r = _lib.MpctResult()
    r.J1, r.j21, r.j22, r.Jnu = _dp(res.J1), _dp(res.j21), _dp(res.j22), _dp(res.Jnu)
    r.status = _ip(res.status)
    r.qp_iters = res.qp_iters.ctypes.data_as(_lib.c_int64_p)
    if want_traj:
        res.y = np.zeros((S, sc.my, sc.nit))
        res.u = np.zeros((S, sc.nu, sc.nit))
        r.y, r.u = _dp(res.y), _dp(res.u)
        if open_loop:
            res.ys = np.zeros((S, sc.my, sc.nit))
            res.uopt = np.zeros((S, sc.nu, sc.nit))
            r.ys, r.uopt = _dp(res.ys), _dp(res.uopt)
    o = _opts(open_loop, want_traj, -1, max_qp_iter, feas_tol)
    rc = sc.lib.mpct_eval_batch_multi(sc.handle, len(devs), _ip(devs), Cn, N2.ctypes.data, Nu.ctypes.data,
                                      delta.ctypes.data, lam.ctypes.data, nref, refs.ctypes.data,
                                      vv.ctypes.data if vv is not None else None, C.byref(o), C.byref(r))
    if rc != 0:
        raise MpctError("mpct_eval_batch_multi failed (%d): %s" % (rc, _lib.last_error()))
    return res
