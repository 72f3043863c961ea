"""Van de Vusse NMPC (config 5, VanDeVusse_NMPC.m / closedloop_toolbox_nmpc.m).

CPU: the oracle restatement (oracle/nmpc_vdv.py) is pinned to the reference's committed NMPC
tuning files (MV bounds, OV bounds, ScaleFactors of the saved nlmpc object), to the model's own
identities (x0 is an equilibrium at u0; the RK4 sensitivities equal finite differences of the RK4
map) and to the optimality of every controller move (projected gradient of the Gauss-Newton
problem = 0 on the bounds).  The product host setup (steady state, references) matches it.
GPU (-m gpu): nmpc_kernel.hip through the C ABI against the oracle: closed-loop and open-loop
trajectories, all cost terms, determinism and batch-order independence.
Trajectories against MATLAB's nlmpc itself: parity unpinned (closed source: fmincon, ode15s)."""
import numpy as np
import pytest

TRAJ_RTOL = 1e-7     # trajectories, relative to the trajectory's peak
COST_RTOL = 1e-6     # BASELINE tolerance on the costs


def _trel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


def test_nmpc_oracle_pinned_to_fixture():
    """VanDeVusse_NMPC_Tuning_*.mat: the saved nlmpc object's MV/OV bounds and ScaleFactors are
    the driver's (VanDeVusse_NMPC.m:43-164) that the oracle and the product use."""
    import json
    import os

    import oracle.nmpc_vdv as nv
    from mpct import nmpc

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tuning_parameters_mat.json")))
    for key in ("vandevusse_25jul2023", "vandevusse_06dec2023"):
        f = fx[key]
        np.testing.assert_array_equal([m["Min"] for m in f["MV"]], nv.LB)
        np.testing.assert_array_equal([m["Max"] for m in f["MV"]], nv.UB)
        np.testing.assert_array_equal([m["ScaleFactor"] for m in f["MV"]], nv.SU)
        np.testing.assert_array_equal([o["Min"] for o in f["OV"]], nv.XMIN[1:])
        np.testing.assert_array_equal([o["Max"] for o in f["OV"]], nv.XMAX[1:])
        np.testing.assert_allclose([o["ScaleFactor"] for o in f["OV"]], nv.SY, rtol=1e-15)
        assert f["Weights"]["ManipulatedVariables"] == [0.0, 0.0]
        assert all(m["RateMin"] == "-inf" and m["RateMax"] == "inf" for m in f["MV"])
        np.testing.assert_array_equal(f["delta"], nmpc.VDV_TUNED["delta"])
        np.testing.assert_array_equal(f["lambda"], nmpc.VDV_TUNED["lam"])
        assert f["N"] == [nmpc.VDV_TUNED["N"]] and f["Nu"] == list(map(float, nmpc.VDV_TUNED["Nu"]))
    np.testing.assert_array_equal(nmpc.VDV_UMIN, nv.LB)
    np.testing.assert_array_equal(nmpc.VDV_XMAX, nv.XMAX)


def test_nmpc_oracle_model_identities():
    import oracle.nmpc_vdv as nv

    x0 = nv.steady_state()
    assert np.max(np.abs(nv.rhs(x0, nv.U0))) < 1e-9
    np.testing.assert_allclose(nv.rk4(x0, nv.U0), x0, rtol=1e-12)
    # RK4 sensitivities (forward mode) vs central differences of the RK4 map
    x = x0 + np.array([0.2, -0.05, 3.0])
    u = np.array([35.0, 110.0])
    xe, X = nv.rk4(x, u, (np.eye(3, 5), np.eye(5)[3:]))
    for k in range(5):
        h = 1e-6 * max(1.0, abs(np.r_[x, u][k]))
        e = np.zeros(5)
        e[k] = h
        fd = (nv.rk4(x + e[:3], u + e[3:]) - nv.rk4(x - e[:3], u - e[3:])) / (2 * h)
        np.testing.assert_allclose(X[:, k], fd, rtol=1e-6, atol=1e-8)


def test_nmpc_oracle_controller_is_optimal():
    """At a non-trivial state the converged Gauss-Newton solution is a KKT point of the NMPC
    problem: the gradient of the cost, projected on the MV bounds, vanishes."""
    import oracle.nmpc_vdv as nv

    x0 = nv.steady_state()
    x = x0 + np.array([0.1, 0.02, -2.0])
    N, Nu, delta, lam = 8, 3, np.array([1.0, 0.5]), np.array([0.05, 0.02])
    rvec = np.array([1.0, 130.0])
    U, it = nv.controller(x, nv.U0, rvec, N, Nu, delta, lam, np.tile(nv.U0, (Nu, 1)))
    assert it < nv.SQP_MAX
    Y, S = nv.predict(x, U, N, Nu)
    wy2 = (np.abs(delta) / nv.SY) ** 2
    wu2 = (np.abs(lam) / nv.SU) ** 2
    g = np.einsum("ij,ijm->m", (Y - rvec) * wy2, S)
    du = np.diff(np.vstack([nv.U0, U]), axis=0)
    for n in range(2):
        for l in range(Nu):
            g[n * Nu + l] += wu2[n] * du[l, n] - (wu2[n] * du[l + 1, n] if l + 1 < Nu else 0.0)
    v = U.T.reshape(-1)
    lo, hi = np.repeat(nv.LB, Nu), np.repeat(nv.UB, Nu)
    pg = np.where(v <= lo + 1e-9, np.minimum(g, 0.0), np.where(v >= hi - 1e-9, np.maximum(g, 0.0), g))
    assert np.max(np.abs(pg)) < 1e-8 * max(1.0, np.max(np.abs(g))), pg


XMAX_TIGHT = np.array([6.0, 1.2, 135.0])   # T <= 135: active after the 130-degree setpoint step


def test_nmpc_oracle_state_bounds_hold():
    """Hard state bounds (VanDeVusse_NMPC.m:143-146 OutputVariables/States Min/Max): candidate 2
    of the seeded grid overshoots T = 135 without them (135.2) and stays on the bound with them."""
    import oracle.nmpc_vdv as nv
    from mpct.nmpc import nmpc_candidate_grid

    N, Nu, d, lam = nmpc_candidate_grid(64)
    x0 = nv.steady_state()
    r, _ = nv.references(x0)
    k = 2
    free = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False,
                              xbounds=(nv.XMIN, np.full(3, np.inf)))
    held = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False,
                              xbounds=(nv.XMIN, XMAX_TIGHT))
    assert free.y[1].max() > 135.1
    assert held.bounds_ok and held.y[1].max() <= 135.0 + 1e-8
    assert held.y[1].max() > 135.0 - 1e-6   # the bound is active, not merely respected


def test_nmpc_product_setup_matches_oracle(built):
    import oracle.nmpc_vdv as nv
    from mpct import nmpc

    x0 = nmpc.steady_state()
    np.testing.assert_allclose(x0, nv.steady_state(), rtol=1e-14)
    r, yref = nmpc.vandevusse_signals(x0)
    ro, yo = nv.references(x0)
    np.testing.assert_array_equal(r, ro)
    np.testing.assert_allclose(yref, yo, rtol=1e-14)
    sc, r2, y2 = nmpc.vandevusse()
    assert sc.lds_bytes(31, 15) <= 64 * 1024


def test_nmpc_scenario_errors(built):
    from mpct import nmpc
    from mpct.engine import MpctError

    x0 = nmpc.steady_state()
    r, yref = nmpc.vandevusse_signals(x0)
    with pytest.raises(MpctError, match="nu\\*nu_max"):
        nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, nmpc.VDV_XMIN, nmpc.VDV_XMAX, yref, 31, 17)
    with pytest.raises(MpctError, match="u_min"):
        nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMAX, nmpc.VDV_UMIN, nmpc.VDV_XMIN, nmpc.VDV_XMAX, yref, 31, 15)
    with pytest.raises(MpctError, match="64 KiB"):
        nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, nmpc.VDV_XMIN, nmpc.VDV_XMAX, yref, 400, 15)


def test_nmpc_oracle_returned_iterate_drift():
    """the controller returns the converged iterate v (round 4), not clip(v + d) (rounds
    1-3).  Which one nlmpcmove returns is unpinned; the two conventions' closed loops stay within
    5 SQP_TOL of each MV's ScaleFactor at every step and 1e-6 relative on J1 (measured on these
    candidates: 2.3e-8 s_u and 7.3e-7 at most)."""
    import oracle.nmpc_vdv as nv
    from mpct.nmpc import nmpc_candidate_grid, steady_state, vandevusse_signals

    r, yref = vandevusse_signals(steady_state())
    N, Nu, d, lam = nmpc_candidate_grid(64)
    for k in (0, 2, 3):
        a = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False)
        b = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False, return_step=True)
        assert np.max(np.abs(a.u - b.u) / nv.SU[:, None]) <= 5 * nv.SQP_TOL, k
        np.testing.assert_allclose(((a.y - yref) ** 2).sum(1), ((b.y - yref) ** 2).sum(1), rtol=COST_RTOL)


def test_nmpc_long_horizon_point_buffers(built):
    """the M <= 15 class's point buffers (four, two or one per simulation) are sized so
    that every (N, Nu) of a long-horizon scenario with nu * nu_max > 15 fits 64 KiB: nu = 2,
    nu_max = 8, n_max = 127 (M = 14 needed ~101 KB with two buffers) and n_max = 80, nu_max = 7
    (refused at ~67 KB before)."""
    from mpct import nmpc

    x0 = nmpc.steady_state()
    r, yref = nmpc.vandevusse_signals(x0)
    for n_max, nu_max in ((127, 8), (80, 7)):
        sc = nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, nmpc.VDV_XMIN, nmpc.VDV_XMAX, yref,
                               n_max, nu_max)
        lds = [sc.lds_bytes(N, Nu) for N in range(1, n_max + 1) for Nu in range(1, nu_max + 1)]
        assert max(lds) <= 64 * 1024, (n_max, nu_max, max(lds))


@pytest.fixture(scope="module")
def gpu(built, has_gpu):
    if not has_gpu:
        pytest.skip("no GPU")
    return True


def _cands():
    from mpct.nmpc import nmpc_candidate_grid

    N, Nu, d, lam = nmpc_candidate_grid(64)
    pick = [0, 1, 2, 3, 5, 8, 13]
    return N[pick], Nu[pick], d[pick], lam[pick]


@pytest.mark.gpu
def test_nmpc_gpu_matches_oracle(gpu):
    """The tuned point and seeded grid candidates: y, u, yopt, uopt and J1/j21/j22/Jnu."""
    import oracle.nmpc_vdv as nv
    from mpct.engine import eval_batch
    from mpct.nmpc import vandevusse

    sc, r, yref = vandevusse()
    N, Nu, d, lam = _cands()
    res = eval_batch(sc, N, Nu, d, lam, r[None], open_loop=True, want_traj=True)
    assert np.all(res.status == 0), res.status
    ink0 = 9
    for k in range(N.size):
        o = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k])
        for a, b in ((res.y[k], o.y), (res.u[k], o.u), (res.ys[k], o.yopt), (res.uopt[k], o.uopt)):
            assert _trel(a, b) < TRAJ_RTOL, (k, _trel(a, b))
        np.testing.assert_allclose(res.J1[k], ((o.y - yref) ** 2).sum(1), rtol=COST_RTOL)
        np.testing.assert_allclose(res.j22[k], ((o.y - yref)[:, ink0:] ** 2).sum(1), rtol=COST_RTOL)
        np.testing.assert_allclose(res.j21[k], ((o.y - o.yopt)[:, ink0:] ** 2).sum(1), rtol=COST_RTOL, atol=1e-12)
        du = np.abs(np.diff(o.uopt, axis=1))
        with np.errstate(divide="ignore", invalid="ignore"):
            xr = np.abs(o.uopt[:, :1]) / du
        xr[~np.isfinite(xr)] = 0.0
        np.testing.assert_allclose(res.Jnu[k], (xr ** 2).sum(1), rtol=COST_RTOL)


@pytest.mark.gpu
def test_nmpc_gpu_long_horizon_point_buffers(gpu):
    """long horizons in the M <= 15 class (nu = 2, nu_max = 8, n_max = 127) run with
    one or two point buffers instead of four (nm_groups); N = 127, Nu = 7 (M = 14, one buffer)
    and N = 70, Nu = 7 (two) equal the oracle's loop, and no slot is left unsimulated."""
    import oracle.nmpc_vdv as nv
    from mpct import nmpc
    from mpct.engine import eval_batch

    x0 = nmpc.steady_state()
    r, yref = nmpc.vandevusse_signals(x0)
    sc = nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, nmpc.VDV_XMIN, nmpc.VDV_XMAX, yref, 127, 8)
    N = np.array([127, 70, 31], np.int32)
    Nu = np.array([7, 7, 8], np.int32)
    d = np.array([[1.0, 0.5], [0.7, 1.0], [1.0, 1.0]])
    lam = np.array([[0.1, 0.1], [0.05, 0.2], [0.1, 0.1]])
    res = eval_batch(sc, N, Nu, d, lam, r[None], want_traj=True)
    assert np.all(res.status == 0), res.status
    for k in range(2):
        o = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False)
        for a, b in ((res.y[k], o.y), (res.u[k], o.u)):
            assert _trel(a, b) < TRAJ_RTOL, (k, _trel(a, b))
        np.testing.assert_allclose(res.J1[k], ((o.y - yref) ** 2).sum(1), rtol=COST_RTOL)


@pytest.mark.gpu
def test_nmpc_gpu_state_bounds_match_oracle(gpu):
    """Tight T bound: the linearised state rows enter the kernel's QP as general constraints
    (LDS bitmap of active rows, staged normals); the loops equal the oracle's re-solve."""
    import oracle.nmpc_vdv as nv
    from mpct.engine import eval_batch
    from mpct import nmpc

    x0 = nmpc.steady_state()
    r, yref = nmpc.vandevusse_signals(x0)
    # ScaleFactors stay the nominal OV ranges (VanDeVusse_NMPC.m:151,159): only the bound moves
    sc = nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, nmpc.VDV_XMIN, XMAX_TIGHT,
                           yref, 31, 15, y_scale=nv.SY)
    N, Nu, d, lam = nmpc.nmpc_candidate_grid(64)
    pick = [2, 6, 0]
    res = eval_batch(sc, N[pick], Nu[pick], d[pick], lam[pick], r[None], open_loop=True, want_traj=True)
    assert np.all(res.status == 0), res.status
    for s, k in enumerate(pick):
        o = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], xbounds=(nv.XMIN, XMAX_TIGHT))
        assert o.bounds_ok
        for a, b in ((res.y[s], o.y), (res.u[s], o.u), (res.ys[s], o.yopt), (res.uopt[s], o.uopt)):
            assert _trel(a, b) < TRAJ_RTOL, (k, _trel(a, b))
        np.testing.assert_allclose(res.J1[s], ((o.y - yref) ** 2).sum(1), rtol=COST_RTOL)
        assert res.y[s][1].max() <= 135.0 + 1e-8


@pytest.mark.gpu
def test_nmpc_gpu_deterministic_and_order_free(gpu):
    from mpct.engine import eval_batch
    from mpct.nmpc import nmpc_candidate_grid, vandevusse

    sc, r, yref = vandevusse()
    N, Nu, d, lam = nmpc_candidate_grid(256)
    a = eval_batch(sc, N, Nu, d, lam, r[None])
    b = eval_batch(sc, N[::-1], Nu[::-1], d[::-1], lam[::-1], r[None])
    np.testing.assert_array_equal(a.J1, b.J1[::-1])
    assert np.mean(a.status == 0) > 0.95, np.unique(a.status, return_counts=True)


@pytest.mark.gpu
def test_nmpc_gpu_vns_references_and_statuses(gpu):
    """VNS on a nonlinear model simulates Xsp.*sel per output (VNS2.m:148-155): two reference
    sets per candidate ride on the reference dimension, each equal to the oracle's loop on that
    reference; padding (N = 0) and bad horizons (Nu > N, N > n_max) come back as status 8 / 16
    with NaN costs; an empty batch is a no-op."""
    import oracle.nmpc_vdv as nv
    from mpct.engine import eval_batch
    from mpct.nmpc import nmpc_candidate_grid, vandevusse
    from mpct.objectives import vns_refs_nonlinear

    sc, r, yref = vandevusse()
    refs = vns_refs_nonlinear(r)
    N, Nu, d, lam = nmpc_candidate_grid(64)
    pick = [0, 4]
    res = eval_batch(sc, N[pick], Nu[pick], d[pick], lam[pick], refs, open_loop=True, want_traj=True)
    assert res.y.shape[0] == 4
    ncmp = 0
    for ci, k in enumerate(pick):
        for j in range(2):
            its = []
            orig = nv.controller

            def spy(*a, _o=orig):
                U, it = _o(*a)
                its.append(it)
                return U, it

            nv.controller = spy
            try:
                o = nv.closedloop_nmpc(refs[j], int(N[k]), int(Nu[k]), d[k], lam[k])
            finally:
                nv.controller = orig
            s = ci * 2 + j
            # a controller call that stops at the iteration cap is path dependent (Armijo decisions
            # at rounding-level ties): both sides must report it, and only converged loops compare
            assert bool(res.status[s] & 32) == (max(its) >= nv.SQP_MAX), (k, j, res.status[s], max(its))
            if res.status[s] & 32:
                continue
            ncmp += 1
            assert _trel(res.y[s], o.y) < TRAJ_RTOL and _trel(res.uopt[s], o.uopt) < TRAJ_RTOL, (k, j)
    assert ncmp >= 2
    bad = eval_batch(sc, [0, 5, 40, 6], [2, 6, 2, 3], np.ones((4, 2)), np.ones((4, 2)) * 0.1, r[None])
    assert bad.status.tolist()[:3] == [8, 16, 16] and bad.status[3] & 31 == 0
    assert np.all(np.isnan(bad.J1[:3])) and np.all(np.isfinite(bad.J1[3]))
    empty = eval_batch(sc, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 2)), np.zeros((0, 2)), r[None])
    assert empty.J1.shape == (0, 2)


@pytest.mark.gpu
def test_nmpc_gpu_anderson_reaches_every_optimum(gpu):
    """Gauss-Newton is linear on this large-residual problem: before the Anderson step 46 of the
    config-5 grid's 4096 GAM-mode simulations (72 with the open-loop leg) hit the 100-iteration cap
    at the setpoint change (status 32).  With it none does, and three of those candidates (156:
    N 27 / Nu 12, 3547: the slowest step left, 77 iterations; 3261) equal the oracle's loop."""
    import oracle.nmpc_vdv as nv
    from mpct.engine import eval_batch
    from mpct.nmpc import nmpc_candidate_grid, vandevusse

    sc, r, yref = vandevusse()
    N, Nu, d, lam = nmpc_candidate_grid(4096)
    for ol in (False, True):
        res = eval_batch(sc, N, Nu, d, lam, r[None], open_loop=ol)
        assert not np.any(res.status & 32), np.flatnonzero(res.status & 32)
        assert np.all(res.status == 0), np.unique(res.status, return_counts=True)
    pick = [156, 3547, 3261]
    res = eval_batch(sc, N[pick], Nu[pick], d[pick], lam[pick], r[None], want_traj=True)
    for s, k in enumerate(pick):
        o = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k], open_loop=False)
        for a, b in ((res.y[s], o.y), (res.u[s], o.u)):
            assert _trel(a, b) < TRAJ_RTOL, (k, _trel(a, b))
        np.testing.assert_allclose(res.J1[s], ((o.y - yref) ** 2).sum(1), rtol=COST_RTOL)
