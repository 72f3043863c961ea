"""CPU: pin the oracle (and the product's host-side model code) against the reference's own
committed data and algebraic identities.

Pins:
  * MPC-Tuning/Shell3x3_Tuning_25Jul2023_12_06.mat (decoded into tests/golden/
    tuning_parameters_mat.json by tests/golden/make_mat_fixtures.py): the scaled discrete plant
    L*c2d(Ps)*R embedded in the saved mpc object (num, den, iodelay), the scaled MV bounds and
    the tuned weights -> c2d ZOH with fractional delay, MPCTuning.m:162-178 scaling.
  * Identities the reference's algorithm relies on: Diophantine A~ E_j + z^-j F_j = 1
    (diophantine.m:35-79), MatG == forced step-response prediction (MatG.m:64-67), the
    free-response predictor S*Yd + Hp*up (DTC_GPC_WW.m:139-146) == the model's own continuation,
    KKT optimality of the oracle QP.
Closed-loop trajectories vs MATLAB's MPC Toolbox remain "parity unpinned" (no MATLAB, no
committed trajectories); the C port is checked against the numpy oracle instead.
"""
import numpy as np
import pytest

from oracle.matlab import DTF, c2d_fopdt, c2d_zoh, conv, lsim_dtf, step_dtf
from oracle.scenarios import (SHELL3_K, SHELL3_L, SHELL3_TAU, SHELL3_TS, load_fixture,
                              shell3x3, shell3x3_plant_scaled)


@pytest.fixture(scope="module")
def fx():
    return load_fixture("shell3x3_25jul2023")


@pytest.fixture(scope="module")
def scen():
    return shell3x3()


def _plant_fixture(fx):
    p = fx["plant_scaled_discrete"]
    return np.array(p["num"]), np.array(p["den"]), np.array(p["iodelay"])


def test_c2d_matches_mat_plant(fx):
    """oracle c2d_zoh (general state-space path) == the mpc object's scaled discrete plant."""
    L, R = np.array(fx["scale"]["L"]), np.array(fx["scale"]["R"])
    num, den, iod = _plant_fixture(fx)
    P = shell3x3_plant_scaled(L, R)
    for i in range(3):
        for j in range(3):
            d = P[i][j]
            assert d.iodelay == iod[i, j]
            np.testing.assert_allclose(d.num, num[i, j], rtol=0, atol=1e-14)
            np.testing.assert_allclose(d.den, den[i, j], rtol=0, atol=1e-14)


def test_c2d_general_equals_closed_form():
    for K, tau, L in [(4.05, 50, 27), (1.77, 60, 28), (7.2, 19, 0), (3.0, 7.0, 4.0), (1.0, 30, 14)]:
        a = c2d_zoh([K], [tau, 1.0], SHELL3_TS, L)
        b = c2d_fopdt(K, tau, SHELL3_TS, L)
        assert a.iodelay == b.iodelay
        np.testing.assert_allclose(a.num, b.num, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(a.den, b.den, rtol=1e-12, atol=1e-15)


def test_product_c2d_matches_mat_plant(fx):
    """The product's host-side model code (mpct.lti, feeds mpct_scenario_create) reproduces the
    same committed plant."""
    from mpct.scenarios import shell3x3_plant

    L, R = np.array(fx["scale"]["L"]), np.array(fx["scale"]["R"])
    num, den, iod = _plant_fixture(fx)
    P = shell3x3_plant(L, R)
    for i in range(3):
        for j in range(3):
            t = P[i][j]
            # mpct.lti.Tf keeps MATLAB's tfdata form: numerator padded to the denominator length
            assert t.delay == iod[i, j]
            np.testing.assert_allclose(t.num, num[i, j], rtol=0, atol=1e-14)
            np.testing.assert_allclose(t.den, den[i, j], rtol=0, atol=1e-14)


def test_scaled_bounds_and_weights(fx):
    """Shell3x3.m:120-123 bounds scaled by R (MPCTuning.m:170-178) == the saved object's MV
    bounds; the saved weights are the tuned delta (OV) and lambda (MV rate)."""
    R = np.array(fx["scale"]["R"])
    for n, mv in enumerate(fx["MV"]):
        assert mv["Min"] == pytest.approx(-1.0 / R[n], rel=1e-15)
        assert mv["Max"] == pytest.approx(0.5 / R[n], rel=1e-15)
        assert mv["RateMin"] == pytest.approx(-0.05 / R[n], rel=1e-15)
        assert mv["RateMax"] == pytest.approx(0.05 / R[n], rel=1e-15)
    np.testing.assert_allclose(fx["Weights"]["OutputVariables"], fx["delta"], rtol=1e-15)
    np.testing.assert_allclose(fx["Weights"]["ManipulatedVariablesRate"], fx["lambda"], rtol=1e-15)
    from mpct.scenarios import SHELL3_L as PL, SHELL3_R as PR, SHELL3_TUNED

    np.testing.assert_array_equal(PL, fx["scale"]["L"])
    np.testing.assert_array_equal(PR, fx["scale"]["R"])
    assert SHELL3_TUNED["N"] == fx["N"][0] == 24


def test_all_mat_fixtures_decoded():
    import json
    import os

    p = os.path.join(os.path.dirname(__file__), "golden", "tuning_parameters_mat.json")
    with open(p) as f:
        d = json.load(f)
    assert set(d) == {"shell3x3_25jul2023", "shell3x3_caso2", "shell7x5_25jul2023", "shell7x5_14sep2024",
                      "vandevusse_25jul2023", "vandevusse_06dec2023"}
    # reference determinism evidence: the two Shell 7x5 files hold identical tunings
    a, b = d["shell7x5_25jul2023"], d["shell7x5_14sep2024"]
    for k in ("N", "Nu", "delta", "lambda"):
        assert a[k] == b[k]
    assert d["shell3x3_caso2"]["N"] == [12] and d["shell3x3_caso2"]["Nu"] == [4, 2, 2]


def test_descomp_ba_mimo_sizes(scen):
    """SURVEY A6/A7 facts for Shell 3x3: dp, na, nb."""
    sc = scen[0]
    np.testing.assert_array_equal(sc.dp, [[6, 7, 6], [4, 3, 3], [5, 5, 0]])
    np.testing.assert_array_equal(sc.na, [2, 3, 3])
    np.testing.assert_array_equal(sc.nb, [[2, 1, 2], [3, 3, 3], [2, 3, 2]])


@pytest.mark.parametrize("d", [0, 3])
def test_diophantine_identity(scen, d):
    from oracle.dtcgpc import diophantine

    sc = scen[0]
    N = 30
    for i in range(sc.my):
        A = np.asarray(sc.A[i], dtype=float)
        AD = conv(A, [1.0, -1.0])
        E, F = diophantine(A, N, d)
        for r in range(N):
            j = d + 1 + r
            Ej = E[r, :j]
            lhs = conv(AD, Ej)
            rhs = np.zeros(max(len(lhs), j + F.shape[1]))
            rhs[: len(lhs)] += lhs
            rhs[j: j + F.shape[1]] += F[r]
            expect = np.zeros_like(rhs)
            expect[0] = 1.0
            np.testing.assert_allclose(rhs, expect, rtol=0, atol=1e-9 * max(1.0, np.abs(F[r]).max()))


def test_matg_is_forced_response(scen):
    """G @ dU == lsim of the model driven by the future moves only (toolbox window t+1..t+N2)."""
    from oracle.toolbox_gpc import prediction_tables

    sc = scen[0]
    N2, Nu = 30, 5
    G, S, Hp, duM = prediction_tables(sc, N2, Nu)
    rng = np.random.default_rng(0)
    dU = rng.standard_normal((sc.nu, Nu))
    y = G @ dU.reshape(-1)
    T = N2 + 1
    for i in range(sc.my):
        acc = np.zeros(T)
        for n in range(sc.nu):
            du = np.zeros(T)
            du[:Nu] = dU[n]
            acc += lsim_dtf(sc.model[i][n], np.cumsum(du))
        np.testing.assert_allclose(y[i * N2:(i + 1) * N2], acc[1:N2 + 1], rtol=1e-12, atol=1e-12)


def test_free_response_predictor(scen):
    """S*Yd + Hp*up (DTC_GPC_WW.m:139-146 state; Diophantine F + deltaUFree) == the model's own
    continuation with zero future moves, after a random past."""
    from oracle.toolbox_gpc import prediction_tables

    sc = scen[0]
    N2, Nu = 30, 5
    G, S, Hp, duM = prediction_tables(sc, N2, Nu)
    rng = np.random.default_rng(1)
    T0 = 60                      # past length (>= every history the predictor reads)
    du = np.zeros((sc.nu, T0 + N2 + 1))
    du[:, :T0 - 1] = rng.standard_normal((sc.nu, T0 - 1)) * 0.1
    u = np.cumsum(du, axis=1)
    Y = np.zeros((sc.my, T0 + N2 + 1))
    for i in range(sc.my):
        for n in range(sc.nu):
            Y[i] += lsim_dtf(sc.model[i][n], u[n])
    t = T0 - 1                   # now: y(t) measured, du(t) is the first free move (zero)
    yd = np.concatenate([Y[i, t - np.arange(sc.na[i] + 1)] for i in range(sc.my)])
    up = np.concatenate([du[n, t - 1 - np.arange(duM[n])] for n in range(sc.nu)])
    f = S @ yd + Hp @ up
    for i in range(sc.my):
        np.testing.assert_allclose(f[i * N2:(i + 1) * N2], Y[i, t + 1:t + 1 + N2], rtol=1e-9, atol=1e-9)


def test_primal_active_set_kkt():
    from oracle.toolbox_gpc import constraint_rows, qp_primal_active_set

    rng = np.random.default_rng(7)
    nu, Nu = 3, 4
    M = nu * Nu
    for trial in range(20):
        W = rng.standard_normal((M + 10, M))
        c = rng.standard_normal(M + 10) * 5
        up = rng.uniform(-0.5, 0.5, nu)
        A, b = constraint_rows(nu, Nu, -0.2 * np.ones(nu), 0.2 * np.ones(nu), -1.0 * np.ones(nu),
                               0.6 * np.ones(nu), up)
        x, it = qp_primal_active_set(W, c, A, b)[:2]
        s = A @ x - b
        assert s.min() > -1e-10
        g = W.T @ (W @ x + c)
        act = np.nonzero(s < 1e-9)[0]
        if len(act):
            # degenerate active sets (a prefix amplitude row = sum of its rate rows) have
            # non-unique multipliers: KKT holds iff SOME lam >= 0 reproduces the gradient
            from scipy.optimize import nnls

            lam, res = nnls(A[act].T, g)
            assert res < 1e-8 * max(1.0, np.abs(g).max()), res
        else:
            assert np.abs(g).max() < 1e-8


def test_c_port_matches_numpy_oracle(scen, built):
    """oracle/cgpc.c (stable QR + dual active set) vs the numpy oracle (lstsq + primal active set):
    two independent QP algorithms, same closed loop."""
    from oracle.cport import CPort
    from oracle.scenarios import candidate_grid
    from oracle.toolbox_gpc import closedloop_toolbox

    sc, r, yref, fx = scen
    N2, Nu, d, l = candidate_grid(3, fx=fx)
    cp = CPort(sc, 30, 500, yref)
    res = cp.eval(N2, Nu, d, l, r[None], open_loop=True, want_traj=True, threads=1)
    for k in range(3):
        o = closedloop_toolbox(sc, r, None, 30, 5, d[k], l[k], 500, open_loop=True)
        for name, a, b in (("y", res["y"][k], o.y), ("u", res["u"][k], o.u), ("ys", res["ys"][k], o.ys),
                           ("uopt", res["uopt"][k], o.uopt)):
            e = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
            assert e < 1e-7, (k, name, e)
    J1 = np.sum((o.y - yref) ** 2, axis=1)
    np.testing.assert_allclose(res["J1"][2], J1, rtol=1e-7)


def test_objectives():
    from oracle.objectives import gam_j1, precon, vns_terms

    assert precon([24, 24, 24], [6, 2, 2])
    assert not precon([6, 24, 24], [6, 2, 2])        # min(N) must exceed max(Nu)
    assert not precon([24, 24, 24], [6, 0, 2])       # no zeros
    y = np.array([[1.0, 2.0, 3.0]])
    np.testing.assert_allclose(gam_j1(y, np.zeros_like(y)), [14.0])
    # VNS2.m:183-191: |uopt(:,1)| ./ |diff(uopt)|, inf/NaN -> 0, then squared and summed
    uopt = np.array([1.0, 1.0, 3.0, 3.0])
    j21, j22, jnu = vns_terms(np.ones(12), np.zeros(12), np.zeros(12), uopt, inK=10)
    assert j21 == pytest.approx(3.0) and j22 == pytest.approx(3.0)
    assert jnu == pytest.approx(0.25)
