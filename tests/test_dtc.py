"""DTC-GPC (config 1): the product's filter design (mpct.dtc) against the oracle
restatement of mimofilter.m / filtro_siso.m, and -- on the GPU -- the engine's DTC mode against
the reference-structured loop of DTC_GPC_WW.m (oracle.dtcgpc.dtc_gpc_ww: full-history lsim per
step, normal-equation gain).  CondMin-free variant L = R = I (no WoodBerry tuning file exists);
trajectories vs MATLAB itself: parity unpinned."""
import numpy as np
import pytest

TRAJ_RTOL = 1e-7


def _trel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


def test_filter_matches_oracle_and_unit_gain():
    from mpct.dtc import WB_K, WB_L, WB_TAU, mimofilter, robust_filter
    from mpct.lti import c2d
    from oracle.dtcgpc import filtro_siso, mimofilter as o_mimofilter, woodberry_models

    Pn = [[c2d([WB_K[i, j]], [WB_TAU[i, j], 1.0], 1.0, WB_L[i, j]) for j in range(2)] for i in range(2)]
    mine = mimofilter(Pn)
    ref = o_mimofilter(woodberry_models()[1])
    for f, (Nr, Dr) in zip(mine, ref):
        np.testing.assert_allclose(f.num, Nr, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(f.den, Dr, rtol=1e-12, atol=1e-14)
        assert np.sum(f.num) / np.sum(f.den) == pytest.approx(1.0, abs=1e-12)   # mimofilter.m:52-57
    # dead time 0: the underdetermined Sylvester system (filtro_siso.m:31-35, mldivide basic solution)
    den = np.convolve([1.0, -0.95], [1.0, -0.9])
    f0 = robust_filter(den, 0)
    Nr0, Dr0 = filtro_siso([0.0, 0.0, 1.0], den, 0, 0.7, 0.8)
    np.testing.assert_allclose(f0.num, Nr0, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(f0.den, Dr0, rtol=1e-12)


@pytest.fixture(scope="module")
def gpu(built, has_gpu):
    if not has_gpu:
        pytest.skip("no GPU")
    return True


@pytest.mark.gpu
@pytest.mark.parametrize("case", [dict(), dict(deltak=0.1), dict(deltak=-0.15, deltaL=1.0), dict(filt=False)])
def test_dtc_gpc_ww_trajectories(gpu, case):
    from mpct.dtc import woodberry_dtc
    from mpct.engine import eval_batch
    from oracle.dtcgpc import dtc_gpc_ww

    sc, r, q = woodberry_dtc(n2_max=10, nu_max=5, **case)
    res = eval_batch(sc, np.array([3], np.int32), np.array([3], np.int32), np.ones((1, 2)), np.ones((1, 2)),
                     r[None], v=q[None], want_traj=True)
    ref = dtc_gpc_ww(**case)
    assert res.status[0] == 0
    assert _trel(res.y[0], ref["y"]) < TRAJ_RTOL, _trel(res.y[0], ref["y"])
    assert _trel(res.u[0], ref["u"]) < TRAJ_RTOL, _trel(res.u[0], ref["u"])
    J1 = np.sum((ref["y"] - ref["r"]) ** 2, axis=1)
    np.testing.assert_allclose(res.J1[0], J1, rtol=1e-6)


@pytest.mark.gpu
def test_dtc_batch_of_candidates(gpu):
    """A batch of (p, m, lambda, delta) candidates in DTC mode: each row equals its own
    single-candidate run (batch independence) and the reference point is among them."""
    from mpct.dtc import woodberry_dtc
    from mpct.engine import eval_batch
    from oracle.dtcgpc import dtc_gpc_ww

    sc, r, q = woodberry_dtc(n2_max=12, nu_max=6)
    rng = np.random.default_rng(3)
    C = 32
    N2 = rng.integers(3, 13, C).astype(np.int32)
    Nu = np.minimum(rng.integers(1, 7, C), N2).astype(np.int32)
    N2[0], Nu[0] = 3, 3
    d = 10.0 ** rng.uniform(-1, 1, (C, 2))
    l = 10.0 ** rng.uniform(-1, 1, (C, 2))
    d[0] = l[0] = 1.0
    res = eval_batch(sc, N2, Nu, d, l, r[None], v=q[None])
    assert np.all(res.status == 0)
    one = eval_batch(sc, N2[5:6], Nu[5:6], d[5:6], l[5:6], r[None], v=q[None])
    np.testing.assert_array_equal(one.J1[0], res.J1[5])
    ref = dtc_gpc_ww()
    np.testing.assert_allclose(res.J1[0], np.sum((ref["y"] - ref["r"]) ** 2, axis=1), rtol=1e-6)


@pytest.mark.gpu
def test_dtc_monte_carlo_variants(gpu):
    """Config 4: simulation (c, k) runs plant variant k -- bitwise equal to a single-plant
    scenario built with that draw, and a uniform-mismatch draw equals the oracle loop."""
    from mpct.dtc import robust_scores, woodberry_dtc, woodberry_mc
    from mpct.engine import Scenario, eval_batch
    from oracle.dtcgpc import dtc_gpc_ww

    D, C = 4, 6
    sc, refs, v, plants = woodberry_mc(draws=D, n2_max=10, nu_max=5)
    rng = np.random.default_rng(5)
    N2 = rng.integers(3, 11, C).astype(np.int32)
    Nu = np.minimum(rng.integers(1, 6, C), N2).astype(np.int32)
    d = 10.0 ** rng.uniform(-1, 1, (C, 2))
    l = 10.0 ** rng.uniform(-1, 1, (C, 2))
    res = eval_batch(sc, N2, Nu, d, l, refs, v=v, want_traj=True)
    assert np.all(res.status == 0)
    for k in (0, 2, 3):
        one_sc, r, q = woodberry_dtc(n2_max=10, nu_max=5)
        # the same disturbance paths as the MC scenario, one plant
        from mpct.dtc import WB_QK, WB_QL, WB_QTAU, mimofilter
        from mpct.lti import c2d
        Pq = [[c2d([WB_QK[i]], [WB_QTAU[i], 1.0], 1.0, WB_QL[i])] for i in range(2)]
        single = Scenario(plants[k], one_sc.model, nu=2, du_min=-np.full(2, np.inf), du_max=np.full(2, np.inf),
                          u_min=-np.full(2, np.inf), u_max=np.full(2, np.inf), yref=r, n2_max=10, nu_max=5,
                          window="gpc", weights_squared=False, exact_carima=False, dtc=True,
                          filters=mimofilter(one_sc.model), dist=Pq)
        rs = eval_batch(single, N2, Nu, d, l, r[None], v=q[None])
        np.testing.assert_array_equal(rs.J1, res.J1.reshape(C, D, 2)[:, k])
    mean, worst = robust_scores(res.J1, C, D)
    assert np.all(worst >= mean)
    # a uniform gain/delay mismatch draw against the reference-structured loop
    from mpct.dtc import WB_K, WB_L, WB_TAU
    from mpct.lti import c2d as c2d_
    Pu = [[c2d_([WB_K[i, j] * 1.1], [WB_TAU[i, j], 1.0], 1.0, WB_L[i, j] + 1.0) for j in range(2)] for i in range(2)]
    sc2, r2, q2 = woodberry_dtc(n2_max=10, nu_max=5, deltak=0.1, deltaL=1.0)
    ru = eval_batch(sc2, np.array([3], np.int32), np.array([3], np.int32), np.ones((1, 2)), np.ones((1, 2)),
                    r2[None], v=q2[None], want_traj=True)
    ref = dtc_gpc_ww(deltak=0.1, deltaL=1.0)
    assert _trel(ru.y[0], ref["y"]) < TRAJ_RTOL
    assert all(Pu[i][j].delay == sc2.plant[i][j].delay for i in range(2) for j in range(2))
