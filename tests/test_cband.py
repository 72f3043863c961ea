"""oracle/cband.c — the C restatement of the config-3 band-mode toolbox loop (oracle/toolbox_band.py)
— and the committed config-3 cost fixture it generated (tests/golden/make_config3_fixture.py).

CPU: the C port equals the numpy oracle (trajectories within 1e-7 of their peak, costs within
1e-6 relative) on the committed Shell 7x5 tuning, on seeded grid candidates and on WoodBerry's
toolbox MPC (rate bounds + tracking weights, the general H path); its per-step replay equals
numpy's replay_moves; and the fixture reproduces.  GPU (-m gpu, tests/test_band.py): the mdband
kernel against this fixture over the config-3 grid.  Against MATLAB's MPC Toolbox itself: parity
unpinned (closed source, no committed trajectories)."""
import os

import numpy as np
import pytest

TRAJ_RTOL = 1e-7
COST_RTOL = 1e-6
FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "config3_cband.npz")


def _trel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


@pytest.fixture(scope="module")
def shell():
    from oracle.cband import CBand
    from oracle.scenarios import shell7x5

    sc, r, v, yref, fx = shell7x5()
    return sc, r, v, yref, fx, CBand(sc, 200, yref)


def test_cband_equals_numpy_oracle_shell7x5(shell):
    from oracle.toolbox_band import closedloop_band

    sc, r, v, yref, fx, cb = shell
    lam = np.array(fx["lambda"])
    cands = [(27, 2, np.zeros(7), lam), (12, 3, np.zeros(7), np.array([0.05, 0.02, 1.6])),
             (20, 4, np.concatenate([np.zeros(2), [0.1, 0.3, 0.5, 0.2, 1.0]]), np.array([0.2, 0.05, 1.0]))]
    for N2, Nu, d, lm in cands:
        ref = closedloop_band(sc, r, v, N2, Nu, d, lm, 200)
        o = cb.eval([N2], [Nu], d[None], lm[None], r[None], v[None], open_loop=True, want_traj=True)
        assert o["status"][0] == 0
        for k, b in (("y", ref.y), ("u", ref.u), ("ys", ref.ys), ("uopt", ref.uopt)):
            assert _trel(o[k][0], b) < TRAJ_RTOL, (N2, Nu, k, _trel(o[k][0], b))
        np.testing.assert_allclose(o["J1"][0], ((ref.y - yref) ** 2).sum(1), rtol=COST_RTOL)
        np.testing.assert_allclose(o["j22"][0], ((ref.y - yref)[:, 9:] ** 2).sum(1), rtol=COST_RTOL)
        np.testing.assert_allclose(o["j21"][0], ((ref.y - ref.ys)[:, 9:] ** 2).sum(1), rtol=COST_RTOL, atol=1e-14)


def test_cband_replay_equals_numpy_replay(shell):
    """Replay of an applied trajectory: at the C port's own free run the oracle moves are the
    applied ones, and on a perturbed trajectory they equal numpy's replay_moves."""
    from oracle.toolbox_band import replay_moves

    sc, r, v, yref, fx, cb = shell
    N2, Nu, lm = 16, 3, np.array([0.1, 0.03, 2.0])
    o = cb.eval([N2], [Nu], np.zeros((1, 7)), lm[None], r[None], v[None], want_traj=True)
    du_o, du_a, st = cb.replay([N2], [Nu], np.zeros((1, 7)), lm[None], r, v, o["u"], T=200)
    assert st[0] == 0 and _trel(du_a[0], du_o[0]) < 1e-12
    U = o["u"][0] * (1 + 1e-3 * np.sin(np.arange(200)))[None, :]
    du_o, du_a, st = cb.replay([N2], [Nu], np.zeros((1, 7)), lm[None], r, v, U[None], T=30)
    no, na_ = replay_moves(sc, r, v, N2, Nu, np.zeros(7), lm, U, T=30)
    assert _trel(du_o[0], no) < 1e-9 and _trel(du_a[0], na_) < 1e-15


def test_cband_equals_numpy_oracle_woodberry():
    """WoodBerry.m's toolbox MPC: rate + amplitude bounds, tracking weights (dense H), one MD."""
    from oracle.cband import CBand
    from oracle.scenarios import woodberry_toolbox
    from oracle.toolbox_band import closedloop_band

    sc, r, v, yref = woodberry_toolbox()
    cb = CBand(sc, 400, yref)
    d, lm = np.array([1.0, 0.5]), np.array([0.1, 0.2])
    ref = closedloop_band(sc, r, v, 12, 3, d, lm, 400)
    o = cb.eval([12], [3], d[None], lm[None], r[None], v[None], open_loop=True, want_traj=True)
    assert o["status"][0] == 0
    for k, b in (("y", ref.y), ("u", ref.u), ("ys", ref.ys), ("uopt", ref.uopt)):
        assert _trel(o[k][0], b) < TRAJ_RTOL, (k, _trel(o[k][0], b))
    np.testing.assert_allclose(o["J1"][0], ((ref.y - yref) ** 2).sum(1), rtol=COST_RTOL)


def test_config3_fixture_reproduces(shell):
    """A spread of the committed fixture's candidates, re-scored by the C port now."""
    from mpct.scenarios import SHELL7_W, config3_grid, config3_stratified

    sc, r, v, yref, fx, cb = shell
    d = np.load(FIXTURE)
    assert d["J1_strat"].shape == (8192, 7) and d["F_full"].shape == (65536,)
    assert int(np.sum(d["st_full"] != 0)) == 0
    N2, Nu, D, L = config3_grid(1024)
    s = config3_stratified(128)
    pick = np.arange(0, 8192, 8192 // 16) + np.arange(16) % 5          # one per 4 cells, N2 <= 127
    idx = s[pick]
    o = cb.eval(N2[idx], Nu[idx], D[idx], L[idx], r[None], v[None], threads=4)
    np.testing.assert_allclose(o["J1"], d["J1_strat"][pick], rtol=1e-12)
    np.testing.assert_allclose(o["J1"] @ SHELL7_W, d["F_full"][idx], rtol=1e-12)


def test_pinned_gap_judges_moves_by_cost(shell):
    """toolbox_band.pinned_gap (the objective form of the replay check): the oracle's own moves
    attain its optimum; on Shell 7x5 after the disturbance enters, a move pushed 5 % off the
    optimum changes the cost by ~1e-13 only (the band slack dominates: the flat optimum of
    DESIGN §11); with tracking weights (WoodBerry) the same push costs visibly more."""
    from oracle.cband import CBand
    from oracle.scenarios import woodberry_toolbox
    from oracle.toolbox_band import pinned_gap

    sc, r, v, yref, fx, cb = shell
    N2, Nu, lm = 16, 3, np.array([0.1, 0.03, 2.0])
    o = cb.eval([N2], [Nu], np.zeros((1, 7)), lm[None], r[None], v[None], want_traj=True)
    U = o["u"][0]
    for t in (5, 25, 60):
        J0, J1, du = pinned_gap(sc, r, v, N2, Nu, np.zeros(7), lm, U, t)
        assert abs(J1 - J0) <= 1e-9 * J0
        np.testing.assert_allclose(du, U[:, t] - U[:, t - 1], rtol=1e-7, atol=1e-15)
    Up = U.copy()
    Up[0, 25:] += 0.05 * abs(U[0, 25] - U[0, 24])
    J0, J1, _ = pinned_gap(sc, r, v, N2, Nu, np.zeros(7), lm, Up, 25)
    assert 0 <= J1 - J0 < 1e-9 * J0                          # flat along the moves
    wsc, wr, wv, wy = woodberry_toolbox()
    d, lw = np.array([1.0, 0.5]), np.array([0.1, 0.2])
    ow = CBand(wsc, 400, wy).eval([12], [3], d[None], lw[None], wr[None], wv[None], want_traj=True)
    Uw = ow["u"][0].copy()
    J0, J1, _ = pinned_gap(wsc, wr, wv, 12, 3, d, lw, Uw, 20)
    assert abs(J1 - J0) <= 1e-9 * J0
    Uw[0, 20:] += 0.05 * abs(Uw[0, 20] - Uw[0, 19])
    J0, J1, _ = pinned_gap(wsc, wr, wv, 12, 3, d, lw, Uw, 20)
    assert J1 - J0 > 1e-6 * J0


def test_cband_replay_gap_equals_numpy_pinned_gap(shell):
    """cband_replay_gap (the C certification of config-3 divergences, tools/config3_certify.py)
    equals toolbox_band.pinned_gap: the free and the pinned QP objectives at the states a perturbed
    trajectory reached, and on the C port's own trajectory the moves replay exactly."""
    from oracle.toolbox_band import pinned_gap

    sc, r, v, yref, fx, cb = shell
    N2, Nu, lm = 16, 3, np.array([0.1, 0.03, 2.0])
    o = cb.eval([N2], [Nu], np.zeros((1, 7)), lm[None], r[None], v[None], want_traj=True)
    U = o["u"][0]
    du_o, du_a, J0, J1, st = cb.replay_gap([N2], [Nu], np.zeros((1, 7)), lm[None], r, v, U[None], threads=2)
    assert st[0] == 0
    assert np.max(np.abs(du_o - du_a)) <= 1e-12 * np.abs(du_a).max()
    Up = U.copy()
    Up[0, 30:] += 1e-4
    du_o, du_a, J0, J1, st = cb.replay_gap([N2], [Nu], np.zeros((1, 7)), lm[None], r, v, Up[None], threads=2)
    for t in (25, 30, 60):
        a, b, _ = pinned_gap(sc, r, v, N2, Nu, np.zeros(7), lm, Up, t)
        np.testing.assert_allclose([J0[0, t], J1[0, t]], [a, b], rtol=1e-12)


def test_cband_warm_path_fixture(shell):
    """The C restatement's second QP path (warm-started dual method, cb_scen.qp_warm) reproduces its
    committed grid costs (tests/golden/config3_cband_warm.npz, the C-vs-C floor of DESIGN §3) on a
    sample of the grid, and differs from the cold path's fixture on ~1 % of F beyond 1e-6."""
    from mpct.scenarios import SHELL7_W, config3_grid
    from oracle.cband import CBand

    sc, r, v, yref, fx, cb = shell
    dw = np.load(os.path.join(os.path.dirname(__file__), "golden", "config3_cband_warm.npz"))
    d = np.load(FIXTURE)
    N2, Nu, D, L = config3_grid(1024)
    idx = np.arange(0, N2.size, 4099)[:16]
    o = CBand(sc, 200, yref, warm=True).eval(N2[idx], Nu[idx], D[idx], L[idx], r[None], v[None], threads=4)
    np.testing.assert_allclose(o["J1"] @ SHELL7_W, dw["F_full"][idx], rtol=1e-12)
    floor = np.mean(np.abs(dw["F_full"] - d["F_full"]) / np.abs(d["F_full"]) > 1e-6)
    assert 0.005 < floor < 0.015, floor
