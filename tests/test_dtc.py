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


def test_mc_draws_match_oracle():
    """Config 4's plant-mismatch draws: the product's (mpct.dtc.woodberry_mc_plants) equal the
    oracle's restatement of the draw recipe (DTC_GPC_WW.m:18-19) entry by entry."""
    from mpct.dtc import woodberry_mc_plants
    from oracle.dtcgpc import woodberry_mc_draws

    mine = woodberry_mc_plants(32)
    ref = woodberry_mc_draws(32)
    for Pm, Po in zip(mine, ref):
        for i in range(2):
            for j in range(2):
                a, b = Pm[i][j], Po[i][j]
                assert a.delay == b.iodelay
                np.testing.assert_allclose(np.trim_zeros(np.asarray(a.num), "f"), np.trim_zeros(b.num, "f"),
                                           rtol=1e-13, atol=0)
                np.testing.assert_allclose(a.den, b.den, rtol=1e-13, atol=0)


def test_config4_grid_shape():
    """SURVEY §8d config 4 grid: p in 3..30, m in 1..min(p, 10), log-uniform weights."""
    from mpct.dtc import config4_candidates

    N2, Nu, d, l = config4_candidates(10000)
    assert N2.min() >= 3 and N2.max() <= 30 and Nu.min() >= 1 and np.all(Nu <= np.minimum(N2, 10))
    assert d.shape == l.shape == (10000, 2) and d.min() >= 1e-3 and l.max() <= 10.0
    sel = (N2 >= 13) & (Nu >= 7)
    assert sel.sum() > 100  # the MAXM = 32 range the GPU test below draws from


def _oracle_compare(res, C, D, N2, Nu, d, l, pairs, plants):
    """Compare simulations (c, k) of a plant-variant batch with the reference-structured loop on
    draw k's plant (oracle.dtcgpc.dtc_gpc_ww(plant=...)): y and u to TRAJ_RTOL of their peak,
    J1 to 1e-6 relative."""
    from oracle.dtcgpc import dtc_gpc_ww

    worst = 0.0
    for c, k in pairs:
        s = c * D + k
        p, m = int(N2[c]), int(Nu[c])
        ref = dtc_gpc_ww(p=(p, p), m=(m, m), lam=tuple(l[c]), delta=tuple(d[c]), plant=plants[k])
        if not np.all(np.isfinite(ref["y"])):
            assert res.status[s] & 4, (c, k, res.status[s])  # overflow on both sides
            continue
        # a draw that destabilises the loop (|y| up to 1e86 on this grid) is still compared: the
        # divergent trajectories agree to the same relative accuracy
        assert res.status[s] == 0, (c, k, res.status[s])
        ey, eu = _trel(res.y[s], ref["y"]), _trel(res.u[s], ref["u"])
        J1 = np.sum((ref["y"] - ref["r"]) ** 2, axis=1)
        ej = float(np.max(np.abs(res.J1[s] - J1) / np.abs(J1)))
        worst = max(worst, ey, eu)
        assert ey < TRAJ_RTOL and eu < TRAJ_RTOL, (c, k, p, m, ey, eu)
        assert ej < 1e-6, (c, k, p, m, ej)
    return worst


@pytest.mark.gpu
def test_dtc_monte_carlo_variants(gpu):
    """Config 4 plant variants: simulation (c, k) runs draw k's plant -- each checked against the
    reference-structured loop on that draw's plant (not against another HIP run)."""
    from mpct.dtc import robust_scores, woodberry_mc
    from mpct.engine import eval_batch
    from oracle.dtcgpc import woodberry_mc_draws

    D, C = 4, 6
    sc, refs, v, _ = woodberry_mc(draws=D, n2_max=10, nu_max=5)
    plants = woodberry_mc_draws(D)
    rng = np.random.default_rng(5)
    N2 = rng.integers(3, 11, C).astype(np.int32)
    Nu = np.minimum(rng.integers(1, 6, C), N2).astype(np.int32)
    d = 10.0 ** rng.uniform(-1, 1, (C, 2))
    l = 10.0 ** rng.uniform(-1, 1, (C, 2))
    res = eval_batch(sc, N2, Nu, d, l, refs, v=v, want_traj=True)
    pairs = [(c, k) for c in range(C) for k in (0, 2, 3)]
    _oracle_compare(res, C, D, N2, Nu, d, l, pairs, plants)
    mean, worst = robust_scores(res.J1, C, D)
    assert np.all(worst >= mean)
    # the cost-only batch runs dtc_small_kernel (no QP: the loop is unconstrained): its J1 against
    # the same reference-structured loop, draw by draw
    cost = eval_batch(sc, N2, Nu, d, l, refs, v=v)
    _oracle_costs(cost, D, N2, Nu, d, l, pairs, plants)


def _oracle_costs(res, D, N2, Nu, d, l, pairs, plants):
    """J1 of simulations (c, k) of a cost-only batch against DTC_GPC_WW.m's loop on draw k's plant,
    1e-6 relative (the BASELINE tolerance); non-finite on both sides where the draw diverges."""
    from oracle.dtcgpc import dtc_gpc_ww

    for c, k in pairs:
        s = c * D + k
        p, m = int(N2[c]), int(Nu[c])
        ref = dtc_gpc_ww(p=(p, p), m=(m, m), lam=tuple(l[c]), delta=tuple(d[c]), plant=plants[k])
        J1 = np.sum((ref["y"] - ref["r"]) ** 2, axis=1)
        if not np.all(np.isfinite(J1)):
            assert res.status[s] & 4, (c, k, res.status[s])
            continue
        assert res.status[s] == 0, (c, k, res.status[s])
        ej = float(np.max(np.abs(res.J1[s] - J1) / np.abs(J1)))
        assert ej < 1e-6, (c, k, p, m, ej)


@pytest.mark.gpu
def test_config4_range_against_oracle(gpu):
    """Config 4 at its own workload: candidates of the seeded 10,000-candidate grid with N2 in
    13..30 and Nu in 7..10 (M = 14..20: the DTC MAXM = 32 kernel instance) on the 32-draw
    Monte-Carlo scenario of the benchmark, every draw scored in one launch, and a spread of
    (candidate, draw) pairs compared with DTC_GPC_WW.m's loop on that draw's plant."""
    from mpct.dtc import config4_candidates, woodberry_mc
    from mpct.engine import eval_batch
    from oracle.dtcgpc import woodberry_mc_draws

    D = 32
    sc, refs, v, _ = woodberry_mc(draws=D, n2_max=30, nu_max=10)
    N2g, Nug, dg, lg = config4_candidates(10000)
    idx = np.flatnonzero((N2g >= 13) & (Nug >= 7))[:8]
    N2, Nu, d, l = N2g[idx], Nug[idx], dg[idx], lg[idx]
    assert len(np.unique(Nu)) >= 2 and Nu.max() * 2 > 16
    from mpct.engine import kernel_instance

    assert kernel_instance(sc, want_traj=True) == "gpc_closed_loop_kernel<16,true,true> + <32,true,true>"
    assert kernel_instance(sc) == "dtc_small_kernel<16> + dtc_small_kernel<32>"
    res = eval_batch(sc, N2, Nu, d, l, refs, v=v, want_traj=True)
    cost = eval_batch(sc, N2, Nu, d, l, refs, v=v)   # the cost-only instance the bench times
    ok = res.status == 0
    # two kernels (the general one with trajectories, dtc_small_kernel for costs): the same loop
    # with the plant terms summed in another order, so equal to rounding, not bitwise
    np.testing.assert_array_equal(cost.status, res.status)
    _costs_agree(cost, res, ok)
    plants = woodberry_mc_draws(D)
    pairs = [(c, (5 * c + j * 11) % D) for c in range(len(idx)) for j in range(3)]
    worst = _oracle_compare(res, len(idx), D, N2, Nu, d, l, pairs, plants)
    _oracle_costs(cost, D, N2, Nu, d, l, pairs, plants)
    print("config-4 range: %d pairs, max traj rel err %.2e" % (len(pairs), worst))


@pytest.mark.gpu
def test_dtc_small_kernel_against_general(gpu):
    """dtc_small_kernel (cost-only, the config-4 bench's launch) against the general DTC kernel
    (the trajectory instance) over every draw of 96 seeded config-4 candidates spanning both QP-size
    classes: identical statuses, J1 and j22 equal to 1e-9 relative wherever the loop stays bounded
    (_costs_agree)."""
    from mpct.dtc import config4_candidates, woodberry_mc
    from mpct.engine import eval_batch

    D = 32
    sc, refs, v, _ = woodberry_mc(draws=D, n2_max=30, nu_max=10)
    N2, Nu, d, l = config4_candidates(10000)
    idx = np.concatenate([np.arange(64), np.flatnonzero(2 * Nu > 16)[:32]])
    cost = eval_batch(sc, N2[idx], Nu[idx], d[idx], l[idx], refs, v=v)
    gen = eval_batch(sc, N2[idx], Nu[idx], d[idx], l[idx], refs, v=v, want_traj=True)
    np.testing.assert_array_equal(cost.status, gen.status)
    ok = cost.status == 0
    assert ok.mean() > 0.5 and np.all(cost.qp_iters == 0)
    _costs_agree(cost, gen, ok)


def _costs_agree(a, b, ok, bound=1e12):
    """Two kernels' costs for the same loops: 1e-9 relative where the closed loop stays bounded
    (every cost below `bound`), 1e-6 relative where a mismatched draw makes it grow without
    settling, since rounding that differs in the last bit is amplified by the growth itself (a
    loop at 1e139 differed by 1.07e-9 in r06j).  The two sets must be the same on both sides."""
    big_a = np.max(np.abs(a.J1), axis=1) >= bound
    big_b = np.max(np.abs(b.J1), axis=1) >= bound
    np.testing.assert_array_equal(big_a[ok], big_b[ok])
    tame = ok & ~big_a
    print("costs compared: %d bounded loops at 1e-9, %d growing at 1e-6" % (tame.sum(), (ok & big_a).sum()))
    for f in ("J1", "j22"):
        np.testing.assert_allclose(getattr(a, f)[tame], getattr(b, f)[tame], rtol=1e-9, atol=0)
        np.testing.assert_allclose(getattr(a, f)[ok & big_a], getattr(b, f)[ok & big_a], rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_config4_full_size_properties(gpu):
    """the launch the dtc-mc bench times, at full size -- the seeded 10,000
    config-4 candidates x 32 plant-mismatch draws (320,000 closed loops, DTC_GPC_WW.m:18-19 /
    WoodBerry.m:34-42 draws) in one call, cost only.  Size-independent properties: statuses are
    only 0 or 4 (the unconstrained DTC loop has no QP; a draw the mismatch destabilises is
    non-finite), the costs are finite exactly where the status is 0, a repeated launch is bitwise
    identical, and scoring the candidates in reversed order gives the same per-simulation bits."""
    import torch
    from mpct.dtc import config4_candidates, robust_scores, woodberry_mc
    from mpct.engine import eval_batch_device

    C, D = 10000, 32
    sc, refs, v, _ = woodberry_mc(draws=D, n2_max=30, nu_max=10)
    N2, Nu, d, l = config4_candidates(C)
    dev = torch.device("cuda", 0)

    def run(perm):
        t = [torch.from_numpy(np.ascontiguousarray(a[perm])).to(dev) for a in (N2, Nu, d, l)]
        out = dict(J1=torch.empty((C * D, 2), dtype=torch.float64, device=dev),
                   status=torch.empty(C * D, dtype=torch.int32, device=dev))
        eval_batch_device(sc, *t, torch.from_numpy(refs).to(dev), out, v=torch.from_numpy(v).to(dev))
        torch.cuda.synchronize(dev)
        return out["J1"].cpu().numpy().reshape(C, D, 2), out["status"].cpu().numpy().reshape(C, D)

    ident = np.arange(C)
    J1, st = run(ident)
    assert set(np.unique(st).tolist()) <= {0, 4}, np.unique(st)
    assert np.all(np.isfinite(J1[st == 0])) and (st == 0).mean() > 0.5
    J1b, stb = run(ident)
    assert np.array_equal(st, stb) and np.array_equal(J1.view(np.int64), J1b.view(np.int64))
    rev = ident[::-1]
    J1r, str_ = run(rev)
    assert np.array_equal(st, str_[::-1]) and np.array_equal(J1.view(np.int64), J1r[::-1].view(np.int64))
    mean, worst = robust_scores(np.where(np.isfinite(J1), J1, np.inf).reshape(C * D, 2), C, D)
    print("config 4 full size: %d of %d closed loops non-finite; best worst-case %.4g"
          % (int((st == 4).sum()), C * D, float(np.min(worst))))
