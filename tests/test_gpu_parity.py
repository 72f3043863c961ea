"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the same inputs.

Tolerance (BASELINE.json north_star): <= 1e-6 relative on du / closed-loop cost; we also hold
trajectories to 1e-7 of their peak magnitude (TRAJ_RTOL) and require an identical
candidate ranking (cost ascending, candidate-index tiebreak).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TRAJ_RTOL = 1e-7   # max |a-b| / max |b| per trajectory (BASELINE: 1e-6 relative on du, cost)
COST_RTOL = 1e-6


def _trel(a, b):
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-300))


@pytest.fixture(scope="module")
def env(built, has_gpu):
    if not has_gpu:
        pytest.skip("no GPU")
    from mpct.scenarios import shell3x3
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3 as o_shell3x3

    sc, r, yref = shell3x3(n2_max=30, nu_max=6)
    osc, orr, oyref, fx = o_shell3x3()
    assert np.array_equal(r, orr) and np.allclose(yref, oyref, rtol=0, atol=1e-15)
    cp = CPort(osc, 30, 500, oyref)
    return dict(sc=sc, r=r, yref=yref, osc=osc, cp=cp, fx=fx)


def _rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-12)))


def test_trajectories_match_oracle(env):
    from mpct.engine import eval_batch
    from mpct.scenarios import candidate_grid

    N2, Nu, d, l = candidate_grid(6)
    res = eval_batch(env["sc"], N2, Nu, d, l, env["r"][None], open_loop=True, want_traj=True)
    ref = env["cp"].eval(N2, Nu, d, l, env["r"][None], open_loop=True, want_traj=True)
    assert np.all(res.status == 0) and np.all(ref["status"] == 0)
    for k in ("y", "u", "ys", "uopt"):
        e = _trel(getattr(res, k), ref[k])
        print("traj", k, e)
        assert e < TRAJ_RTOL, (k, e)
    assert _rel(res.J1, ref["J1"]) < COST_RTOL
    assert _rel(res.j22, ref["j22"]) < COST_RTOL


def test_numpy_oracle_fixture_point(env):
    """The committed tuned point (Shell3x3_Tuning_25Jul2023: N=24, Nu=[6 2 2] -> max 6) through
    the drop-in closedloop_toolbox vs the numpy oracle (primal active-set QP)."""
    from mpct.engine import closedloop_toolbox
    from oracle.toolbox_gpc import closedloop_toolbox as o_cl

    fx = env["fx"]
    y, u, t, ys, uopt = closedloop_toolbox(env["sc"], env["r"], None, fx["N"], fx["Nu"], fx["delta"],
                                           fx["lambda"], 500)
    ref = o_cl(env["osc"], env["r"], None, 24, 6, fx["delta"], fx["lambda"], 500, open_loop=True)
    assert _trel(y, ref.y) < TRAJ_RTOL, _trel(y, ref.y)
    assert _trel(u, ref.u) < TRAJ_RTOL, _trel(u, ref.u)
    assert _trel(ys, ref.ys) < TRAJ_RTOL, _trel(ys, ref.ys)
    assert _trel(uopt, ref.uopt) < TRAJ_RTOL, _trel(uopt, ref.uopt)
    assert t[1] - t[0] == 4.0


def test_costs_and_ranking(env):
    from mpct.engine import eval_batch
    from mpct.objectives import rank
    from mpct.scenarios import candidate_grid

    N2, Nu, d, l = candidate_grid(96)
    res = eval_batch(env["sc"], N2, Nu, d, l, env["r"][None])
    ref = env["cp"].eval(N2, Nu, d, l, env["r"][None])
    assert np.all(res.status == 0)
    assert _rel(res.J1, ref["J1"]) < COST_RTOL
    w = np.array([0.05, 0.40, 0.55])  # Shell3x3.m:161 Pareto weights
    assert np.array_equal(rank(res.J1 @ w), rank(ref["J1"] @ w))
    assert np.array_equal(rank(res.J1.sum(1)), rank(ref["J1"].sum(1)))


def test_vns_objective(env):
    from mpct.objectives import vns_objective
    from mpct.scenarios import candidate_grid, vns_step_refs

    N2, Nu, d, l = candidate_grid(5)
    N2 = np.array([30, 24, 16, 12, 30], dtype=np.int32)
    Nu = np.array([5, 6, 3, 2, 1], dtype=np.int32)
    F, j21, j22, jnu, res = vns_objective(env["sc"], N2, Nu, d, l)
    refs = vns_step_refs(3, 500)
    ref = env["cp"].eval(N2, Nu, d, l, refs, open_loop=True)
    idx = np.arange(3)
    rj21 = ref["j21"].reshape(5, 3, 3)[:, idx, idx]
    rj22 = ref["j22"].reshape(5, 3, 3)[:, idx, idx]
    assert np.all(res.status == 0)
    assert _rel(j21, rj21) < COST_RTOL
    assert _rel(j22, rj22) < COST_RTOL
    # Jnu divides by |diff(uopt)| (VNS2.m:185): compare where the oracle's moves are not tiny
    rjnu = ref["Jnu"].reshape(5, 3, 3)[:, idx, idx]
    ok = rjnu < 1e6
    assert _rel(jnu[ok], rjnu[ok]) < 1e-5


def test_gpc_window_unsquared_and_rounded(env, built):
    """MatG/DTC window (t+dmin+1..), DTC_GPC_WW.m weighting (unsquared) and BA_MIMO's rounded
    LCM, each against the oracle built the same way."""
    from mpct.engine import eval_batch
    from mpct.scenarios import candidate_grid, shell3x3
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3 as o_shell3x3

    N2, Nu, d, l = candidate_grid(8, N2=20, Nu=4)
    for kw, okw in [(dict(window="gpc"), dict(window="gpc")),
                    (dict(weights_squared=False), dict(weights_squared=False)),
                    (dict(exact_carima=False), dict(round_roots=True))]:
        sc, r, yref = shell3x3(n2_max=20, nu_max=4, **kw)
        osc, orr, oyref, _ = o_shell3x3(**okw)
        cp = CPort(osc, 20, 500, oyref)
        res = eval_batch(sc, N2, Nu, d, l, r[None], want_traj=True)
        ref = cp.eval(N2, Nu, d, l, orr[None], want_traj=True)
        assert np.all(res.status == 0), kw
        assert _trel(res.y, ref["y"]) < TRAJ_RTOL, (kw, _trel(res.y, ref["y"]))
        assert _rel(res.J1, ref["J1"]) < COST_RTOL, kw


def test_full_grid_properties(env):
    """Full metric batch (4096 candidates): clean status, finite costs, bitwise determinism and
    independence from batch order / composition (the library dispatches the candidates in its own
    heaviest-first order, gpc_kernel.hip order_candidates; results stay in the caller's order)."""
    from mpct.engine import eval_batch
    from mpct.scenarios import candidate_grid

    N2, Nu, d, l = candidate_grid(4096)
    a = eval_batch(env["sc"], N2, Nu, d, l, env["r"][None])
    b = eval_batch(env["sc"], N2, Nu, d, l, env["r"][None])
    assert np.all(a.status == 0)
    assert np.all(np.isfinite(a.J1))
    assert np.array_equal(a.J1, b.J1)
    perm = np.random.default_rng(1).permutation(4096)
    c = eval_batch(env["sc"], N2[perm], Nu[perm], d[perm], l[perm], env["r"][None])
    assert np.array_equal(c.J1, a.J1[perm])
    # the whole batch against the C port (same stable QR / dual active-set arithmetic on the CPU)
    ref = env["cp"].eval(N2, Nu, d, l, env["r"][None], threads=16)
    rel = np.max(np.abs(a.J1 - ref["J1"]) / np.maximum(np.abs(ref["J1"]), 1e-12), axis=1)
    print("full grid J1: max rel %.2e, 99.9%% %.2e" % (rel.max(), np.quantile(rel, 0.999)))
    assert rel.max() < COST_RTOL, (int(np.argmax(rel)), rel.max())
    w = np.array([0.05, 0.40, 0.55])
    from mpct.objectives import rank
    assert np.array_equal(rank(a.J1 @ w), rank(ref["J1"] @ w))


# simulations of test_dispatch_key_mixed_horizons_and_step_refs whose status differs from the C
# port's (QP iteration caps on degenerate active sets, rounding-sensitive), per reference count
KEY_TEST_STATUS_MISMATCH = {1: [], 3: []}


def test_dispatch_key_mixed_horizons_and_step_refs(built):
    """The controller-based dispatch key (work_order.hip order_keys_gpc) runs for batches of >= 256
    candidates. Cover both of its solve paths: lanes over (output, move) when my*M <= 64, and one
    lane per output when my*M > 64 (Nu = 8: M = 24). Include bad horizons and the VNS step
    references (nref = 3). The order must not change any result: compare with the C port, and
    with the same batch reversed."""
    from mpct.engine import eval_batch
    from mpct.scenarios import shell3x3, vns_step_refs
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3 as o_shell3x3

    rng = np.random.default_rng(7)
    C = 320
    N2 = rng.integers(8, 31, size=C).astype(np.int32)
    Nu = np.minimum(rng.integers(1, 9, size=C), N2).astype(np.int32)
    N2[:4] = (0, 31, 5, 12)  # skipped, N2 > n2_max, Nu > N2, valid
    Nu[:4] = (3, 2, 7, 8)
    d = 10.0 ** rng.uniform(-3, 0, size=(C, 3))
    l = 10.0 ** rng.uniform(-4, -1, size=(C, 3))
    sc, r, yref = shell3x3(n2_max=30, nu_max=8, nit=150)
    osc, orr, oyref, _ = o_shell3x3()
    cp = CPort(osc, 30, 150, np.ascontiguousarray(oyref[:, :150]))
    mismatches = {}
    for refs, orefs in ((r[None], orr[None, :, :150]), (vns_step_refs(3, 150), vns_step_refs(3, 150))):
        res = eval_batch(sc, N2, Nu, d, l, refs)
        rev = eval_batch(sc, N2[::-1].copy(), Nu[::-1].copy(), d[::-1].copy(), l[::-1].copy(), refs)
        ref = cp.eval(N2, Nu, d, l, orefs, threads=8)
        st = res.status.reshape(C, -1)
        assert np.all(st[0] == 8) and np.all(st[1] == 16) and np.all(st[2] == 16)
        assert np.array_equal(st, rev.status.reshape(C, -1)[::-1])
        assert np.array_equal(res.J1, rev.J1.reshape(C, -1, 3)[::-1].reshape(res.J1.shape), equal_nan=True)
        # unit steps drive a few aggressive candidates into the QP iteration cap (status 1) on
        # both sides; which ones is rounding-sensitive (degenerate active sets: the Givens and the
        # Householder prologue QR agree to 3e-12 on every clean simulation here and differ by one
        # capped simulation of 960, tools/diag/qr_status_ab.py); compare the ones clean on both
        cst = np.asarray(ref["status"]).reshape(C, -1)
        ok = np.all(st == 0, axis=1) & np.all(cst == 0, axis=1)
        # pin WHICH simulations differ in status from the C port (not a fraction)
        mism = sorted(int(k) for k in np.nonzero(np.any(st != cst, axis=1))[0] if k >= 3)
        capped = sorted(int(k) for k in np.nonzero(np.any(st == 1, axis=1))[0])
        print("refs %d: status mismatches vs C port %s; capped on the device %s" % (refs.shape[0], mism, capped))
        mismatches[refs.shape[0]] = mism
        a = res.J1.reshape(C, -1)[ok]
        b = np.asarray(ref["J1"]).reshape(C, -1)[ok]
        assert _rel(a, b) < COST_RTOL, _rel(a, b)
    assert mismatches == KEY_TEST_STATUS_MISMATCH, mismatches


def test_rank_device_matches_stable_sort(built):
    """mpct_rank_device (the ranking after the cost all-gather, mpct.dist.rank_candidates on GPU
    tensors) against a stable CPU sort of the same rule.  Costs are small integers and weights powers
    of two, so every weighted sum is exact and the expected order is unambiguous. The rows include
    ties, NaN costs (last, by index), +-inf, and -0 next to +0."""
    import torch

    from mpct.dist import rank_candidates

    rng = np.random.default_rng(3)
    C = 5000
    costs = rng.integers(0, 40, size=(C, 3)).astype(float)
    costs[rng.integers(0, C, 60), rng.integers(0, 3, 60)] = np.nan
    costs[10] = (np.inf, 0.0, 0.0)
    costs[11] = (-np.inf, 0.0, 0.0)
    costs[12] = (-0.0, -0.0, -0.0)
    costs[13] = (0.0, 0.0, 0.0)
    costs[14] = costs[13]
    w = np.array([0.5, 0.25, 1.0])
    s = costs @ w
    s[np.isnan(s)] = np.inf
    expect = np.argsort(s, kind="stable")
    dev = torch.device("cuda", 0)
    got = rank_candidates(torch.from_numpy(costs).to(dev), torch.from_numpy(w).to(dev)).cpu().numpy()
    assert np.array_equal(got, expect)
    # the C = prefix form used by the padded multi-rank batch
    got2 = rank_candidates(torch.from_numpy(costs).to(dev), torch.from_numpy(w).to(dev), C=3000).cpu().numpy()
    assert np.array_equal(got2, np.argsort(s[:3000], kind="stable"))
    # both sides of the counting rank's batch limit (work_order.hip kCountRankMaxC = 8192: counting
    # rank up to it, hipCUB's radix sort above), odd sizes and one-element batches
    big = np.concatenate([costs, costs, rng.integers(0, 40, size=(6500, 3)).astype(float)])
    sb = big @ w
    sb[np.isnan(sb)] = np.inf
    tb = torch.from_numpy(big).to(dev)
    for n in (1, 2, 257, 8191, 8192, 8193, 16500):
        got = rank_candidates(tb, torch.from_numpy(w).to(dev), C=n).cpu().numpy()
        assert np.array_equal(got, np.argsort(sb[:n], kind="stable")), n


def test_status_edges(env):
    from mpct.engine import eval_batch

    sc = env["sc"]
    N2 = np.array([0, 30, 4, 31], dtype=np.int32)
    Nu = np.array([5, 5, 6, 5], dtype=np.int32)
    d = np.full((4, 3), 0.1)
    l = np.full((4, 3), 0.01)
    res = eval_batch(sc, N2, Nu, d, l, env["r"][None])
    assert res.status[0] == 8            # skipped sentinel
    assert res.status[1] == 0
    assert res.status[2] == 16           # Nu > N2
    assert res.status[3] == 16           # N2 > n2_max
    assert np.all(np.isnan(res.J1[[0, 2, 3]]))
    empty = eval_batch(sc, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 3)),
                       np.zeros((0, 3)), env["r"][None])
    assert empty.J1.shape == (0, 3)


def test_vns_search_ranges(built, has_gpu):
    """MPCTuning.m:163 (nbp=7, nbc=4): N2 up to 127 and Nu up to 15, i.e. M = 45 QP rows and
    M + nx = 80 > 64 columns in the prologue QR (multi-pass) -- against the C port."""
    if not has_gpu:
        pytest.skip("no GPU")
    from mpct.engine import eval_batch
    from mpct.scenarios import shell3x3
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3 as o_shell3x3

    sc, r, yref = shell3x3(n2_max=127, nu_max=15)
    osc, orr, oyref, _ = o_shell3x3()
    cp = CPort(osc, 127, 500, oyref)
    rng = np.random.default_rng(11)
    N2 = np.array([127, 127, 64, 16, 100, 33, 90, 127], dtype=np.int32)
    Nu = np.array([15, 2, 15, 15, 7, 12, 1, 10], dtype=np.int32)
    d = 10.0 ** rng.uniform(-3, 0, (8, 3))
    l = 10.0 ** rng.uniform(-4, -1, (8, 3))
    res = eval_batch(sc, N2, Nu, d, l, r[None], open_loop=True, want_traj=True)
    ref = cp.eval(N2, Nu, d, l, orr[None], open_loop=True, want_traj=True)
    assert np.all(res.status == 0) and np.all(ref["status"] == 0)
    assert _rel(res.J1, ref["J1"]) < COST_RTOL
    assert _trel(res.u, ref["u"]) < TRAJ_RTOL
    assert _trel(res.uopt, ref["uopt"]) < TRAJ_RTOL


def test_two_streams_share_a_scenario(env):
    """Two device calls on one scenario, enqueued back to back on two streams without a host
    sync: each launch reads its own heaviest-first permutation (work_order.hip), and the second
    call's sort waits for the first launch before rewriting the shared buffer."""
    import torch

    from mpct.engine import eval_batch, eval_batch_device
    from mpct.scenarios import candidate_grid

    sc = env["sc"]
    dev = torch.device("cuda", 0)
    N2, Nu, d, l = candidate_grid(2048)
    halves = [slice(0, 1024), slice(1024, 2048)]
    ref = [eval_batch(sc, N2[h], Nu[h], d[h], l[h], env["r"][None]) for h in halves]
    tr = torch.from_numpy(env["r"][None].copy()).to(dev)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = []
    for h in halves:
        t = [torch.from_numpy(np.ascontiguousarray(a[h])).to(dev) for a in (N2, Nu, d, l)]
        out = dict(J1=torch.empty((1024, sc.my), dtype=torch.float64, device=dev),
                   status=torch.empty(1024, dtype=torch.int32, device=dev),
                   qp_iters=torch.empty(1024, dtype=torch.int64, device=dev))
        outs.append((out, t))
    torch.cuda.synchronize(dev)  # inputs resident; then the two launches are enqueued back to back
    for (out, t), st in zip(outs, streams):
        eval_batch_device(sc, *t, tr, out, stream=st)
    torch.cuda.synchronize(dev)
    for (out, _), rf in zip(outs, ref):
        assert np.array_equal(out["J1"].cpu().numpy(), rf.J1)


@pytest.fixture(scope="module")
def metric(built, has_gpu):
    """The benchmark's own scenario: shell3x3(n2_max=30, nu_max=5) -- nu*nu_max = 15, so the
    cost-only calls launch gpc_small_kernel (the small-plant kernel bench.py times), trajectory calls
    the general gpc_closed_loop_kernel<16,false,true> instance."""
    if not has_gpu:
        pytest.skip("no GPU")
    from mpct.engine import kernel_instance
    from mpct.scenarios import shell3x3
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3 as o_shell3x3

    sc, r, yref = shell3x3(n2_max=30, nu_max=5)
    assert kernel_instance(sc) == "gpc_small_kernel"
    assert kernel_instance(sc, want_traj=True) == "gpc_closed_loop_kernel<16,false,true>"
    osc, orr, oyref, _ = o_shell3x3()
    return dict(sc=sc, r=r, osc=osc, oyref=oyref, cp=CPort(osc, 30, 500, oyref))


def test_metric_instance_full_grid(metric):
    """The exact kernel instance and workload the benchmark times (4096 candidates, N2=30, Nu=5,
    cost only) against the C port on the whole grid: J1 within COST_RTOL, identical ranking on
    the Pareto-weighted and the plain sum of costs."""
    from mpct.engine import eval_batch
    from mpct.objectives import rank
    from mpct.scenarios import candidate_grid

    N2, Nu, d, l = candidate_grid(4096)
    res = eval_batch(metric["sc"], N2, Nu, d, l, metric["r"][None])
    ref = metric["cp"].eval(N2, Nu, d, l, metric["r"][None], threads=16)
    assert np.all(res.status == 0) and np.all(ref["status"] == 0)
    rel = np.max(np.abs(res.J1 - ref["J1"]) / np.abs(ref["J1"]), axis=1)
    print("metric instance, 4096 grid: J1 max rel %.2e" % rel.max())
    assert rel.max() < COST_RTOL, (int(np.argmax(rel)), rel.max())
    w = np.array([0.05, 0.40, 0.55])  # Shell3x3.m:161
    assert np.array_equal(rank(res.J1 @ w), rank(ref["J1"] @ w))
    assert np.array_equal(rank(res.J1.sum(1)), rank(ref["J1"].sum(1)))


def test_metric_instance_numpy_oracle_sample(metric):
    """16 candidates of the metric grid through the timed instance against the independent numpy
    oracle (primal active-set QP on the least-squares form, oracle/toolbox_gpc.py): J1 within
    COST_RTOL and the same ranking."""
    from mpct.engine import eval_batch
    from mpct.objectives import rank
    from mpct.scenarios import candidate_grid
    from oracle.toolbox_gpc import closedloop_toolbox as o_cl

    N2, Nu, d, l = candidate_grid(4096)
    pick = np.r_[0, np.random.default_rng(7).choice(np.arange(1, 4096), 15, replace=False)]
    res = eval_batch(metric["sc"], N2[pick], Nu[pick], d[pick], l[pick], metric["r"][None])
    J = np.zeros((16, 3))
    for k, c in enumerate(pick):
        o = o_cl(metric["osc"], metric["r"], None, 30, 5, d[c], l[c], 500, open_loop=False)
        J[k] = ((o.y - metric["oyref"]) ** 2).sum(axis=1)
    rel = np.max(np.abs(res.J1 - J) / np.abs(J))
    print("metric instance vs numpy oracle: J1 max rel %.2e" % rel)
    assert rel < COST_RTOL
    w = np.array([0.05, 0.40, 0.55])
    assert np.array_equal(rank(res.J1 @ w), rank(J @ w))


def test_multi_device_entry_equals_single(metric):
    """mpct_eval_batch_multi, bitwise equal to mpct_eval_batch: on the box's devices, and with the
    threaded strided path exercised on one GPU by listing device 0 twice and three times (each
    occurrence is its own context, stream and host thread).  Results land in
    the caller's order whatever the split."""
    import torch

    from mpct.engine import eval_batch, eval_batch_multi
    from mpct.scenarios import candidate_grid

    N2, Nu, d, l = candidate_grid(1000)
    devs = list(range(torch.cuda.device_count()))
    a = eval_batch(metric["sc"], N2, Nu, d, l, metric["r"][None], device=0)
    for dl in (devs, [0, 0], [0, 0, 0]):
        b = eval_batch_multi(metric["sc"], dl, N2, Nu, d, l, metric["r"][None])
        assert np.array_equal(a.J1, b.J1) and np.array_equal(a.status, b.status), dl
        assert np.array_equal(a.qp_iters, b.qp_iters), dl
    # open-loop + trajectories and two reference sets through the same entry (every result array
    # is gathered and scattered, simulation s = c*nref + k)
    from mpct.scenarios import vns_step_refs

    refs = vns_step_refs(3, 500)[:2]
    c = eval_batch(metric["sc"], N2[:9], Nu[:9], d[:9], l[:9], refs, open_loop=True, want_traj=True, device=0)
    for dl in (devs, [0, 0]):
        e = eval_batch_multi(metric["sc"], dl, N2[:9], Nu[:9], d[:9], l[:9], refs, open_loop=True, want_traj=True)
        for k in ("J1", "j21", "j22", "Jnu", "status", "qp_iters", "y", "u", "ys", "uopt"):
            assert np.array_equal(getattr(c, k), getattr(e, k)), (dl, k)
