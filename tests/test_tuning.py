"""CPU: the tuning loop around the engine (mpct.tuning) -- MPCTuning's bit encoding, the VNS2
enumeration semantics (orders {1, 3}, first improvement, restarts), the batched speculative
replay (identical decisions to the sequential search), the GAM goal-attainment restatement and
the Tuning_Parameters record.  Neighbours are scored by synthetic functions or by the C port
(oracle/cgpc.c) standing in for the GPU engine."""
import math

import numpy as np
import pytest

from mpct.tuning import (TuningPar, bit_weights, bits_of, de2bi, gam_fgoalattain, save_tuning_parameters,
                         vns2, vns2_batched)


def test_bits():
    assert de2bi(5, 4) == [1, 0, 1, 0]           # least significant first (de2bi default)
    assert bits_of(5, 4) == [0, 1, 0, 1]         # flip(de2bi(.)): Xv layout (MPCTuning.m:285)
    assert bits_of(127, 7) == [1] * 7
    np.testing.assert_array_equal(bit_weights(7, 4), [64, 32, 16, 8, 4, 2, 1, 8, 4, 2, 1])
    p = TuningPar(my=3, ny=3, nbp=7, nbc=4)
    np.testing.assert_array_equal(p.N, [127, 127, 127])      # MPCTuning.m:288-289
    np.testing.assert_array_equal(p.Nu, [2, 2, 2])
    assert p.Xv2 == [[1, 1, 1, 1]] * 3                        # MPC_TFob.m:46-50 (all ones)
    assert TuningPar(my=1, ny=1, nbp=2, nbc=4).nbp == 4       # MPCTuning.m:138-140


def test_vns2_enumeration_count():
    """Never-improving search from MPCTuning's start (N = 127, Nu = [2 2 2], Xv2 = 15):
    order 1: 3 x 7 (N search repeated my times) + 3 x 4 Nu flips (each rejected flip leaves
    Nu(H) at the incumbent bits' value 15, VNS2.m:218-220); order 3: 3 x (C(7,3) - 1) N triples
    (N = 127 - 112 = 15 fails PreCon against Nu = 15) + 3 x 3 Nu triples (Nu = 1 is invalid,
    VNS2.m:135) = 144 evaluations."""
    par = TuningPar(my=3, ny=3, nbp=7, nbc=4, dmin=np.array([6, 3, 0]))
    seen = []

    def ev(N, Nu):
        seen.append((N, Nu))
        return math.inf

    N, Nu, Xv1, Xv2, Fvns, fv, n = vns2(par, ev, 1e30)
    assert n == 144 == len(seen)
    assert Fvns == 1e30
    # every N neighbour of order 1 flips one bit of 127; order 3 flips three distinct bits
    order1 = {k[0][0] for k in seen if k[1] == (2, 2, 2)}          # first pass: Nu still [2 2 2]
    order3 = {k[0][0] for k in seen if k[1] == (15, 15, 15) and k[0][0] != 127}
    assert order1 == {127 - 2 ** b for b in range(7)}
    assert order3 == {127 - (2 ** a + 2 ** b + 2 ** c)
                      for a in range(7) for b in range(a) for c in range(b)} - {15}
    # the returned horizons come from the incumbent bits (quirk: Xv2 = 15 when nothing improved)
    np.testing.assert_array_equal(N, [127] * 3)
    np.testing.assert_array_equal(Nu, [15] * 3)


def _synthetic(N, Nu):
    return (N[0] - 37) ** 2 + sum((u - 5) ** 2 for u in Nu) + 0.5 * N[0] + 0.01 * sum(Nu)


def test_vns2_batched_equals_sequential_synthetic():
    par = TuningPar(my=3, ny=3, nbp=7, nbc=4, dmin=np.array([6, 3, 0]))
    seq = vns2(par, _synthetic, 1e30)
    calls = []

    def batch(keys):
        calls.append(len(keys))
        return [_synthetic(*k) for k in keys]

    bat = vns2_batched(par, batch, 1e30)
    np.testing.assert_array_equal(seq[0], bat[0])
    np.testing.assert_array_equal(seq[1], bat[1])
    assert seq[2] == bat[2] and seq[3] == bat[3] and seq[4] == bat[4]
    assert seq[6] == bat[6]                          # same number of scored neighbours
    assert len(calls) == bat[7] and max(calls) <= 512
    assert seq[4] < 1e30                             # the synthetic search does improve


def test_vns2_first_improvement_restart():
    """Hand-traced from VNS2.m (nbp = 4, nbc = 2, one output/input, F = |N - 5| + 0.1 Nu):
    order 1 flips from index Nt = the least significant bit (VNS2.m:108) and restarts there after
    every improvement (:198-215, 233-236): 15 -> 14 (better) -> 15 x, 12 (better) -> 13 x, 14 x,
    8 (better) -> 9 x, 10 x, 12 x, 0 invalid.  The Nu search starts from Xv2 recomputed at the
    first improvement (bits of Nu = 2): (8, 3) x.  Order 3 flips bits {4, 3} statically and then
    bit 2 -> 15 x, bit 1 -> 3 (better): an improvement ends an order-3 block.  Nu has only 2 bits,
    so its order-3 block is empty.  Result N = 3, F = 2.2."""
    par = TuningPar(my=1, ny=1, nbp=4, nbc=2)
    trace = []

    def ev(N, Nu):
        trace.append((N[0], Nu[0]))
        return abs(N[0] - 5) + 0.1 * Nu[0]

    N, Nu, _, _, F, _, n = vns2(par, ev, 1e30)
    assert trace == [(14, 2), (15, 2), (12, 2), (13, 2), (14, 2), (8, 2), (9, 2), (10, 2), (12, 2),
                     (8, 3), (15, 2), (3, 2)]
    assert N[0] == 3 and Nu[0] == 2 and F == pytest.approx(2.2) and n == 12


def test_gam_goal_attainment_synthetic():
    """min gamma s.t. |J_i(x) - goal| <= w_i gamma, x >= 1e-5, forward differences with step
    DiffMinChange = 0.5 (MPCTuning.m:88-91), Jacobian = one batch of n+1 points."""
    par = TuningPar(my=2, ny=1, w=np.array([0.5, 0.5]))
    par.x0 = np.array([2.0, 2.0, 2.0])
    a = np.array([1.0, 3.0, 0.5])

    def batch_j1(X):
        X = np.atleast_2d(X)
        J0 = (X[:, 0] - a[0]) ** 2 + 0.1 * X[:, 2] ** 2 + 1e-3
        J1 = (X[:, 1] - a[1]) ** 2 + 0.1 * X[:, 2] ** 2 + 1e-3
        return np.stack([J0, J1], axis=1)

    F0 = batch_j1(par.x0)[0]
    att0 = np.max(np.abs(F0 - 1e-3) / par.w)
    x, att, Fx, nb, last = gam_fgoalattain(par, batch_j1)
    assert np.all(x >= par.lb1)
    assert att < 0.5 * att0
    assert att == pytest.approx(np.max(np.abs(Fx - 1e-3) / par.w))
    assert nb >= 2


def test_gam_function_evaluation_budget_and_memo():
    """fgoalattain's MaxFunctionEvaluations (default 100 * numel(x0); MPCTuning.m:88-91 does not
    set it) counts every evaluated point, forward differences included: the search stops after the
    iteration that reaches it.  A memo shared by two identical GAM rounds (mpc_tfob) makes the
    second one free and identical."""
    a = np.array([1.0, 3.0, 0.5])
    pts = []

    def batch_j1(X):
        X = np.atleast_2d(X)
        pts.extend(map(tuple, X))
        J0 = np.abs(X[:, 0] - a[0]) ** 1.5 + 0.1 * X[:, 2] ** 2 + np.sin(7 * X[:, 1]) ** 2
        J1 = (X[:, 1] - a[1]) ** 2 + 0.1 * X[:, 2] ** 2 + 1e-3
        return np.stack([J0, J1], axis=1)

    par = TuningPar(my=2, ny=1, w=np.array([0.5, 0.5]))
    par.x0 = np.array([2.0, 2.0, 2.0])
    x_free, *_ = gam_fgoalattain(par, batch_j1, max_iter=400, max_fun_evals=10 ** 6)
    n_free = len(set(pts))
    pts.clear()
    x, att, Fx, nb, last = gam_fgoalattain(par, batch_j1, max_iter=400, max_fun_evals=12)
    n_cap = len(set(pts) - {tuple(x)})
    assert n_free > 20 and 12 <= n_cap <= 12 + 2 * (par.my + par.ny + 1)
    assert np.all(x >= par.lb1) and att == pytest.approx(np.max(np.abs(Fx - 1e-3) / par.w))
    # default budget: 100 * numel(x0)
    pts.clear()
    gam_fgoalattain(par, batch_j1, max_iter=400)
    assert len(set(pts)) <= 300 + 2 * (par.my + par.ny + 1) + 1
    memo = {}
    r1 = gam_fgoalattain(par, batch_j1, max_iter=30, memo=memo)
    r2 = gam_fgoalattain(par, batch_j1, max_iter=30, memo=memo)
    assert r1[3] > 0 and r2[3] == 0
    for u, v in zip(r1[:3] + r1[4:], r2[:3] + r2[4:]):
        np.testing.assert_array_equal(u, v)


def test_tuning_parameters_roundtrip(tmp_path):
    from scipy.io import loadmat

    p = str(tmp_path / "Shell3x3_Tuning_test.mat")
    import datetime

    from mpct.tuning import scale_record

    save_tuning_parameters(p, [24, 24, 24], [6, 2, 2], [0.01, 0.004, 0.0008], [9e-5, 5e-4, 1.5e-3],
                           scale={"L": np.eye(3), "R": np.diag([0.5, 0.25, 0.125])},
                           date=datetime.datetime(2026, 10, 15, 12, 0, 0))
    m = loadmat(p, squeeze_me=False, struct_as_record=False)["Tuning_Parameters"][0, 0]
    assert int(m.N[0, 0]) == 24
    np.testing.assert_array_equal(m.Nu, [[6, 2, 2]])
    np.testing.assert_allclose(m.delta, [[0.01, 0.004, 0.0008]])
    sc = m.scale[0, 0]
    np.testing.assert_allclose(sc.L, np.eye(3))
    # MPCTuning.m:156-160: Ru = R(1:ny,1:ny), Rv = R(ny+1:end,...) (0x0 without MDs); the
    # resume path of Shell3x3.m:180-183 reads all four fields
    np.testing.assert_allclose(sc.Ru, np.diag([0.5, 0.25, 0.125]))
    assert sc.Rv.size == 0
    # datetime cannot be written outside MATLAB: its datenum (datenum(2026,10,15,12,0,0))
    assert float(m.date[0, 0]) == 740270.5
    # Shell 7x5: R is 5x5 over 3 MVs and 2 MDs -> Rv is the 2x2 MD block
    r5 = scale_record(np.ones(7), np.arange(1.0, 6.0), 3)
    np.testing.assert_allclose(r5["Rv"], np.diag([4.0, 5.0]))
    assert r5["Ru"].shape == (3, 3)
    j = str(tmp_path / "t.json")
    rec = save_tuning_parameters(j, [12], [4, 2, 2], [1, 1, 1], [1, 1, 1])
    assert rec["N"] == 12


def test_vns2_batched_equals_sequential_cport(built):
    """The real Shell 3x3 VNS call (MPCTuning's start, fixture-tuned weights) scored by the C port:
    the batched replay takes exactly the sequential search's decisions."""
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3, vns_step_refs

    osc, r, yref, fx = shell3x3()
    cp = CPort(osc, 127, 500, yref)
    refs = np.asarray(vns_step_refs(3, 500))
    delta, lam = np.asarray(fx["delta"]), np.asarray(fx["lambda"])
    idx = np.arange(3)

    def score(keys, threads):
        C = len(keys)
        N2 = np.array([max(k[0]) for k in keys], dtype=np.int32)
        Nu = np.array([max(k[1]) for k in keys], dtype=np.int32)
        res = cp.eval(N2, Nu, np.tile(delta, (C, 1)), np.tile(lam, (C, 1)), refs, open_loop=True,
                      threads=threads)
        j21 = res["j21"].reshape(C, 3, 3)[:, idx, idx]
        j22 = res["j22"].reshape(C, 3, 3)[:, idx, idx]
        jnu = res["Jnu"].reshape(C, 3, 3)[:, idx, idx]
        return j21.sum(1) + j22.sum(1) + N2 + jnu.sum(1)

    par = TuningPar(my=3, ny=3, nbp=7, nbc=4, dmin=np.array([6, 3, 0]))
    bat = vns2_batched(par, lambda keys: score(keys, 8), 1e30)
    cache = {}

    def seq_eval(N, Nu):
        if (N, Nu) not in cache:
            cache[(N, Nu)] = float(score([(N, Nu)], 3)[0])
        return cache[(N, Nu)]

    seq = vns2(par, seq_eval, 1e30)
    np.testing.assert_array_equal(seq[0], bat[0])
    np.testing.assert_array_equal(seq[1], bat[1])
    assert seq[4] == bat[4] and seq[6] == bat[6]
    assert seq[4] < 1e30


def _stub_eval(statuses):
    """A stand-in for mpct.engine.eval_batch (no GPU): smooth finite costs of the weights, and the
    statuses given (cycled over the simulations)."""
    from mpct.engine import EvalResult

    def ev(sc, N2, Nu, delta, lam, refs, v=None, open_loop=False, want_traj=False, device=-1, **kw):
        N2 = np.atleast_1d(N2)
        C_ = N2.size
        refs = np.asarray(refs).reshape(-1, sc.my, sc.nit)
        S = C_ * refs.shape[0]
        d = np.repeat(np.asarray(delta, float).reshape(C_, sc.my), refs.shape[0], axis=0)
        l_ = np.repeat(np.asarray(lam, float).reshape(C_, sc.nu), refs.shape[0], axis=0)
        J1 = (np.log10(d + 1e-9) + 1.0) ** 2 + l_.sum(1, keepdims=True) + 1.0
        st = np.resize(np.asarray(statuses, dtype=np.int32), S)
        ev.calls.append(dict(nref=refs.shape[0], v=v, open_loop=open_loop))
        return EvalResult(J1=J1, j21=J1 * 0.5, j22=J1 * 0.25, Jnu=np.ones((S, sc.nu)), status=st,
                          qp_iters=np.zeros(S, np.int64), nref=refs.shape[0])

    ev.calls = []
    return ev


class _Sc:
    def __init__(self, my, nu, nit=50):
        self.my, self.nu, self.nit, self.nd, self.nq = my, nu, nit, 0, 0


def test_iteration_caps_keep_finite_costs(monkeypatch):
    """only the fatal status bits (QP infeasible, non-finite, skipped, bad horizon)
    score NaN; QP_MAXITER (1), SQP_MAXITER (32) and BOUNDS (64) keep the last iterate's finite
    cost as mpcmove / nlmpcmove do (closedloop_toolbox_nmpc.m:69), so GAM's finite differences
    and goal-attainment constraints stay finite."""
    import mpct.engine
    import mpct.objectives
    from mpct.objectives import failed
    from mpct.tuning import engine_evaluators

    assert list(failed([0, 1, 2, 4, 8, 16, 32, 64, 33, 34])) == [False, False, True, True, True, True, False,
                                                                  False, False, True]
    stub = _stub_eval([32, 1, 64, 0])
    monkeypatch.setattr(mpct.engine, "eval_batch", stub)
    monkeypatch.setattr(mpct.objectives, "eval_batch", stub)
    par = TuningPar(my=2, ny=2, nbp=5, nbc=4, w=np.array([0.1, 0.5]), q0=np.ones(2), w0=np.full(2, 0.1))
    bj1, bvns = engine_evaluators(_Sc(2, 2), np.zeros((2, 50)), par)
    J = bj1(np.array([[1.0, 1.0, 0.1, 0.1], [0.5, 2.0, 0.2, 0.1]]))
    assert np.all(np.isfinite(J))
    x, attain, Fx, nb, last = gam_fgoalattain(par, bj1, max_iter=5)
    assert np.all(np.isfinite(x)) and np.isfinite(attain) and np.all(np.isfinite(Fx))
    assert np.all(np.isfinite(bvns([((31, 31), (2, 2)), ((15, 15), (3, 3))], [1, 1], [0.1, 0.1])))
    # a fatal bit on any of a candidate's simulations makes its VNS score NaN (never improves)
    stub2 = _stub_eval([0, 2])
    monkeypatch.setattr(mpct.objectives, "eval_batch", stub2)
    monkeypatch.setattr(mpct.engine, "eval_batch", stub2)
    bj1, bvns = engine_evaluators(_Sc(2, 2), np.zeros((2, 50)), par)
    F = bvns([((31, 31), (2, 2))], [1, 1], [0.1, 0.1])
    assert np.isnan(F[0])
    J = bj1(np.array([[1.0, 1.0, 0.1, 0.1], [0.5, 2.0, 0.2, 0.1]]))
    assert np.isfinite(J[0]).all() and np.isnan(J[1]).all()


def test_nonsquare_vns_and_mdv(monkeypatch):
    """VNS2.m:166-169: a non-square plant is simulated ONCE per neighbour with Xsp (every output
    stepped at inK, VNS2.m:58-61), j21/j22 over its my outputs and Jnu over its nu MVs, F =
    sum(j21 + j22) + N(1) + sum(Jnu); Par.mdv reaches every simulation (VNS2.m:153,168,
    GAM_fun.m:81)."""
    import mpct.engine
    import mpct.objectives
    from mpct.objectives import vns_objective
    from mpct.tuning import engine_evaluators

    stub = _stub_eval([0])
    monkeypatch.setattr(mpct.objectives, "eval_batch", stub)
    monkeypatch.setattr(mpct.engine, "eval_batch", stub)
    sc = _Sc(7, 3, nit=40)
    mdv = np.ones((2, 40))
    d = np.full((2, 7), 0.0)
    l_ = np.full((2, 3), 0.1)
    F, j21, j22, jnu, res = vns_objective(sc, [27, 16], [2, 3], d, l_, mdv=mdv)
    c = stub.calls[-1]
    assert c["nref"] == 1 and c["open_loop"] and c["v"].shape == (1, 2, 40)
    assert j21.shape == (2, 7) and jnu.shape == (2, 3)
    np.testing.assert_allclose(F, j21.sum(1) + j22.sum(1) + np.array([27, 16]) + jnu.sum(1))
    from mpct.objectives import vns_refs_nonsquare

    R = vns_refs_nonsquare(7, 40)
    assert R.shape == (1, 7, 40) and np.all(R[0, :, 9:] == 1) and np.all(R[0, :, :9] == 0)
    # square plants: one simulation per output, MDs to each
    sq = _Sc(2, 2, nit=40)
    vns_objective(sq, [10], [2], np.ones((1, 2)), np.ones((1, 2)), mdv=np.ones((1, 40)))
    assert stub.calls[-1]["nref"] == 2 and stub.calls[-1]["v"].shape == (1, 1, 40)
    par = TuningPar(my=7, ny=3, nbp=7, nbc=4, w=np.ones(7), q0=np.zeros(7), w0=np.full(3, 0.1))
    bj1, bvns = engine_evaluators(sc, np.zeros((7, 40)), par, mdv=mdv)
    bj1(np.ones((1, 10)))
    assert stub.calls[-1]["v"].shape == (1, 2, 40) and not stub.calls[-1]["open_loop"]
    bvns([((27,) * 7, (2, 2, 2))], np.zeros(7), [0.1] * 3)
    assert stub.calls[-1]["nref"] == 1 and stub.calls[-1]["v"] is not None


def test_fgam_is_the_last_evaluated_j1():
    """MPC_TFob.m:104 computes Fgam = round(sum(F), 2) from the global F that GAM_fun.m:114 set
    on its LAST call -- fgoalattain's last evaluated point (a forward-difference point when the
    search stops after a gradient), not the returned XOt.  gam_fgoalattain reports that J1 in
    evaluation order (a Jacobian batch is x, then x + h_k e_k), and mpc_tfob's stop test uses it."""
    from mpct.tuning import mpc_tfob

    a = np.array([1.0, 3.0, 0.5])

    def make():
        calls = []

        def batch_j1(X):
            X = np.atleast_2d(X)
            calls.append(X.copy())
            J0 = (X[:, 0] - a[0]) ** 2 + 0.1 * X[:, 2] ** 2 + 1e-3
            J1 = (X[:, 1] - a[1]) ** 2 + 0.1 * X[:, 2] ** 2 + 1e-3
            return np.stack([J0, J1], axis=1)
        return batch_j1, calls

    par = TuningPar(my=2, ny=1, w=np.array([0.5, 0.5]))
    par.x0 = np.array([2.0, 2.0, 2.0])
    bj, calls = make()
    x, att, Fx, nb, last = gam_fgoalattain(par, bj, max_iter=20, speculate=False)
    np.testing.assert_array_equal(last, bj(calls[-1][-1:])[0])    # the last row of the last batch
    assert not np.array_equal(last, Fx)                              # here: not the returned point
    # speculation (each trial point scored with its forward-difference points) changes neither
    # the iterates nor the last requested evaluation, and needs fewer engine calls
    bj2, calls2 = make()
    x2, att2, Fx2, nb2, last2 = gam_fgoalattain(par, bj2, max_iter=20, speculate=True)
    np.testing.assert_array_equal(x2, x)
    np.testing.assert_allclose(last2, last, rtol=1e-9)   # points matched to 13 digits (stub rounding too)
    assert nb2 < nb
    # mpc_tfob: Fgam of each GAM round from that last evaluation (logged), VNS stub never improves
    logs = []
    for mode in ("last_eval", "returned"):
        p2 = TuningPar(my=2, ny=1, nbp=3, nbc=2, w=np.array([0.5, 0.5]))
        p2.x0 = np.array([2.0, 2.0, 2.0])
        bj, calls = make()
        out = []
        mpc_tfob(p2, bj, lambda keys, d, l: [math.inf] * len(keys), log=out.append, gam_max_iter=20,
                 fgam_from=mode)
        logs.append(float(out[0].split(";")[0].split("=")[1]))
    assert logs[0] == round(float(np.sum(last)), 2) and logs[1] == round(float(np.sum(Fx)), 2)


def test_vns_stale_rows_semantics():
    """VNS2.m:148-165 square plants: row i of Xy/Xu/Xyma/Xuma is copied from simulation i only
    when it succeeds; a failed simulation leaves the row of the last successful evaluation, so F
    mixes neighbours.  Rows never assigned are MATLAB's zero fill (T_i0 = sum Yref_i^2 from inK);
    while fewer than my rows exist, VNS2.m:173 throws (here NaN, never taken)."""
    from mpct.tuning import StaleRows, stale_rows_for

    s = StaleRows([10.0, 20.0, 30.0])
    assert math.isnan(s.score(5, [1, 2, 3], [True, True, False]))     # row 3 never assigned: throws
    assert s.score(5, [4, 5, 6], [True, False, True]) == 4 + 2 + 6 + 5  # row 2 stale (from the 1st)
    assert s.score(7, [7, 8, 9], [False, False, False]) == 4 + 2 + 6 + 7
    s.reset()
    assert s.score(5, [1, 2, 3], [False, True, True]) == 10 + 2 + 3 + 5  # row 1: zero fill
    Y = np.zeros((2, 20))
    Y[0, 9:] = 1.0
    Y[1, 5:] = 2.0
    np.testing.assert_allclose(stale_rows_for(Y).init, [11.0, 4.0 * 11])


def test_vns_stale_rows_one_row_broadcasts():
    """with only row 1 of Xy assigned, VNS2.m:173 Xy - Yref broadcasts (implicit
    expansion) and F is finite: the row-1 simulation's broadcast term (lazy, evaluated once) plus
    N(1), kept while later neighbours' row-1 simulations fail; with 1 < rows < my it throws."""
    from mpct.tuning import StaleRows

    calls = []

    def bc(v):
        def f():
            calls.append(v)
            return v
        return f

    s = StaleRows([10.0, 20.0, 30.0])
    assert s.score(5, [1, 2, 3], [True, False, False], bc(100.0)) == 105.0
    assert s.score(6, [4, 5, 6], [False, False, False], bc(7.0)) == 106.0   # row 1 stale: its term
    assert s.score(6, [4, 5, 6], [True, False, False], bc(200.0)) == 206.0  # row 1 replaced
    assert calls == [100.0, 200.0]
    assert math.isnan(s.score(6, [4, 5, 6], [False, True, False], bc(1.0)))  # two rows: throws
    assert s.score(6, [4, 5, 6], [False, False, True], bc(1.0)) == 4 + 5 + 6 + 6
    s.reset()
    assert math.isnan(s.score(5, [1, 2, 3], [True, False, False]))  # no broadcast term given


def test_vns2_batched_stale_rows_equals_sequential():
    """The speculative batched VNS with stale-row scoring takes the sequential search's decisions:
    a synthetic square plant where some neighbours' simulations fail."""
    from mpct.tuning import StaleRows

    par = TuningPar(my=3, ny=3, nbp=7, nbc=4, dmin=np.array([6, 3, 0]))

    def rows(N, Nu):
        T = np.array([(N[0] - 37) ** 2 / 3.0 + (u - 5) ** 2 + 0.01 * u for u in Nu])
        ok = np.array([(N[0] * 7 + 3 * i + Nu[i]) % 5 != 0 for i in range(3)])
        return T, ok

    seq_state = StaleRows([50.0, 60.0, 70.0])

    def seq_eval(N, Nu):
        T, ok = rows(N, Nu)
        return seq_state.score(N[0], T, ok)

    seq = vns2(par, seq_eval, 1e30)
    bat = vns2_batched(par, lambda keys: [rows(*k) for k in keys], 1e30, stale=StaleRows([50.0, 60.0, 70.0]))
    np.testing.assert_array_equal(seq[0], bat[0])
    np.testing.assert_array_equal(seq[1], bat[1])
    assert seq[4] == bat[4] and seq[6] == bat[6] and seq[4] < 1e30
