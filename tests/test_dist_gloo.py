"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py — strided
candidate shards (rank r scores r, r + W, ...) with sentinel padding, one all-gather of the per-candidate cost records, and an
identical ranking on every rank that equals the single-process ranking.  Per-candidate costs come
from the C port (oracle/cgpc.c) here, standing in for the kernel, which needs a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _costs(N2, Nu, d, l):
    """Cost records [n, my] for a shard; sentinel candidates (N2 == 0) -> NaN like the kernel."""
    from oracle.cport import CPort
    from oracle.scenarios import shell3x3

    osc, r, yref, _ = shell3x3()
    out = np.full((len(N2), 3), np.nan)
    ok = N2 > 0
    if ok.any():
        res = CPort(osc, 30, 500, yref).eval(N2[ok], Nu[ok], d[ok], l[ok], r[None], threads=1)
        out[ok] = res["J1"]
    return out


def _worker(rank, world, port, C, q, keyed=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpct.dist import gather_costs, pad_shard, rank_candidates, shard_indices, shard_indices_keyed
        from mpct.scenarios import candidate_grid

        N2, Nu, d, l = candidate_grid(C)
        owners = None
        if keyed:   # any work key: the weight ratio stands in for config 3's latency estimate
            w = d.max(1) / l.min(1)
            owners = [shard_indices_keyed(w, world, k) for k in range(world)]
        sN2, sNu, sd, sl = pad_shard(N2, Nu, d, l, owners[rank] if keyed else shard_indices(C, world, rank))
        local = torch.from_numpy(_costs(sN2, sNu, sd, sl))
        g = gather_costs(local, owners=owners)
        w = torch.tensor([0.05, 0.40, 0.55], dtype=torch.float64)
        order = rank_candidates(g, w, C)
        q.put((rank, g.numpy(), order.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("C,keyed", [(12, False), (11, False), (11, True)])
def test_two_rank_gather_and_rank(built, C, keyed):
    from mpct.scenarios import candidate_grid

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, C, q, keyed)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort(key=lambda t: t[0])
    N2, Nu, d, l = candidate_grid(C)
    ref = _costs(N2, Nu, d, l)
    w = np.array([0.05, 0.40, 0.55])
    ref_order = np.argsort(ref @ w, kind="stable")
    per = -(-C // world)
    for rank, g, order in got:
        assert g.shape == (world * per, 3)
        np.testing.assert_array_equal(g[:C], ref)              # bit-identical gathered records
        assert np.all(np.isnan(g[C:]))                         # sentinel padding
        np.testing.assert_array_equal(order, ref_order)        # identical ranking on every rank
    np.testing.assert_array_equal(got[0][2], got[1][2])


def test_shard_indices_cover_grid_and_match_library(built):
    """The ranks' strided split (mpct.dist.shard_indices) covers every candidate exactly once, pads
    fewer than W sentinels, and equals the library's split of mpct_eval_batch_multi
    (mpct_shard_candidates) on the real candidates."""
    from mpct.dist import shard_indices
    from mpct.engine import shard_candidates

    for C in (1, 7, 4096, 65536):
        for W in (1, 2, 3, 8):
            parts = [shard_indices(C, W, r) for r in range(W)]
            allc = np.sort(np.concatenate(parts))
            np.testing.assert_array_equal(allc[:C], np.arange(C))
            assert allc.size - C < W and np.all(allc[C:] >= C)
            for r in range(W):
                np.testing.assert_array_equal(shard_candidates(C, W, r), parts[r][parts[r] < C])


def test_config3_plans_against_the_cell_table():
    """Config 3's grid is cell-ordered (1024 lambda draws per (N2, Nu) cell, N2-major).  Against the
    committed one-GPU time of every cell (mpct/config3_cells.json, tools/shard_balance.py --cells;
    VERDICT r5 item 1: a measured table, not a work model): the contiguous split of round 2 gives
    rank r of 8 one N2 and a predicted max/mean far from 1; the cell plan (plan_cells_lpt) gives
    every rank whole cells, covers the grid exactly once, pads with distinct sentinels and balances
    the predicted shard times; the strided split hands every rank 1/W of every cell (the split of
    the other workloads)."""
    from mpct.dist import SHARD_OVERLAP, load_cell_table, plan_cells_lpt, shard_indices
    from mpct.scenarios import CONFIG3_N2, CONFIG3_NU, config3_grid

    table = load_cell_table()
    assert set(table) == {(n, u) for n in CONFIG3_N2 for u in CONFIG3_NU}
    assert all(t["ms"] > 0 and len(t["half_ms"]) == 2 and t["n"] == 1024 for t in table.values())
    N2, Nu, D, L = config3_grid(1024)
    C = N2.size

    def pred(idx):  # the packing model: heaviest cell + SHARD_OVERLAP x the rest (pro rata)
        idx = idx[idx < C]
        ts = sorted((table[k]["ms"] * np.count_nonzero((N2[idx] == k[0]) & (Nu[idx] == k[1])) / 1024
                     for k in set(zip(N2[idx].tolist(), Nu[idx].tolist()))), reverse=True)
        return ts[0] + SHARD_OVERLAP * sum(ts[1:])

    for W in (2, 4, 8):
        owners, loads = plan_cells_lpt(N2, Nu, L, W)
        allc = np.concatenate(owners)
        assert len({o.size for o in owners}) == 1                     # equal sizes for the all-gather
        np.testing.assert_array_equal(np.sort(allc[allc < C]), np.arange(C))
        assert np.unique(allc).size == allc.size                       # distinct sentinels
        for o, ld in zip(owners, loads):
            live = o[o < C]
            cells = set(zip(N2[live].tolist(), Nu[live].tolist()))
            assert live.size == 1024 * len(cells)                      # whole cells only
            assert abs(pred(o) - ld) < 1e-6 * ld
        assert max(loads) / np.mean(loads) < 1.06
        contiguous = [pred(np.arange(r * C // W, (r + 1) * C // W)) for r in range(W)]
        assert max(contiguous) / np.mean(contiguous) > 1.1
        assert max(loads) < max(contiguous)
        for r in range(W):
            sh = shard_indices(C, W, r)
            assert all(np.count_nonzero((N2[sh] == n) & (Nu[sh] == u)) == 1024 // W for (n, u) in table)


# ---- bench.py's config-3 and config-4 multi-rank logic: mpct.dist.plan_shards
# (keyed owners for config 3, strided otherwise), worst_over_draws (config 4's plant-mismatch draws
# co-located on the candidate's rank) and gather_and_rank, with C-restatement costs standing in
def _c3_subgrid():
    """Nine light config-3 grid candidates (N2 <= 24, Nu <= 2: the C port scores them in ms) with
    the measured disturbances of Shell7x5.m."""
    from mpct.scenarios import config3_grid

    N2, Nu, D, L = config3_grid(1024)
    pick = np.nonzero((N2 <= 24) & (Nu <= 2))[0][::997][:9]
    return N2[pick], Nu[pick], D[pick], L[pick]


def _c3_costs(N2, Nu, d, l):
    """per-output J1 of config-3 candidates by oracle/cband.c with the measured disturbance v; NaN
    rows for sentinels (N2 == 0), like the kernel's status-8 records"""
    from oracle.cband import CBand
    from oracle.scenarios import shell7x5

    osc, r, v, yref, fx = shell7x5()
    out = np.full((len(N2), 7), np.nan)
    ok = N2 > 0
    if ok.any():
        out[ok] = CBand(osc, 200, yref).eval(N2[ok], Nu[ok], d[ok], l[ok], r[None], v[None], threads=1)["J1"]
    return out


C4_DRAWS = 3


def _c4_grid():
    from mpct.dtc import config4_candidates

    N2, Nu, d, l = config4_candidates(40)
    pick = np.nonzero((N2 <= 10) & (Nu <= 3))[0][:5]
    return N2[pick], Nu[pick], d[pick], l[pick]


def _c4_costs(N2, Nu, d, l):
    """[n * draws, 2] simulation records s = c*draws + k: J1 of oracle/dtcgpc.py dtc_gpc_ww
    (DTC_GPC_WW.m's loop) with Monte-Carlo plant draw k; NaN for sentinels"""
    from oracle.dtcgpc import dtc_gpc_ww, woodberry_mc_draws

    plants = woodberry_mc_draws(C4_DRAWS)
    out = np.full((len(N2) * C4_DRAWS, 2), np.nan)
    for c in range(len(N2)):
        if N2[c] <= 0:
            continue
        for k in range(C4_DRAWS):
            p, m = int(N2[c]), int(Nu[c])
            o = dtc_gpc_ww(p=(p, p), m=(m, m), lam=tuple(l[c]), delta=tuple(d[c]), plant=plants[k])
            out[c * C4_DRAWS + k] = ((o["y"] - o["r"]) ** 2).sum(1)
    return out


def _cfg_worker(rank, world, port, cfg, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpct.dist import gather_and_rank, pad_shard, plan_shards
        from mpct.scenarios import SHELL7_W

        if cfg == "shell7x5":
            N2, Nu, d, l = _c3_subgrid()
            costs, nref, w = _c3_costs, 1, SHELL7_W
        else:
            N2, Nu, d, l = _c4_grid()
            costs, nref, w = _c4_costs, C4_DRAWS, np.ones(2)
        idx, owners = plan_shards(N2, Nu, l, world, rank, keyed="cells" if cfg == "shell7x5" else False)
        sN2, sNu, sd, sl = pad_shard(N2, Nu, d, l, idx)
        J = torch.from_numpy(costs(sN2, sNu, sd, sl))
        g, order = gather_and_rank(J, idx.size, nref, torch.tensor(w, dtype=torch.float64), len(N2), owners=owners)
        q.put((rank, idx, None if owners is None else [o.tolist() for o in owners], g.numpy(), order.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", ["shell7x5", "dtc-mc"])
def test_two_rank_bench_workloads(built, cfg):
    """bench.py's multi-rank paths of configs 3 and 4 at world size 2 over gloo: config 3's cell-plan
    owners (plan_cells_lpt over the committed cell table: whole cells per rank, unequal live counts
    padded with sentinels; measured disturbances in every simulation) and config 4's draws
    co-located on their candidate's rank with the worst case over draws.  Every rank holds
    bit-identical gathered records equal to the single-process costs, NaN sentinel padding, and the
    same ranking as a single process."""
    from mpct.dist import plan_cells_lpt
    from mpct.scenarios import SHELL7_W

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cfg_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort(key=lambda t: t[0])
    if cfg == "shell7x5":
        N2, Nu, d, l = _c3_subgrid()
        ref, w = _c3_costs(N2, Nu, d, l), SHELL7_W
        owners, _ = plan_cells_lpt(N2, Nu, l, world)
        for rank, idx, own, g, order in got:
            np.testing.assert_array_equal(idx, owners[rank])
            assert own == [o.tolist() for o in owners]
        # not the strided split (it is the point of the test)
        assert not np.array_equal(owners[0][owners[0] < len(N2)], np.arange(0, len(N2), 2))
    else:
        N2, Nu, d, l = _c4_grid()
        sims = _c4_costs(N2, Nu, d, l).reshape(len(N2), C4_DRAWS, 2)
        ref, w = sims.max(axis=1), np.ones(2)
        assert np.all(sims.max(axis=1) > sims.min(axis=1))   # the draws differ: amax selects
    C = len(N2)
    per = got[0][1].size  # the shards' common (padded) size
    ref_order = np.argsort(ref @ w, kind="stable")
    for rank, idx, own, g, order in got:
        assert g.shape == (world * per, ref.shape[1])
        np.testing.assert_array_equal(g[:C], ref)          # bit-identical gathered records
        assert np.all(np.isnan(g[C:]))                     # sentinel padding
        np.testing.assert_array_equal(order, ref_order)    # identical ranking on every rank
    np.testing.assert_array_equal(got[0][4], got[1][4])
