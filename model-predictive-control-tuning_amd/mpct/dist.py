"""Candidate-level data parallelism: one process per GPU, strided candidate shards,
one all-gather of the per-candidate cost records, identical ranking on every rank.

Rank r of W scores candidates r, r+W, r+2W, ... (the split of mpct_eval_batch_multi /
mpct_shard_candidates).  The tuning grids are built cell by cell (config 3: all 1024 lambda draws
of one (N2, Nu) pair together, N2-major), so a contiguous split hands rank r one horizon and the
heaviest rank sets the time; the strided split gives every rank the same mix of cells.

Nothing is exchanged during a simulation (VNS2.m:148-169 and GAM_fun.m:79-91 evaluate every
candidate in isolation), so the only collective is the final all-gather.  The functions here are
backend-agnostic (torch.distributed with "nccl" = RCCL on the GPU box, "gloo" in the CPU tests).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

SKIPPED_N2 = 0  # sentinel candidate: the kernel returns status MPCT_ST_SKIPPED (8) and NaN costs


def shard_indices(C: int, world: int, rank: int) -> np.ndarray:
    """Candidates of rank's strided shard of a C-candidate grid padded to a multiple of world:
    rank, rank + world, ... (ceil(C / world) of them); indices >= C are sentinel padding."""
    per = -(-C // world)
    return rank + world * np.arange(per, dtype=np.int64)


def band_work_estimate(N2, Nu, lam, nu=3):
    """A-priori latency estimate of one band-mode simulation (config 3, mdband_kernel.hip): the
    per-step output-row scan and QP grow with N2 and the QP size 3 Nu + 1, and smaller move weights
    bind the bands more often.  Fitted on the config-3 grid's measured GI iterations and DESIGN §7's
    flop model (log-linear, Spearman 0.98 over the grid, 0.49 within an (N2, Nu) cell):
    N2^0.77 (nu Nu + 1)^2.07 prod(lambda)^-0.099."""
    N2 = np.asarray(N2, dtype=float)
    M1 = nu * np.asarray(Nu, dtype=float) + 1.0
    lg = np.log10(np.maximum(np.abs(np.asarray(lam, dtype=float)), 1e-300)).reshape(N2.size, -1).sum(1)
    return N2 ** 0.769 * M1 ** 2.067 * 10.0 ** (-0.0988 * lg)


def shard_indices_keyed(work, world: int, rank: int, heavy_first: bool = False) -> np.ndarray:
    """Work-keyed split: candidates sorted by descending estimated work, dealt to the ranks in snake
    order (0..W-1, W-1..0, ...), so every rank gets one candidate of every work level and the heavy
    tail is spread evenly; each rank's candidates in ascending index order, or with heavy_first in
    descending estimated work (the band kernel dispatches in input order).  Pads like
    shard_indices (indices >= C are sentinels, dealt last)."""
    C = len(work)
    per = -(-C // world)
    order = np.concatenate([np.argsort(-np.asarray(work, dtype=float), kind="stable"),
                            np.arange(C, per * world)])
    pos = np.arange(per * world)
    rnd, j = pos // world, pos % world
    owner = np.where(rnd % 2 == 0, j, world - 1 - j)
    mine = order[owner == rank]
    return mine if heavy_first else np.sort(mine)


def pad_shard(N2, Nu, delta, lam, idx):
    """The candidate arrays at ``idx`` (shard_indices), padding indices >= C with skipped
    sentinels (N2 = 0: status 8, NaN costs)."""
    C = len(N2)
    idx = np.asarray(idx, dtype=np.int64)
    live = idx < C
    n = idx.size
    my, nu = delta.shape[1], lam.shape[1]
    oN2 = np.full(n, SKIPPED_N2, dtype=np.int32)
    oNu = np.ones(n, dtype=np.int32)
    od = np.ones((n, my))
    ol = np.ones((n, nu))
    oN2[live], oNu[live] = N2[idx[live]], Nu[idx[live]]
    od[live], ol[live] = delta[idx[live]], lam[idx[live]]
    return oN2, oNu, od, ol


def gather_costs(local: torch.Tensor, group=None, owners=None) -> torch.Tensor:
    """All-gather equal-size per-rank cost records [n, K] -> [world * n, K] in candidate order.
    Strided shards (owners None): the gathered block is rank-major, row j of rank r is candidate
    r + j*world, so one transpose of the (world, n) leading axes restores the grid's order.  Other
    splits: owners[r] = rank r's candidate indices (shard_indices_keyed, identical on every rank);
    the rows are scattered to them (sentinel indices >= C land past the end)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = local.shape[0]
    out = torch.empty((world * n,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    if owners is None:
        return out.view((world, n) + tuple(local.shape[1:])).transpose(0, 1).reshape((world * n,) + tuple(local.shape[1:]))
    idx = torch.as_tensor(np.concatenate(owners), dtype=torch.int64, device=local.device)
    res = torch.empty_like(out)
    res[idx] = out
    return res


def rank_candidates(costs: torch.Tensor, weights: torch.Tensor, C: int | None = None) -> torch.Tensor:
    """Candidate order by ascending weighted cost (Shell3x3.m:161 Pareto weights), ties by
    candidate index; NaN costs (failed / sentinel candidates) sort last.  Identical on every
    rank because every rank sorts the same gathered tensor.  GPU tensors go through the
    library's mpct_rank_device (one key kernel + a stable device radix sort on the current
    stream); CPU tensors (the gloo tests) through torch."""
    if C is not None:
        costs = costs[:C]
    if costs.is_cuda:
        from . import _lib

        c = costs.to(torch.float64).contiguous()
        w = weights.to(device=c.device, dtype=torch.float64).contiguous()
        perm = torch.empty(c.shape[0], dtype=torch.int32, device=c.device)
        stream = torch.cuda.current_stream(c.device).cuda_stream
        rc = _lib.load().mpct_rank_device(c.data_ptr(), c.shape[0], c.shape[1], w.data_ptr(), perm.data_ptr(),
                                          stream)
        if rc != 0:
            raise RuntimeError("mpct_rank_device failed (%d): %s" % (rc, _lib.load().mpct_last_error().decode()))
        return perm.to(torch.int64)
    s = costs @ weights
    s = torch.where(torch.isnan(s), torch.full_like(s, float("inf")), s)
    return torch.argsort(s, stable=True)


# measured one-GPU time of every config-3 cell alone (tools/shard_balance.py --cells): the (N2, Nu)
# cells of mpct.scenarios.config3_grid with 1024 lambda draws each, whole and in two halves
CELL_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config3_cells.json")


def load_cell_table(path: str = CELL_TABLE) -> dict:
    """{(N2, Nu): {"ms": whole cell, "half_ms": [half 0, half 1], "n": draws}} from the committed
    table (tools/shard_balance.py --cells writes it)."""
    with open(path) as f:
        tj = json.load(f)
    return {(int(c["N2"]), int(c["Nu"])): dict(ms=float(c["ms"]), half_ms=[float(x) for x in c["half_ms"]],
                                               n=int(c["n"])) for c in tj["cells"]}


def cell_halves(idx, work):
    """The two halves of one cell's candidates `idx` (ascending): sorted by descending estimated
    work (ties by index) and dealt alternately, so both halves get the same share of the heavy draws."""
    order = np.asarray(idx)[np.argsort(-np.asarray(work, dtype=float), kind="stable")]
    return np.sort(order[0::2]), np.sort(order[1::2])


# overlap of a shard's cells on one GPU: the cells' class launches run side by side and their
# alone-times are mostly latency, not occupancy, so a shard takes about its heaviest cell plus a
# fraction of the others.  Least squares over the 48 shards of six measured plans
# (profiles/r06b_shard_plans.json): 0.873 x heaviest + 0.470 x the rest (rms 12 ms), i.e. the rest
# at 0.54 of the heaviest's weight
SHARD_OVERLAP = 0.54
# cells costlier than this are split into their two halves before packing (None: an even share,
# total / world).  Splitting measured no better: a half's alone-time is most of its cell's (the
# heaviest cell 129 ms whole, 119 + 93 ms as halves; mpct/config3_cells.json, profiles/r06a_shard_balance.json), so halves add load
SPLIT_MS = None


def plan_cells_lpt(N2, Nu, lam, world: int, table: dict | None = None, nu: int = 3, split_ms: float | None = SPLIT_MS,
                   beta: float = SHARD_OVERLAP):
    """Config 3's split from measured cell times.  The candidates are grouped
    into their (N2, Nu) cells, every cell costed by the committed table (a partial cell pro rata by
    its count; a cell the table lacks by band_work_estimate, scaled by the table's median ms per
    estimate unit).  A cell costlier than split_ms (None: an even share, total / world) is split
    into two halves (cell_halves; their own measured times for a whole table cell).  Then greedy
    longest-processing-time packing under the shard model of SHARD_OVERLAP: a shard's predicted
    time is its heaviest unit plus beta times the rest (beta = 1: plain LPT on sums); units by
    descending time (ties by cell), each to the rank whose prediction it raises least (ties by
    rank).  Every rank scores few cells, so its class launches stay full, and the predicted times
    balance.  Deterministic: every rank derives the same owners.

    Returns (owners, loads): owners[r] = rank r's candidate indices, ascending, padded to one size
    with distinct sentinel indices >= C (gather_costs scatters them past the grid); loads[r] = the
    predicted ms of rank r."""
    N2 = np.asarray(N2)
    Nu = np.asarray(Nu)
    C = N2.size
    table = load_cell_table() if table is None else table
    work = band_work_estimate(N2, Nu, lam, nu)
    keys = sorted(set(zip(N2.tolist(), Nu.tolist())))
    groups = {k: np.nonzero((N2 == k[0]) & (Nu == k[1]))[0] for k in keys}
    scale = float(np.median([t["ms"] / np.sum(band_work_estimate(np.full(t["n"], k[0]), np.full(t["n"], k[1]),
                                                                   np.ones((t["n"], nu)), nu))
                             for k, t in table.items()])) if table else 1.0
    cost = {}
    for k, idx in groups.items():
        t = table.get(k)
        cost[k] = t["ms"] * idx.size / t["n"] if t else scale * float(np.sum(work[idx]))
    lim = sum(cost.values()) / world if split_ms is None else split_ms
    units = []  # (ms, cell rank for ties, half, indices)
    for ci, k in enumerate(keys):
        idx = groups[k]
        t = table.get(k)
        if cost[k] > lim and idx.size >= 2:
            halves = cell_halves(idx, work[idx])
            for h, part in enumerate(halves):
                ms = t["half_ms"][h] * 2 * part.size / t["n"] if t else cost[k] * part.size / idx.size
                units.append((ms, ci, h, part))
        else:
            units.append((cost[k], ci, 0, idx))
    units.sort(key=lambda u: (-u[0], u[1], u[2]))
    top = [0.0] * world   # heaviest unit of each rank
    rest = [0.0] * world  # the sum of its others
    mine = [[] for _ in range(world)]
    for ms, _, _, idx in units:
        new = [max(top[r], ms) + beta * (rest[r] + min(top[r], ms)) for r in range(world)]
        r = int(np.argmin(new))
        rest[r] += min(top[r], ms)
        top[r] = max(top[r], ms)
        mine[r].append(idx)
    loads = [top[r] + beta * rest[r] for r in range(world)]
    owners = [np.sort(np.concatenate(m)) if m else np.zeros(0, np.int64) for m in mine]
    n = max(o.size for o in owners)
    nxt = C
    for r in range(world):
        pad = n - owners[r].size
        owners[r] = np.concatenate([owners[r], np.arange(nxt, nxt + pad)]).astype(np.int64)
        nxt += pad
    return owners, loads


def plan_shards(N2, Nu, lam, world: int, rank: int, keyed: bool | str = False, nu: int = 3):
    """The candidates rank scores and the owners table gather_costs needs: strided shards (owners
    None); keyed="cells" (config 3, bench.py): plan_cells_lpt over the committed cell-time table;
    keyed=True: round 3's snake deal of shard_indices_keyed by band_work_estimate (kept for the
    shard-balance comparison: measured slower).  The owners are identical on every
    rank, so the gathered rows land in the grid's order.  Returns (idx, owners)."""
    if keyed == "cells":
        owners, _ = plan_cells_lpt(N2, Nu, lam, world, nu=nu)
        return owners[rank], owners
    if keyed:
        work = band_work_estimate(N2, Nu, lam, nu)
        owners = [shard_indices_keyed(work, world, k) for k in range(world)]
        return owners[rank], owners
    return shard_indices(len(N2), world, rank), None


def worst_over_draws(J: torch.Tensor, n: int, nref: int) -> torch.Tensor:
    """Per-candidate cost of a Monte-Carlo batch (config 4): the plant-mismatch draws of one
    candidate ride the reference dimension (simulation s = c*nref + k, DTC_GPC_WW.m:18-19 with one
    mismatched plant per draw) and so sit on the candidate's rank; its record is the worst case over
    them, per output.  A failed or sentinel draw (NaN) makes the candidate's record NaN."""
    if nref == 1:
        return J
    return J.view(n, nref, J.shape[-1]).amax(dim=1)


def gather_and_rank(J: torch.Tensor, n: int, nref: int, weights: torch.Tensor, C: int, owners=None,
                    distributed: bool = True):
    """The data-parallel epilogue of one scoring step: the rank's simulation records J [n*nref, K]
    -> per-candidate records (worst_over_draws) -> one all-gather (gather_costs, owners as
    plan_shards returns them) -> the ranking every rank computes (rank_candidates) over the C real
    candidates.  Returns (gathered records [>= C, K], order [C])."""
    local = worst_over_draws(J, n, nref)
    costs = gather_costs(local, owners=owners) if distributed else local
    return costs, rank_candidates(costs, weights, C)
