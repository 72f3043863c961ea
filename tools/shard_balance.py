"""Per-shard time of the 8-rank splits on one GPU: for config 3 (the 65,536
Shell 7x5 grid, cell-ordered) and config 4 (10,000 WoodBerry DTC candidates x 32 draws), each of
the 8 shards of the contiguous (round 2), strided (mpct.dist.shard_indices) and, for config 3,
work-keyed (mpct.dist.shard_indices_keyed, candidates in index order or heaviest first) splits is
scored alone on cuda:0 and timed with HIP events (median of 3); max/mean shard time predicts the
8-GPU efficiency loss from imbalance.

--cells: first time every config-3 (N2, Nu) cell alone, whole and as its two
halves (mpct.dist.cell_halves), write the table (--table-out, the committed
mpct/config3_cells.json that mpct.dist.plan_cells_lpt reads), then time the shards of the LPT plan
built from that table beside the contiguous and keyed splits, in the same call.
Usage: python tools/shard_balance.py [--out FILE] [--only shell7x5] [--cells --table-out FILE]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]
import torch  # noqa: E402

from mpct.dist import (band_work_estimate, cell_halves, pad_shard, plan_cells_lpt, shard_indices,  # noqa: E402
                       shard_indices_keyed)
from mpct.engine import eval_batch_device  # noqa: E402


def workload(name):
    if name == "shell7x5":
        from mpct.scenarios import config3_grid, shell7x5

        sc, r, v, _ = shell7x5(n2_max=127, nu_max=15)
        return sc, config3_grid(1024), r[None], v[None], 1
    from mpct.dtc import config4_candidates, woodberry_mc

    sc, r, v, _ = woodberry_mc(draws=32, n2_max=30, nu_max=10)
    return sc, config4_candidates(10000), r, v, 32


def time_shard(sc, cand, refs, v, nref, idx, reps=3):
    dev = torch.device("cuda:0")
    N2, Nu, d, l = pad_shard(*cand, idx)
    t = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in dict(N2=N2, Nu=Nu, d=d, l=l, r=refs).items()}
    tv = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    S = idx.size * nref
    out = dict(J1=torch.empty((S, sc.my), dtype=torch.float64, device=dev),
               status=torch.empty(S, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(S, dtype=torch.int64, device=dev))
    s = torch.cuda.current_stream()
    ms = []
    for k in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        eval_batch_device(sc, t["N2"], t["Nu"], t["d"], t["l"], t["r"], out, v=tv, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        if k:
            ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


def cell_table(sc, cand, refs, v, nref):
    """Every (N2, Nu) cell of the config-3 grid alone, whole and as its two halves (median of 3)."""
    N2, Nu, _, lam = cand
    work = band_work_estimate(N2, Nu, lam)
    cells = []
    for n2, nu in sorted(set(zip(N2.tolist(), Nu.tolist()))):
        idx = np.nonzero((N2 == n2) & (Nu == nu))[0]
        whole = time_shard(sc, cand, refs, v, nref, idx)
        halves = [time_shard(sc, cand, refs, v, nref, h) for h in cell_halves(idx, work[idx])]
        cells.append(dict(N2=n2, Nu=nu, n=int(idx.size), ms=whole, half_ms=halves))
        print("cell", n2, nu, "%.2f ms  halves %.2f %.2f" % (whole, halves[0], halves[1]), flush=True)
    return cells


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--only", default=None, help="shell7x5 or dtc-mc")
    ap.add_argument("--cells", action="store_true", help="config 3: time the cells, then the LPT plan's shards")
    ap.add_argument("--table-out", default=None, help="where --cells writes the cell table")
    ap.add_argument("--plans", default=None,
                    help="config 3: comma-separated LPT plans beta:split_ms (split 'none' = never) timed from the "
                         "committed cell table, e.g. 0.4:none,1:none")
    a = ap.parse_args()
    W = a.world
    rep = {}
    for name in ("shell7x5", "dtc-mc"):
        if a.only and name != a.only:
            continue
        sc, cand, refs, v, nref = workload(name)
        C = len(cand[0])
        per = -(-C // W)
        res = {}
        splits = ("contiguous", "strided", "keyed", "keyed_heavy_first") if name == "shell7x5" else ("contiguous", "strided")
        table = None
        plans = {}
        if name == "shell7x5" and a.plans:
            splits = ("contiguous", "keyed")
            for pl in a.plans.split(","):
                b, sp = pl.split(":")
                plans["lpt_%s_%s" % (b, sp)] = (float(b), None if sp == "none" else float(sp))
            splits = splits + tuple(plans)
        if name == "shell7x5" and a.cells:
            cells = cell_table(sc, cand, refs, v, nref)
            res["cells"] = cells
            if a.table_out:
                with open(a.table_out, "w") as f:
                    json.dump({"source": "tools/shard_balance.py --cells: each config-3 (N2, Nu) cell (1024 lambda "
                                         "draws of mpct.scenarios.config3_grid) scored alone on one MI355X, whole "
                                         "and as the two halves of mpct.dist.cell_halves; HIP events, median of 3, "
                                         "ms", "cells": cells}, f, indent=1)
            table = {(c["N2"], c["Nu"]): dict(ms=c["ms"], half_ms=c["half_ms"], n=c["n"]) for c in cells}
            splits = ("contiguous", "keyed", "lpt")
        for split in splits:
            times = []
            pred = None
            if split == "lpt":
                owners, pred = plan_cells_lpt(cand[0], cand[1], cand[3], W, table=table)
            elif split in plans:
                owners, pred = plan_cells_lpt(cand[0], cand[1], cand[3], W, beta=plans[split][0],
                                              split_ms=plans[split][1])
            for rk in range(W):
                if split == "contiguous":
                    idx = np.arange(rk * per, (rk + 1) * per)
                elif split == "strided":
                    idx = shard_indices(C, W, rk)
                elif split == "lpt" or split in plans:
                    idx = owners[rk]
                else:
                    idx = shard_indices_keyed(band_work_estimate(cand[0], cand[1], cand[3]), W, rk,
                                              heavy_first=split == "keyed_heavy_first")
                times.append(time_shard(sc, cand, refs, v, nref, idx))
                print(name, split, rk, "%.1f ms" % times[-1], flush=True)
            res[split] = dict(shard_ms=times, max_over_mean=max(times) / float(np.mean(times)), total_ms=sum(times))
            if pred is not None:
                res[split]["predicted_ms"] = pred
        rep[name] = res
    print(json.dumps({k: {s: {kk: vv for kk, vv in d.items() if kk != "shard_ms"} if isinstance(d, dict) else None
                          for s, d in v.items() if s != "cells"} for k, v in rep.items()}, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
