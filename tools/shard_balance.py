"""Per-shard time of the 8-rank splits on one GPU: for config 3 (the 65,536
Shell 7x5 grid, cell-ordered) and config 4 (10,000 WoodBerry DTC candidates x 32 draws), each of
the 8 shards of the contiguous (round 2), strided (mpct.dist.shard_indices) and, for config 3,
work-keyed (mpct.dist.shard_indices_keyed, candidates in index order or heaviest first) splits is scored alone on cuda:0 and timed with HIP
events (median of 3); max/mean shard time predicts the 8-GPU efficiency loss from imbalance.
Usage: python tools/shard_balance.py [--out FILE]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]
import torch  # noqa: E402

from mpct.dist import band_work_estimate, pad_shard, shard_indices, shard_indices_keyed  # noqa: E402
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--only", default=None, help="shell7x5 or dtc-mc")
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
        for split in splits:
            times = []
            for rk in range(W):
                if split == "contiguous":
                    idx = np.arange(rk * per, (rk + 1) * per)
                elif split == "strided":
                    idx = shard_indices(C, W, rk)
                else:
                    idx = shard_indices_keyed(band_work_estimate(cand[0], cand[1], cand[3]), W, rk,
                                              heavy_first=split == "keyed_heavy_first")
                times.append(time_shard(sc, cand, refs, v, nref, idx))
                print(name, split, rk, "%.1f ms" % times[-1], flush=True)
            res[split] = dict(shard_ms=times, max_over_mean=max(times) / float(np.mean(times)))
        rep[name] = res
    print(json.dumps(rep, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
