"""C-vs-C floor of the config-3 parity: the whole 65,536-candidate grid scored by
the C restatement a second time, with an equally valid QP path -- every step's dual method
warm-started from the previous step's final active set (oracle/cband.c cb_scen.qp_warm) instead of
cold from the unconstrained minimum -- and compared with the committed cold fixture
(tests/golden/config3_cband.npz).  Both paths solve the same strictly convex QPs to the same
termination test, so the fraction of candidates whose Pareto-weighted F = J1 @ SHELL7_W differs by
more than 1e-6 is what two correct implementations of the reference's loop cannot agree on: the
floor the device's fraction is stated against.  CPU only (oracle/ is test
infrastructure).  Usage: python tools/config3_floor.py [--threads 8] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]

from mpct.scenarios import SHELL7_W, config3_grid, config3_stratified  # noqa: E402
from oracle.cband import CBand  # noqa: E402
from oracle.scenarios import shell7x5  # noqa: E402


def rank_prefix(F, Fr):
    o, orr = np.argsort(F, kind="stable"), np.argsort(Fr, kind="stable")
    first = np.nonzero(o != orr)[0]
    return int(first[0]) if first.size else int(F.size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--out", default=None)
    ap.add_argument("--save", default=None, help="npz of the warm path's F and status")
    a = ap.parse_args()
    d = np.load(os.path.join(ROOT, "tests", "golden", "config3_cband.npz"))
    sc, r, v, yref, fx = shell7x5()
    cb = CBand(sc, 200, yref, warm=True)
    N2, Nu, D, L = config3_grid(1024)
    C = N2.size
    J1 = np.zeros((C, 7))
    st = np.zeros(C, np.int32)
    it = np.zeros(C, np.int64)
    t0 = time.time()
    order = np.argsort((np.arange(C) * 7919) % C, kind="stable")
    for k in range(0, C, a.chunk):
        idx = order[k:k + a.chunk]
        o = cb.eval(N2[idx], Nu[idx], D[idx], L[idx], r[None], v[None], threads=a.threads)
        J1[idx], st[idx], it[idx] = o["J1"], o["status"], o["qp_iters"]
        print("%d / %d  %.0f s" % (k + idx.size, C, time.time() - t0), flush=True)
    F, F0 = J1 @ SHELL7_W, d["F_full"]
    relF = np.abs(F - F0) / np.abs(F0)
    s = config3_stratified(128)
    relJ = np.max(np.abs(J1[s] - d["J1_strat"]) / np.abs(d["J1_strat"]), axis=1)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_band import rank_stats  # noqa: E402

    rep = dict(path="cband.c warm-started dual method vs the committed cold fixture",
               candidates=int(C), failed_warm=int(np.sum(st != 0)),
               F_frac_gt_1e6=float(np.mean(relF > 1e-6)), F_count_gt_1e6=int(np.sum(relF > 1e-6)),
               F_median_rel=float(np.median(relF)), F_max_rel=float(relF.max()),
               J1_strat_frac_gt_1e6=float(np.mean(relJ > 1e-6)),
               ranking_identical_prefix=rank_prefix(F, F0), rank=rank_stats(F, F0),
               qp_iters_mean_warm=float(it.mean()), seconds=round(time.time() - t0, 1), threads=a.threads)
    print(json.dumps(rep, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)
    if a.save:
        np.savez_compressed(a.save, F=F, st=st.astype(np.int8))


if __name__ == "__main__":
    main()
