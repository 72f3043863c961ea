"""GPU-vs-oracle check of the NMPC kernel (config 5): prints per-candidate trajectory errors."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]
import torch  # noqa: E402,F401

import oracle.nmpc_vdv as nv  # noqa: E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.nmpc import nmpc_candidate_grid, vandevusse  # noqa: E402


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main():
    sc, r, yref = vandevusse()
    N, Nu, d, lam = nmpc_candidate_grid(int(os.environ.get("NC", "6")))
    t0 = time.time()
    res = eval_batch(sc, N, Nu, d, lam, r[None], open_loop=True, want_traj=True)
    print("gpu %.3fs status %s iters %s" % (time.time() - t0, res.status.tolist(), res.qp_iters.tolist()), flush=True)
    for k in range(min(N.size, int(os.environ.get("NO", "6")))):
        t1 = time.time()
        o = nv.closedloop_nmpc(r, int(N[k]), int(Nu[k]), d[k], lam[k])
        print("k=%d N=%d Nu=%d y %.2e u %.2e yopt %.2e uopt %.2e J1 %s/%s it %d/%d (%.1fs)" % (
            k, N[k], Nu[k], rel(res.y[k], o.y), rel(res.u[k], o.u), rel(res.ys[k], o.yopt),
            rel(res.uopt[k], o.uopt), res.J1[k], ((o.y - yref) ** 2).sum(1), res.qp_iters[k], o.sqp_iters,
            time.time() - t1), flush=True)
        if k == 0:
            print(" gpu u", res.u[k][:, :6], "\n orc u", o.u[:, :6])


if __name__ == "__main__":
    main()
