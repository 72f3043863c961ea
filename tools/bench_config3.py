"""Config 3: Shell 7x5 band-mode MPC, 65,536 candidates = N2 in {16,24,32,48,64,96,
112,127} x Nu in {2,3,4,6,8,10,12,15} x 1024 lambda draws (log10 U(-3,1), seed 20250307),
delta = 0, nit = 200, closed loop + GAM J1 (GAM_fun.m:110-111) per candidate, inputs resident in
HBM.  Prints one JSON line (sims/s, kernel ms, status counts, best candidate)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]
import torch  # noqa: E402

from mpct.engine import eval_batch_device  # noqa: E402
from mpct.scenarios import SHELL7_W, shell7x5  # noqa: E402

from mpct.scenarios import config3_grid as grid  # noqa: E402,F401  (the grid lives in the product)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sc, r, v, yref = shell7x5(n2_max=127, nu_max=15)
    N2, Nu, D, L = grid(a.per)
    C = N2.size
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(x).to(dev) for k, x in dict(N2=N2, Nu=Nu, D=D, L=L).items()}
    rr = torch.from_numpy(r[None].copy()).to(dev)
    vv = torch.from_numpy(v[None].copy()).to(dev)
    out = dict(J1=torch.empty((C, 7), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    s = torch.cuda.current_stream()
    times = []
    for rep in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        e0.record(s)
        eval_batch_device(sc, t["N2"], t["Nu"], t["D"], t["L"], rr, out, v=vv, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        wall = time.perf_counter() - w0
        if rep:
            times.append(e0.elapsed_time(e1))
        print("rep %d: %.1f ms (wall %.1f ms)" % (rep, e0.elapsed_time(e1), wall * 1e3), flush=True)
    J1 = out["J1"].cpu().numpy()
    st = out["status"].cpu().numpy()
    it = out["qp_iters"].cpu().numpy()
    F = J1 @ SHELL7_W                      # Pareto-weighted GAM objective (Shell7x5.m:202)
    F[st != 0] = np.inf
    b = int(np.argmin(F))
    ms = float(np.median(times))
    rec = dict(workload="config3 Shell 7x5 band-mode MPC", candidates=C, nit=200, kernel_ms=ms,
               sims_per_s=C / (ms * 1e-3), status_nonzero=int(np.sum(st != 0)),
               status_codes={int(k): int(n) for k, n in zip(*np.unique(st, return_counts=True))},
               qp_iters_mean_per_step=float(it.mean() / 200), lds_bytes_max=int(sc.lds_bytes(127, 15)),
               best=dict(N2=int(N2[b]), Nu=int(Nu[b]), lam=L[b].tolist(), F=float(F[b])))
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
        np.savez_compressed(os.path.splitext(a.out)[0] + ".npz", status=st, qp_iters=it, J1=J1)


if __name__ == "__main__":
    main()
