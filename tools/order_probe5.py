"""Probe: config-5 (NMPC) batch time in grid order vs orders by measured per-candidate work
(SQP iterations x horizon), descending and ascending, and by simple a-priori keys."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch_device  # noqa: E402
from mpct.nmpc import nmpc_candidate_grid, vandevusse  # noqa: E402

sc, r, yref = vandevusse()
N, Nu, d, l = nmpc_candidate_grid(4096)
dev = torch.device("cuda", 0)
C = N.size


def timed(perm, reps=2):
    t = [torch.from_numpy(np.ascontiguousarray(a[perm])).to(dev) for a in (N, Nu, d, l)]
    tr = torch.from_numpy(r[None].copy()).to(dev)
    out = dict(J1=torch.empty((C, 2), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    eval_batch_device(sc, *t, tr, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eval_batch_device(sc, *t, tr, out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    it = np.empty(C, np.int64)
    it[perm] = out["qp_iters"].cpu().numpy()
    return float(np.median(ts)), it


base = np.arange(C)
tb, it = timed(base)
np.savez(os.path.join(ROOT, "gpurun_out", "nmpc_work.npz"), N=N, Nu=Nu, d=d, l=l, it=it)
w = it * N
print("grid order     %.1f ms  sqp iters/sim: min %d median %d max %d" % (tb, it.min(), np.median(it), it.max()), flush=True)
print("desc it*N      %.1f ms" % timed(np.argsort(-w, kind="stable"))[0], flush=True)
print("asc it*N       %.1f ms" % timed(np.argsort(w, kind="stable"))[0], flush=True)
print("desc N*Nu      %.1f ms" % timed(np.argsort(-(N * Nu), kind="stable"))[0], flush=True)
