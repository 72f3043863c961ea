"""Probe: metric-kernel time for the 4096-candidate Shell 3x3 batch in grid order, in descending
and in ascending order of each candidate's measured QP work (longest-processing-time-first vs
last), and by ascending min(lambda) -- does the dispatch order of the second, partial round of
workgroups matter?"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch_device  # noqa: E402
from mpct.scenarios import candidate_grid, shell3x3  # noqa: E402

sc, r, yref = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
dev = torch.device("cuda", 0)


def timed(perm, reps=5):
    t = [torch.from_numpy(np.ascontiguousarray(a[perm])).to(dev) for a in (N2, Nu, d, l)]
    tr = torch.from_numpy(r[None].copy()).to(dev)
    out = dict(J1=torch.empty((4096, 3), dtype=torch.float64, device=dev),
               status=torch.empty(4096, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(4096, dtype=torch.int64, device=dev))
    for _ in range(2):
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
    return float(np.median(ts)), out["qp_iters"].cpu().numpy()


base = np.arange(4096)
tb, it = timed(base)
print("grid order   %.3f ms  qp iters/sim: min %d median %d max %d" % (tb, it.min(), np.median(it), it.max()))
print("desc work    %.3f ms" % timed(np.argsort(-it, kind="stable"))[0])
print("asc work     %.3f ms" % timed(np.argsort(it, kind="stable"))[0])
print("asc min(lam) %.3f ms" % timed(np.argsort(l.min(axis=1), kind="stable"))[0])
