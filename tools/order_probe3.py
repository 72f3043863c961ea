"""Probe: config-3 (Shell 7x5 band) batch time in grid order (N2 ascending blocks) vs orders by
measured work (QP iterations) and by a-priori keys (N2 x Nu descending)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT, os.path.join(ROOT, "tools")]
from bench_config3 import grid  # noqa: E402
from mpct.engine import eval_batch_device  # noqa: E402
from mpct.scenarios import shell7x5  # noqa: E402

sc, r, v, yref = shell7x5(n2_max=127, nu_max=15)
N2, Nu, D, L = grid(1024)
C = N2.size
dev = torch.device("cuda", 0)


def timed(perm):
    t = [torch.from_numpy(np.ascontiguousarray(a[perm])).to(dev) for a in (N2, Nu, D, L)]
    tr = torch.from_numpy(r[None].copy()).to(dev)
    tv = torch.from_numpy(v[None].copy()).to(dev)
    out = dict(J1=torch.empty((C, 7), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eval_batch_device(sc, *t, tr, out, v=tv)
    e1.record()
    torch.cuda.synchronize()
    it = np.empty(C, np.int64)
    it[perm] = out["qp_iters"].cpu().numpy()
    return e0.elapsed_time(e1), it


base = np.arange(C)
tb, it = timed(base)
print("grid order      %.1f ms  qp iters/sim: min %d median %d max %d" % (tb, it.min(), np.median(it), it.max()), flush=True)
print("desc measured   %.1f ms" % timed(np.argsort(-it * N2, kind="stable"))[0], flush=True)
print("desc N2*Nu      %.1f ms" % timed(np.argsort(-(N2.astype(np.int64) * Nu), kind="stable"))[0], flush=True)
print("reverse grid    %.1f ms" % timed(base[::-1].copy())[0], flush=True)
