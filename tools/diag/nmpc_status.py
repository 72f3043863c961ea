"""Config-5 grid (GAM mode and with the open-loop leg): statuses and Gauss-Newton iteration totals
per candidate -> gpurun_out/nmpc_status.npz (tools/diag for the SQP-cap analysis)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import torch  # noqa: F401,E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.nmpc import nmpc_candidate_grid, vandevusse  # noqa: E402

sc, r, yref = vandevusse()
N, Nu, d, l = nmpc_candidate_grid(4096)
out = {}
for ol in (0, 1):
    res = eval_batch(sc, N, Nu, d, l, r[None], open_loop=bool(ol))
    out["status%d" % ol] = res.status
    out["iters%d" % ol] = res.qp_iters
    out["J1%d" % ol] = res.J1
    print("open_loop=%d: status32 %d, status nonzero %d, GN iters mean %.1f max %d" % (
        ol, int(((res.status & 32) != 0).sum()), int((res.status != 0).sum()), res.qp_iters.mean(), res.qp_iters.max()))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "nmpc_status.npz"), N=N, Nu=Nu, d=d, l=l, **out)
