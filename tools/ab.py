"""A/B wall time of libmpct builds on the 4096-candidate Shell 3x3 batch (interleaved rounds,
one process per build is not possible: one HIP library per process -> run this per build)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
import torch
from mpct.engine import eval_batch_device
from mpct.scenarios import candidate_grid, shell3x3
sc, r, yref = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
dev = torch.device("cuda", 0)
t = [torch.from_numpy(a.copy()).to(dev) for a in (N2, Nu, d, l, r[None])]
out = dict(J1=torch.empty((4096, 3), dtype=torch.float64, device=dev),
           status=torch.empty(4096, dtype=torch.int32, device=dev),
           qp_iters=torch.empty(4096, dtype=torch.int64, device=dev))
for _ in range(2):
    eval_batch_device(sc, *t, out)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); eval_batch_device(sc, *t, out); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
print(os.path.basename(os.environ.get("MPCT_LIB", "libmpct.so")), "kernel ms: median %.2f min %.2f" % (np.median(ts), min(ts)),
      "status nz", int((out["status"] != 0).sum()))
