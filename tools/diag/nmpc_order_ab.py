import os, sys
import numpy as np
import torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch_device
from mpct.nmpc import nmpc_candidate_grid, vandevusse
sc, r, yref = vandevusse()
N, Nu, d, l = nmpc_candidate_grid(4096)
dev = torch.device("cuda", 0); C = N.size
def timed(perm, reps=3):
    t = [torch.from_numpy(np.ascontiguousarray(a[perm])).to(dev) for a in (N, Nu, d, l)]
    tr = torch.from_numpy(r[None].copy()).to(dev)
    out = dict(J1=torch.empty((C, 2), dtype=torch.float64, device=dev), status=torch.empty(C, dtype=torch.int32, device=dev), qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    eval_batch_device(sc, *t, tr, out); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eval_batch_device(sc, *t, tr, out); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))
print(os.path.basename(os.environ.get("MPCT_LIB", "libmpct.so")), "grid input %.1f ms" % timed(np.arange(C)), "desc N*Nu input %.1f ms" % timed(np.argsort(-(N * Nu), kind="stable")), flush=True)
