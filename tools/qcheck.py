"""Quick GPU-vs-C-port check of the closed-loop kernel for one template size class:
python tools/qcheck.py NU_MAX [C]  (nu_max 5 -> MAXM=16 kernel, 6..10 -> 32, >10 -> 64)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
from mpct.engine import eval_batch
from mpct.scenarios import candidate_grid, shell3x3
from oracle.cport import CPort
from oracle.scenarios import shell3x3 as o_shell3x3

numax = int(sys.argv[1]) if len(sys.argv) > 1 else 5
C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
sc, r, yref = shell3x3(n2_max=30, nu_max=numax)
osc, orr, oyref, _ = o_shell3x3()
cp = CPort(osc, 30, 500, oyref)
N2, Nu, d, l = candidate_grid(C)
res = eval_batch(sc, N2, Nu, d, l, r[None])
ref = cp.eval(N2, Nu, d, l, orr[None], threads=16)
rel = np.max(np.abs(res.J1 - ref["J1"]) / np.maximum(np.abs(ref["J1"]), 1e-12), axis=1)
bad = np.nonzero(res.status)[0]
print("nu_max %d C %d: status!=0 %d %s  max rel %.2e  gpu iters %d  cport iters %d" % (
    numax, C, len(bad), bad[:8].tolist(), np.nanmax(rel), res.qp_iters.sum(), ref["qp_iters"].sum()))
w = np.argsort(-np.nan_to_num(rel, nan=1.0))[:5]
print("  worst:", [(int(k), float(rel[k]), int(res.qp_iters[k]), int(ref["qp_iters"][k])) for k in w])
