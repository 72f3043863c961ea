"""Dump GPU and C-port J1 for the full Shell 3x3 grid (diagnostics)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
from mpct.engine import eval_batch
from mpct.scenarios import candidate_grid, shell3x3
from oracle.cport import CPort
from oracle.scenarios import shell3x3 as o3
sc, r, yref = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
g = eval_batch(sc, N2, Nu, d, l, r[None])
osc, orr, oyref, _ = o3()
c = CPort(osc, 30, 500, oyref).eval(N2, Nu, d, l, orr[None], threads=16)
np.savez(os.path.join(ROOT, "gpurun_out", "grid_dump.npz"), gJ1=g.J1, cJ1=c["J1"], gst=g.status, cst=c["status"],
         git=g.qp_iters, cit=c["qp_iters"])
rel = np.max(np.abs(g.J1 - c["J1"]) / np.maximum(np.abs(c["J1"]), 1e-12), axis=1)
o = np.argsort(-rel)[:10]
print("worst", list(zip(o.tolist(), rel[o].tolist())))
print("count rel>1e-6:", int((rel > 1e-6).sum()), "rel>1e-9:", int((rel > 1e-9).sum()))
