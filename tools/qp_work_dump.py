"""Dump the per-candidate QP iteration counts of the 4096-candidate Shell 3x3 metric batch
(GPU) with the candidate arrays, for choosing a dispatch-order key offline."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch  # noqa: E402
from mpct.scenarios import candidate_grid, shell3x3  # noqa: E402

sc, r, yref = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
res = eval_batch(sc, N2, Nu, d, l, r[None])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "qp_work.npz"), N2=N2, Nu=Nu, d=d, l=l, it=res.qp_iters)
print("saved", res.qp_iters.sum())
