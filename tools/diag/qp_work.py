"""QP work distribution over the metric grid (wave kernel): GI iterations per simulation."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import torch  # noqa: F401,E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.scenarios import candidate_grid, shell3x3  # noqa: E402

sc, r, _ = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
res = eval_batch(sc, N2, Nu, d, l, r[None])
it = res.qp_iters
print("qp iters per sim: mean %.1f  pct 50/75/90/99/max %s" % (it.mean(), np.percentile(it, [50, 75, 90, 99, 100])))
print("sims with 0 iterations: %d, < 20: %d, >= 200: %d" % ((it == 0).sum(), (it < 20).sum(), (it >= 200).sum()))
np.save(os.path.join(ROOT, "gpurun_out", "qp_iters.npy"), it)
