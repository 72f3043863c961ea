"""Config 3: time the slowest simulations of the grid alone (C = 1) -- is the batch time set by
one simulation's latency?"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT, os.path.join(ROOT, "tools")]
from bench_config3 import grid  # noqa: E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.scenarios import shell7x5  # noqa: E402

sc, r, v, yref = shell7x5(n2_max=127, nu_max=15)
N2, Nu, D, L = grid(1024)
res = eval_batch(sc, N2, Nu, D, L, r[None], v=v[None])
it = res.qp_iters
top = np.argsort(-it)[:5]
for k in top:
    eval_batch(sc, N2[k:k + 1], Nu[k:k + 1], D[k:k + 1], L[k:k + 1], r[None], v=v[None])
    t = time.perf_counter()
    eval_batch(sc, N2[k:k + 1], Nu[k:k + 1], D[k:k + 1], L[k:k + 1], r[None], v=v[None])
    print("cand %d N2=%d Nu=%d qp_iters=%d alone %.1f ms" % (k, N2[k], Nu[k], it[k], (time.perf_counter() - t) * 1e3), flush=True)
print("qp iters percentiles 50/90/99/99.9/max:", np.percentile(it, [50, 90, 99, 99.9, 100]).astype(int))
