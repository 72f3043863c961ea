"""NMPC order dependence probe: the 256-candidate grid of test_nmpc_gpu_deterministic_and_order_free
in grid and reversed order; for every candidate whose J1 differs, its parameters, statuses and SQP
iteration counts in both orders, alone (C = 1), and twice in a row.
Usage: python tools/diag/nmpc_order.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch  # noqa: E402
from mpct.nmpc import nmpc_candidate_grid, vandevusse  # noqa: E402

sc, r, yref = vandevusse()
N, Nu, d, lam = nmpc_candidate_grid(256)
a = eval_batch(sc, N, Nu, d, lam, r[None])
b = eval_batch(sc, N[::-1], Nu[::-1], d[::-1], lam[::-1], r[None])
a2 = eval_batch(sc, N, Nu, d, lam, r[None])
bJ = b.J1[::-1]
bad = np.nonzero(np.any(a.J1 != bJ, axis=1))[0]
print("mismatching candidates:", bad.tolist(), "repeat-identical:", bool(np.array_equal(a.J1, a2.J1)))
for k in bad:
    one = eval_batch(sc, N[k:k + 1], Nu[k:k + 1], d[k:k + 1], lam[k:k + 1], r[None])
    print("cand %d N=%d Nu=%d M=%d | grid J1 %s st %d it %d | rev J1 %s st %d it %d | alone J1 %s st %d it %d" % (
        k, N[k], Nu[k], 2 * Nu[k], a.J1[k], a.status[k], a.qp_iters[k], bJ[k], b.status[::-1][k],
        b.qp_iters[::-1][k], one.J1[0], one.status[0], one.qp_iters[0]), flush=True)
