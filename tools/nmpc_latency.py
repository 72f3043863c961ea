"""Latency of small NMPC batches (the tuning loop's GAM finite differences): C = 1 and 8 at the
tuning's candidates, with the nominal state bounds and with them removed."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct import nmpc  # noqa: E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.objectives import vns_refs_nonlinear  # noqa: E402

x0 = nmpc.steady_state()
r, yref = nmpc.vandevusse_signals(x0)
refs = vns_refs_nonlinear(r)
for name, xmax in (("bounds", nmpc.VDV_XMAX), ("no bounds", np.full(3, np.inf))):
    xmin = nmpc.VDV_XMIN if name == "bounds" else np.full(3, -np.inf)
    sc = nmpc.NmpcScenario(x0, nmpc.VDV_U0, nmpc.VDV_UMIN, nmpc.VDV_UMAX, xmin, xmax, yref, 31, 15,
                           y_scale=nmpc.VDV_XMAX[1:] - nmpc.VDV_XMIN[1:])
    for (N, Nu, d, l) in ((31, 2, [11.0, 8.6], [21.4, 40.4]), (31, 2, [0.86, 0.29], [1.03, 1.25]), (3, 2, [1, 1], [0.1, 0.1])):
        for C in (1, 8):
            a = [np.full(C, N, np.int32), np.full(C, Nu, np.int32), np.tile(d, (C, 1)), np.tile(l, (C, 1))]
            eval_batch(sc, *a, refs, open_loop=True)
            t = time.perf_counter()
            res = eval_batch(sc, *a, refs, open_loop=True)
            print("%-9s N=%d Nu=%d d=%s l=%s C=%d: %.1f ms status %s sqp %s" % (
                name, N, Nu, d, l, C, (time.perf_counter() - t) * 1e3, np.unique(res.status), res.qp_iters[:2]), flush=True)
