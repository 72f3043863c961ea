"""Where a Van de Vusse GAM run's time goes: the first goal-attainment phase of tune_vandevusse.py
(MPC_TFob.m's GAM, max_iter GAM iterations) with every engine call timed.  Prints the number of
calls, the batch sizes, the wall time per call inside eval_batch and outside it (SLSQP and the
Python host), and the mean SQP iterations per simulation.
Usage: python tools/diag/gam_calls.py [max_iter]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import mpct.engine as eng  # noqa: E402
from mpct import tuning  # noqa: E402
from mpct.nmpc import VDV_W, vandevusse  # noqa: E402

max_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 60
sc, r, yref = vandevusse(n_max=31, nu_max=15)
calls = []
orig = eng.eval_batch


def timed(*a, **k):
    t = time.perf_counter()
    res = orig(*a, **k)
    calls.append((time.perf_counter() - t, len(a[1]), float(np.mean(res.qp_iters)), int(a[1][0]), int(a[2][0])))
    return res


eng.eval_batch = timed
t0 = time.perf_counter()


class Stop(Exception):
    pass


def log(msg):
    print(msg, flush=True)
    if msg.startswith("Fgam="):  # the first GAM phase is done
        raise Stop


try:
    tuning.mpc_tuning(sc, r, my=2, ny=2, w=VDV_W, nbp=5, nbc=4, dmin=np.zeros(2, dtype=int),
                      q0=np.array([1.0, 1.0]), w0=np.array([0.1, 0.1]), lineal=False, log=log,
                      save_path=os.path.join(ROOT, "gpurun_out", "gam_calls.mat"), gam_max_iter=max_iter)
except Stop:
    pass
wall = time.perf_counter() - t0
dt = np.array([c[0] for c in calls])
C = np.array([c[1] for c in calls])
it = np.array([c[2] for c in calls])
print("GAM phase (max_iter %d): %.1f s wall, %d engine calls, %.1f s inside eval_batch (%.1f ms per call, "
      "median %.1f ms), %.1f s outside" % (max_iter, wall, len(calls), dt.sum(), 1e3 * dt.mean(),
                                             1e3 * np.median(dt), wall - dt.sum()))
print("batch sizes:", dict(zip(*np.unique(C, return_counts=True))), "N/Nu:", sorted({(c[3], c[4]) for c in calls}))
print("SQP iterations per simulation: mean %.1f, max %.1f" % (it.mean(), it.max()))
