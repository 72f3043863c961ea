"""Diagnostic: per-draw kernel vs oracle peak |y| for the config-4 plant variants."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
from mpct.dtc import woodberry_mc, woodberry_dtc
from mpct.engine import eval_batch, Scenario
from oracle.dtcgpc import dtc_gpc_ww, woodberry_mc_draws

D = 4
sc, refs, v, plants = woodberry_mc(draws=D, n2_max=10, nu_max=5)
N2 = np.array([8], np.int32); Nu = np.array([4], np.int32)
rng = np.random.default_rng(5)
rng.integers(3, 11, 6); rng.integers(1, 6, 6)
d = 10.0 ** rng.uniform(-1, 1, (6, 2))[:1]
l = 10.0 ** rng.uniform(-1, 1, (6, 2))[:1]
res = eval_batch(sc, N2, Nu, d, l, refs, v=v, want_traj=True)
op = woodberry_mc_draws(D)
for k in range(D):
    ref = dtc_gpc_ww(p=(8, 8), m=(4, 4), lam=tuple(l[0]), delta=tuple(d[0]), plant=op[k])
    print("draw", k, "status", res.status[k], "kernel max|y| %.3e" % np.abs(res.y[k]).max(),
          "oracle max|y| %.3e" % np.abs(ref["y"]).max(), "y[:, :5] kernel", res.y[k][:, 60:64].ravel(),
          "oracle", ref["y"][:, 60:64].ravel())
    print("   plant k", [(p.num, p.den, p.delay) for row in plants[k] for p in row])
