"""End-to-end NMPC tuning of the Van de Vusse reactor (VanDeVusse_NMPC.m:200-205:
MPCTuning(nlobj_proj, r, lineal=false, w=[0.7 0.3], nit, Yref, mdv, nbp=5, nbc=4, model, init)) on
the GPU engine: GAM weights + VNS horizons alternated as MPC_TFob.m, Tuning_Parameters written
like MPCTuning.m:374-381.  Initial weights: the nlmpc object's delta = [1 1], lambda = [0.1 0.1]
(VanDeVusse_NMPC.m:193-198).  Finally the tuner's point and the committed
VanDeVusse_NMPC_Tuning_25Jul2023 point are scored under the same VNS / GAM objectives.
python tools/tune_vandevusse.py [out.mat] [gam_max_iter]"""
import sys

import numpy as np

from tune_common import log, run, score_point
from mpct.nmpc import VDV_TUNED, VDV_W, vandevusse
from mpct.objectives import vns_refs_nonlinear

out = sys.argv[1] if len(sys.argv) > 1 else None
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
sc, r, yref = vandevusse(n_max=31, nu_max=15)
N, Nu, delta, lam, Fob, dt = run("VanDeVusse_NMPC", sc, r, 2, 2, VDV_W, 5, 4, np.zeros(2, dtype=int),
                                 q0=np.array([1.0, 1.0]), w0=np.array([0.1, 0.1]), lineal=False, out=out,
                                 gam_max_iter=gmax)
for tag, pt in (("tuner", (N, Nu, delta, lam)),
                ("committed 25Jul2023", (VDV_TUNED["N"], VDV_TUNED["Nu"], VDV_TUNED["delta"], VDV_TUNED["lam"]))):
    F, J1, Jw, st = score_point(sc, r, *pt, VDV_W, vns_refs=vns_refs_nonlinear(r))
    log("score %-20s N=%s Nu=%s: Fvns=%.4f  J1=%s  w'J1=%.5f  status=%d" % (tag, np.max(pt[0]), list(pt[1]), F,
                                                                          np.round(J1, 5), Jw, st))
