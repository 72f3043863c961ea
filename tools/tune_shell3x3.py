"""End-to-end MPC tuning of the Shell 3x3 benchmark (Shell3x3.m:163 MPCTuning(..., nbp=7, nbc=4))
on the GPU engine: GAM weights + VNS horizons, alternated as MPC_TFob.m, Tuning_Parameters written
like MPCTuning.m:374-381 (scale.{L,R,Ru,Rv}).  GAM starts from x0 = [q0 w0] = the mpc object's
weights (MPCTuning.m:163-164,300); Shell3x3.m:108 builds mpc(sysd, Ts) without setting Weights, so
those are the toolbox defaults OV = 1, MVRate = 0.1 (toolbox documentation; parity unpinned).
Finally the tuner's point and the committed Shell3x3_Tuning_25Jul2023 point (N = 24, Nu = [6 2 2])
are scored under the same VNS / GAM objectives.
python tools/tune_shell3x3.py [out.mat] [gam_max_iter]"""
import sys

import numpy as np

from tune_common import log, run, score_point
from mpct.scenarios import SHELL3_L, SHELL3_R, SHELL3_TUNED, shell3x3
from mpct.tuning import scale_record

out = sys.argv[1] if len(sys.argv) > 1 else None
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
w = np.array([0.05, 0.40, 0.55])                                    # Shell3x3.m:161
sc, r, yref = shell3x3(n2_max=127, nu_max=15)
N, Nu, delta, lam, Fob, dt = run("Shell3x3", sc, r, 3, 3, w, 7, 4, sc.dmin, q0=np.ones(3), w0=np.full(3, 0.1),
                                 scale=scale_record(SHELL3_L, SHELL3_R, 3), out=out, gam_max_iter=gmax)
for tag, pt in (("tuner", (N, Nu, delta, lam)),
                ("committed 25Jul2023", (SHELL3_TUNED["N"], SHELL3_TUNED["Nu"], SHELL3_TUNED["delta"],
                                         SHELL3_TUNED["lam"]))):
    F, J1, Jw, st = score_point(sc, r, *pt, w)
    log("score %-20s N=%s Nu=%s: Fvns=%.4f  J1=%s  w'J1=%.5f  status=%d" % (tag, np.max(pt[0]), list(pt[1]), F,
                                                                          np.round(J1, 5), Jw, st))
