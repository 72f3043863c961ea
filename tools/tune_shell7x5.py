"""End-to-end tuning of the Shell 7x5 benchmark (Shell7x5.m:204 MPCTuning(mpc, Xsp, lineal, w, nit,
Yref, mdv, 7, 4)) on the GPU engine: a non-square 7x3 plant with 2 measured disturbances and soft
output bands (band mode, every OV weight 0: GAM varies the MV-rate weights only, GAM_fun.m:62-72).
VNS simulates each neighbour once with Xsp (VNS2.m:166-169); mdv (0.5 from k = 20, scaled by Rv,
MPCTuning.m:191) reaches every simulation.  x0: Weights.OV = 0 (q0), Weights.MVRate = 0.1 (w0)
(Shell7x5.m:186-188); w = Shell7x5.m:201.  Tuning_Parameters carries scale.{L,R,Ru,Rv}.
python tools/tune_shell7x5.py [out.mat] [gam_max_iter]"""
import sys

import numpy as np

from tune_common import log, run, score_point
from mpct.scenarios import SHELL7_L, SHELL7_R, SHELL7_TUNED, SHELL7_W, shell7x5
from mpct.tuning import scale_record

out = sys.argv[1] if len(sys.argv) > 1 else None
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
sc, r, v, yref = shell7x5(n2_max=127, nu_max=15)
N, Nu, delta, lam, Fob, dt = run("Shell7x5", sc, r, 7, 3, SHELL7_W, 7, 4, sc.dmin, q0=np.zeros(7),
                                 w0=np.full(3, 0.1), scale=scale_record(SHELL7_L, SHELL7_R, 3), mdv=v, out=out,
                                 gam_max_iter=gmax)
for tag, pt in (("tuner", (N, Nu, delta, lam)),
                ("committed 14Sep2024", (SHELL7_TUNED["N"], SHELL7_TUNED["Nu"], SHELL7_TUNED["delta"],
                                         SHELL7_TUNED["lam"]))):
    F, J1, Jw, st = score_point(sc, r, *pt, SHELL7_W, mdv=v)
    log("score %-20s N=%s Nu=%s: Fvns=%.4f  w'J1=%.5f  status=%d" % (tag, np.max(pt[0]), list(pt[1]), F, Jw, st))
