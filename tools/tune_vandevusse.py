"""End-to-end NMPC tuning of the Van de Vusse reactor (VanDeVusse_NMPC.m:200-205:
MPCTuning(nlobj_proj, r, lineal=false, w=[0.7 0.3], nit, Yref, mdv, nbp=5, nbc=4, model, init)) on
the GPU engine: GAM weights + VNS horizons alternated as MPC_TFob.m, Tuning_Parameters written
like MPCTuning.m:374-381.  Initial weights: the nlmpc object's delta = [1 1], lambda = [0.1 0.1]
(VanDeVusse_NMPC.m:193-198).  python tools/tune_vandevusse.py [out.mat] [gam_max_iter]"""
import sys

import numpy as np

from tune_common import run
from mpct.nmpc import VDV_W, vandevusse

out = sys.argv[1] if len(sys.argv) > 1 else None
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
sc, r, yref = vandevusse(n_max=31, nu_max=15)
run("VanDeVusse_NMPC", sc, r, 2, 2, VDV_W, 5, 4, np.zeros(2, dtype=int), q0=np.array([1.0, 1.0]),
    w0=np.array([0.1, 0.1]), lineal=False, out=out, gam_max_iter=gmax)
