"""End-to-end tuning of the Wood-Berry column with the toolbox MPC (WoodBerry.m:156 MPCTuning(mpc,
Xsp, lineal, w, nit, Yref, mdv, 7, 4)) on the GPU engine: square 2x2 plant with one measured
disturbance (mdv = -0.25 from k = 300, WoodBerry.m:92-94), rate / amplitude bounds, nit = 400.
x0 = the mpc(sysd, Ts) default weights OV = 1, MVRate = 0.1 (WoodBerry.m:107 sets none); w =
[0.1 0.5] (WoodBerry.m:155).  The reference commits no WoodBerry tuning file, so CondMin's scaling
is not pinned: L = R = I (labelled in the record).  python tools/tune_woodberry.py [out] [gam_max_iter]"""
import sys

import numpy as np

from tune_common import run
from mpct.scenarios import WB_W, woodberry_toolbox
from mpct.tuning import scale_record

out = sys.argv[1] if len(sys.argv) > 1 else None
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
sc, r, v, yref = woodberry_toolbox(n2_max=127, nu_max=15, nit=400)
run("WoodBerry", sc, r, 2, 2, WB_W, 7, 4, sc.dmin, q0=np.ones(2), w0=np.full(2, 0.1),
    scale=scale_record(np.ones(2), np.ones(3), 2), mdv=v, out=out, gam_max_iter=gmax)
