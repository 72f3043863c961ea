"""End-to-end MPC tuning of the Shell 3x3 benchmark (Shell3x3.m:163 MPCTuning(..., nbp=7, nbc=4))
on the GPU engine: GAM weights + VNS horizons, alternated as MPC_TFob.m, Tuning_Parameters
written like MPCTuning.m:374-381.  python tools/tune_shell3x3.py [out.mat] [gam_max_iter]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
from mpct.scenarios import SHELL3_L, SHELL3_R, shell3x3
from mpct.tuning import mpc_tuning

out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "Shell3x3_Tuning.mat")
gmax = int(sys.argv[2]) if len(sys.argv) > 2 else 400
sc, r, yref = shell3x3(n2_max=127, nu_max=15)
t0 = time.time()
N, Nu, delta, lam, Fob = mpc_tuning(sc, r, my=3, ny=3, w=np.array([0.05, 0.40, 0.55]), nbp=7, nbc=4,
                                    dmin=sc.dmin, log=print, save_path=out, gam_max_iter=gmax,
                                    scale={"L": np.diag(SHELL3_L), "R": np.diag(SHELL3_R)})
print("N=%s Nu=%s delta=%s lambda=%s Fob=%s  (%.1f s)" % (N, Nu, delta, lam, Fob, time.time() - t0))
