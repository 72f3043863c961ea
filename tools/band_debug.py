"""Per-step trace of one Shell 7x5 band-mode simulation: GPU (debug library built with
-DMPCT_DEBUG_BAND, printf from the kernel) next to the oracle's steps."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "model-predictive-control-tuning_amd", "csrc")
T = int(os.environ.get("NT", "40"))
if __name__ == "__main__" and "--oracle" not in sys.argv:
    lib = os.path.join(CSRC, "libmpct_dbg.so")
    if not os.path.exists(lib):
        objs = []
        for f in ("gpc_kernel.hip", "mdband_kernel.hip", "mpct_host.cpp"):
            o = os.path.join("/tmp", f + ".dbg.o")
            subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DMPCT_DEBUG_BAND=%d" % T,
                            "-c", os.path.join(CSRC, f), "-o", o], check=True)
            objs.append(o)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", lib], check=True)
    os.environ["MPCT_LIB"] = lib
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]

N2, NU = int(os.environ.get("N2", "27")), int(os.environ.get("NU", "2"))
LAM = np.array([float(x) for x in os.environ.get("LAM", "0.055949075594369936,0.016702486485524682,1.6101890690935143").split(",")])


def oracle():
    from oracle.scenarios import shell7x5
    from oracle.toolbox_band import band_qp, closedloop_band, dyn_matrix, simulate, step_table

    sc, r, v, yref, fx = shell7x5()
    tr = []
    res = closedloop_band(sc, r, v, N2, NU, np.zeros(7), LAM, 200, open_loop=False, trace=tr)
    for t in range(T):
        print("o t=%d it=? eps=%.9e du=%.9e %.9e %.9e F0=%.9e Fend=%.9e y6=%.9e" % (
            t, res.eps[t], res.du_hist[0, t], res.du_hist[1, t], res.du_hist[2, t], tr[t][0], tr[t][N2 - 1], tr[t][6 * N2]))


DEL = os.environ.get("DEL")


def gpu():
    import torch  # noqa: F401
    from mpct.engine import eval_batch
    from mpct.scenarios import shell7x5, woodberry_toolbox

    if os.environ.get("SCEN") == "wb":
        sc, r, v, yref = woodberry_toolbox()
        D = np.array([float(x) for x in DEL.split(",")])[None]
    else:
        sc, r, v, yref = shell7x5(n2_max=int(os.environ.get("N2MAX", "40")), nu_max=int(os.environ.get("NUMAX", "8")))
        D = np.zeros((1, 7))
    res = eval_batch(sc, [N2], [NU], D, LAM[None], r[None], v=v[None], open_loop=False, device=0)
    torch.cuda.synchronize()
    print("status", res.status, "iters", res.qp_iters, flush=True)


if __name__ == "__main__":
    if "--oracle" in sys.argv:
        oracle()
    else:
        gpu()
