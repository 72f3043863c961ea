"""Section breakdown of the closed-loop kernel from the -DMPCT_PROFILE diagnostic build
(libmpct_prof.so; in-kernel s_memtime stamps).  Stamps add overhead: read shares, not totals.
Usage: python tools/kprof.py [C] [heavy]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCT_LIB", os.path.join(ROOT, "model-predictive-control-tuning_amd", "csrc", "libmpct_prof.so"))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
from mpct.engine import eval_batch
from mpct.scenarios import candidate_grid, shell3x3
C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sc, r, yref = shell3x3()
N2, Nu, d, l = candidate_grid(4096)
# "heavy": the C candidates with the most measured QP work (a first, unprofiled pass)
sel = np.arange(C)
if "heavy" in sys.argv[2:]:
    sel = np.argsort(-eval_batch(sc, N2, Nu, d, l, r[None]).qp_iters, kind="stable")[:C]
N2, Nu, d, l = N2[sel], Nu[sel], d[sel], l[sel]
eval_batch(sc, N2[:64], Nu[:64], d[:64], l[:64], r[None])
t = time.perf_counter()
res = eval_batch(sc, N2, Nu, d, l, r[None])
print("wall %.2f ms for %d sims, qp iters/step %.3f" % ((time.perf_counter() - t) * 1e3, C, res.qp_iters.mean() / 500))
