"""Config-5 grid J1 / j21 / status / SQP iterations with the library in MPCT_LIB ->
gpurun_out/nmpc_<tag>.npz, compared with another tag's file when given (A/B of NMPC-kernel variants:
a restructuring that keeps the arithmetic must match bitwise).  python tools/diag/nmpc_ab.py TAG [OTHER]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import torch  # noqa: F401,E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.nmpc import nmpc_candidate_grid, vandevusse  # noqa: E402

tag = sys.argv[1]
sc, r, yref = vandevusse()
N, Nu, D, L = nmpc_candidate_grid(4096)
res = eval_batch(sc, N, Nu, D, L, r[None], open_loop=True)
out = os.path.join(ROOT, "gpurun_out", "nmpc_%s.npz" % tag)
np.savez(out, J1=res.J1, j21=res.j21, Jnu=res.Jnu, status=res.status, qp=res.qp_iters)
print(tag, "status codes", dict(zip(*[a.tolist() for a in np.unique(res.status, return_counts=True)])),
      "sqp iters mean", res.qp_iters.mean())
if len(sys.argv) > 2:
    o = np.load(os.path.join(ROOT, "gpurun_out", "nmpc_%s.npz" % sys.argv[2]))
    for k in ("J1", "j21", "Jnu", "status", "qp"):
        a, b = np.asarray(getattr(res, {"qp": "qp_iters"}.get(k, k))), o[k]
        same = np.array_equal(a, b, equal_nan=True) if a.dtype.kind == "f" else np.array_equal(a, b)
        print("vs %s: %-6s bitwise equal %s" % (sys.argv[2], k, same))
