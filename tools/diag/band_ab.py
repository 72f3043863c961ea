"""Config-3 grid J1 / status / QP work with the library in MPCT_LIB -> gpurun_out/band_<tag>.npz, and a
comparison against another tag's file when given (A/B of band-kernel variants).
python tools/diag/band_ab.py TAG [OTHER_TAG]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT, os.path.join(ROOT, "tools")]
import torch  # noqa: F401,E402
from bench_config3 import grid  # noqa: E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.scenarios import shell7x5  # noqa: E402

tag = sys.argv[1]
sc, r, v, yref = shell7x5()
N2, Nu, d, l = grid()
res = eval_batch(sc, N2, Nu, d, l, r[None], v=v[None])
out = os.path.join(ROOT, "gpurun_out", "band_%s.npz" % tag)
np.savez(out, J1=res.J1, status=res.status, qp=res.qp_iters)
print(tag, "status nonzero", int((res.status != 0).sum()), "qp iters mean", res.qp_iters.mean())
if len(sys.argv) > 2:
    o = np.load(os.path.join(ROOT, "gpurun_out", "band_%s.npz" % sys.argv[2]))
    ok = (res.status == 0) & (o["status"] == 0)
    rel = np.max(np.abs(res.J1[ok] - o["J1"][ok]) / np.maximum(np.abs(o["J1"][ok]), 1e-300), axis=1)
    print("vs %s: statuses equal %s, J1 max rel %.2e, > 1e-6: %d of %d, median %.1e" % (
        sys.argv[2], bool(np.array_equal(res.status, o["status"])), rel.max(), int((rel > 1e-6).sum()), ok.sum(),
        np.median(rel)))
