"""Statuses and costs of test_dispatch_key_mixed_horizons_and_step_refs's batch for one build (MPCT_LIB): QP
iteration caps under the prologue QR variants.  Usage: python tools/diag/qr_status_ab.py OUT.npz"""
import os, sys
import numpy as np
ROOT = "/root/repo"
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
from mpct.engine import eval_batch
from mpct.scenarios import shell3x3, vns_step_refs
rng = np.random.default_rng(7)
C = 320
N2 = rng.integers(8, 31, size=C).astype(np.int32)
Nu = np.minimum(rng.integers(1, 9, size=C), N2).astype(np.int32)
N2[:4] = (0, 31, 5, 12); Nu[:4] = (3, 2, 7, 8)
d = 10.0 ** rng.uniform(-3, 0, size=(C, 3)); l = 10.0 ** rng.uniform(-4, -1, size=(C, 3))
sc, r, yref = shell3x3(n2_max=30, nu_max=8, nit=150)
out = {}
for k, refs in enumerate((r[None], vns_step_refs(3, 150))):
    res = eval_batch(sc, N2, Nu, d, l, refs)
    st = res.status.reshape(C, -1)
    out["st%d" % k] = st; out["J%d" % k] = res.J1; out["it%d" % k] = res.qp_iters
    print(os.path.basename(os.environ.get("MPCT_LIB", "libmpct.so")), "refs", k, "status counts", {int(u): int((st == u).sum()) for u in np.unique(st)})
np.savez(sys.argv[1], **out)
