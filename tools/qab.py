"""Kernel time of the Shell 3x3 metric batch at several batch sizes (HIP events, median of 5) for
the library in MPCT_LIB (default libmpct.so; variant builds: tools/variant.sh).
Usage: python tools/qab.py [C ...]   (hC: the C candidates of the 4096 grid with the most QP work;
QAB_DUMP=f.npz saves the 4096 batch's J1 and QP iterations for a bitwise comparison of builds)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mpct.engine import eval_batch_device, kernel_instance  # noqa: E402
from mpct.scenarios import candidate_grid, shell3x3  # noqa: E402

sc, r, yref = shell3x3()
dev = torch.device("cuda", 0)
tag = "%s %s" % (os.path.basename(os.environ.get("MPCT_LIB", "libmpct.so")), kernel_instance(sc))
for arg in sys.argv[1:] or ["1024", "4096", "8192"]:
    heavy = arg.startswith("h")
    C = int(arg.lstrip("h"))
    N2, Nu, d, l = candidate_grid(4096 if heavy else C)
    if heavy:  # a first pass measures each candidate's QP iterations
        tt = [torch.from_numpy(a.copy()).to(dev) for a in (N2, Nu, d, l, r[None])]
        o = dict(J1=torch.empty((4096, 3), dtype=torch.float64, device=dev),
                 status=torch.empty(4096, dtype=torch.int32, device=dev),
                 qp_iters=torch.empty(4096, dtype=torch.int64, device=dev))
        eval_batch_device(sc, *tt, o)
        sel = np.argsort(-o["qp_iters"].cpu().numpy(), kind="stable")[:C]
        N2, Nu, d, l = N2[sel], Nu[sel], d[sel], l[sel]
    t = [torch.from_numpy(a.copy()).to(dev) for a in (N2, Nu, d, l, r[None])]
    out = dict(J1=torch.empty((C, 3), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    for _ in range(2):
        eval_batch_device(sc, *t, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eval_batch_device(sc, *t, out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    if os.environ.get("QAB_DUMP") and arg == "4096":  # bitwise A/B of variant builds
        np.savez(os.environ["QAB_DUMP"], J1=out["J1"].cpu().numpy(), it=out["qp_iters"].cpu().numpy())
    print("%s C=%6s kernel ms: median %.3f min %.3f  (%.0f sims/s) status nz %d" % (
        tag, arg, np.median(ts), min(ts), C / np.median(ts) * 1e3, int((out["status"] != 0).sum())), flush=True)
