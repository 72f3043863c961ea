"""Single-simulation latency of the metric kernel: time subsets of the Shell 3x3 grid chosen by
their measured QP work (lightest / median / heaviest 256, i.e. one workgroup per CU) and the full
grid, with HIP events on the launch stream.  Reports ms and cycles per closed-loop step at the
measured clock (2.4 GHz nominal).  python tools/latency_probe.py [lib]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
    os.environ["MPCT_LIB"] = sys.argv[1]
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import numpy as np
import torch
from mpct.engine import eval_batch, eval_batch_device
from mpct.scenarios import candidate_grid, shell3x3

sc, r, yref = shell3x3(n2_max=30, nu_max=5)
N2, Nu, d, l = candidate_grid(4096)
res = eval_batch(sc, N2, Nu, d, l, r[None])
work = res.qp_iters
order = np.argsort(work, kind="stable")
dev = torch.device("cuda", 0)
tr = torch.from_numpy(r[None].copy()).to(dev)


def timeit(idx, reps=5):
    t = [torch.from_numpy(np.ascontiguousarray(a[idx])).to(dev) for a in (N2, Nu, d, l)]
    C = len(idx)
    out = dict(J1=torch.empty((C, 3), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    st = torch.cuda.current_stream(dev)
    eval_batch_device(sc, *t, tr, out, stream=st)
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        eval_batch_device(sc, *t, tr, out, stream=st)
        e1.record(st)
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


for name, idx in (("lightest 256", order[:256]), ("median 256", order[1920:2176]), ("heaviest 256", order[-256:]),
                  ("one lightest", order[:1]), ("one heaviest", order[-1:]), ("full 4096", np.arange(4096)),
                  ("3072 lightest", order[:3072])):
    ms = timeit(idx)
    print("%-14s %8.3f ms  %7.0f cycles/step @2.4GHz  qp iters/sim mean %.0f max %d" % (
        name, ms, ms * 1e-3 * 2.4e9 / 500, work[idx].mean(), work[idx].max()), flush=True)
