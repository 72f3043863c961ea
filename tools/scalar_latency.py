"""Latency of the scalar drop-in: the unchanged callers (GAM_fun.m:81,
VNS2.m:153) reach the engine through matlab/closedloop_toolbox.m one candidate per call, with the
scenario sized 127 / 15 the way that wrapper sizes it (:18), open-loop leg and trajectories on
(:25).  Measured on Shell 3x3 (nit = 500) through the same host entry the MEX calls
(mpct_eval_batch), C = 1 (GAM_fun.m:81) and the square VNS call (VNS2.m:148-165, my simulations,
one reference set each), at the committed tuning (N = 24, Nu = 6) and at the metric horizon.

Breakdown per call: the whole host call (H2D of candidates and signals, launches, D2H of costs and
four trajectories, the stream wait); the same call with the signals unchanged (their upload is
skipped, DevCtx::sig_host); the kernels alone (eval_batch_device, inputs resident, HIP events);
and the host-side remainder.  Usage: python tools/scalar_latency.py [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import torch  # noqa: E402

from mpct.engine import eval_batch, eval_batch_device  # noqa: E402
from mpct.scenarios import SHELL3_TUNED, shell3x3, vns_step_refs  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    sc, r, yref = shell3x3(n2_max=127, nu_max=15)      # matlab/closedloop_toolbox.m:18 sizing
    d = np.array(SHELL3_TUNED["delta"])
    l = np.array(SHELL3_TUNED["lam"])
    refs_vns = vns_step_refs(3, 500)
    dev = torch.device("cuda:0")
    rep = {"scenario": "Shell 3x3, n2_max = 127, nu_max = 15, nit = 500, open loop + trajectories", "cases": []}
    for (N2, Nu) in ((24, 6), (30, 5)):
        for name, refs in (("GAM_fun call (C = 1, nref = 1)", r[None]), ("VNS2 square call (C = 1, nref = 3)", refs_vns)):
            args = (np.array([N2], np.int32), np.array([Nu], np.int32), d[None], l[None])
            call = lambda rr=refs: eval_batch(sc, *args, rr, open_loop=True, want_traj=True)  # noqa: E731
            call()
            same = med(call, a.reps)
            # signals that change every call (the upload is not skipped)
            k = [0]

            def fresh(rr=refs):
                k[0] += 1
                x = rr.copy()
                x[..., -1] += 1e-300 * k[0]
                return eval_batch(sc, *args, x, open_loop=True, want_traj=True)

            changed = med(fresh, a.reps)
            # kernels alone: the same launch(es) with device-resident inputs, HIP events
            t = {kk: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for kk, x in
                 dict(N2=args[0], Nu=args[1], d=args[2], l=args[3], r=refs).items()}
            S = refs.shape[0]
            out = dict(J1=torch.empty((S, 3), dtype=torch.float64, device=dev),
                       j21=torch.empty((S, 3), dtype=torch.float64, device=dev),
                       j22=torch.empty((S, 3), dtype=torch.float64, device=dev),
                       Jnu=torch.empty((S, 3), dtype=torch.float64, device=dev),
                       status=torch.empty(S, dtype=torch.int32, device=dev),
                       qp_iters=torch.empty(S, dtype=torch.int64, device=dev))
            s = torch.cuda.current_stream()
            ks = []
            for _ in range(a.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                eval_batch_device(sc, t["N2"], t["Nu"], t["d"], t["l"], t["r"], out, open_loop=True, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                ks.append(e0.elapsed_time(e1))
            kern = float(np.median(ks[1:]))
            res = call()
            rep["cases"].append(dict(call=name, N2=N2, Nu=Nu, host_call_ms=same, host_call_new_signals_ms=changed,
                                     kernel_ms=kern, host_overhead_ms=same - kern,
                                     signal_upload_saved_ms=changed - same, status=res.status.tolist(),
                                     qp_iters=res.qp_iters.tolist()))
            print(json.dumps(rep["cases"][-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
