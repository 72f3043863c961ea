"""Workgroup timeline of the metric launch from the -DMPCT_TIMELINE build (libmpct_tl.so,
tools/variant.sh tl -DMPCT_TIMELINE): per slot the s_memrealtime (100 MHz) start and end, the
XCC / SE / CU / SIMD it ran on, and the simulation.  Answers what sets the 4096-candidate launch
time: the latest finishers' start, duration, QP work and co-residents, and how much longer the
heaviest simulations run beside the rest of the batch than alone.
Usage: python tools/diag/timeline.py [--out FILE.json]"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MPCT_LIB", os.path.join(ROOT, "model-predictive-control-tuning_amd", "csrc", "libmpct_tl.so"))
sys.path[:0] = [os.path.join(ROOT, "model-predictive-control-tuning_amd"), ROOT]
import torch  # noqa: E402

from mpct.engine import eval_batch_device  # noqa: E402
from mpct.scenarios import candidate_grid, shell3x3  # noqa: E402

TL = os.path.join(tempfile.gettempdir(), "mpct_timeline.bin")
os.environ["MPCT_TIMELINE_OUT"] = TL
dev = torch.device("cuda", 0)
sc, r, yref = shell3x3()


def run(sel, reps=3):
    N2, Nu, d, l = (a[sel] for a in candidate_grid(4096))
    C = len(sel)
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (N2, Nu, d, l, r[None])]
    out = dict(J1=torch.empty((C, 3), dtype=torch.float64, device=dev),
               status=torch.empty(C, dtype=torch.int32, device=dev),
               qp_iters=torch.empty(C, dtype=torch.int64, device=dev))
    for _ in range(reps):
        eval_batch_device(sc, *t, out)
    torch.cuda.synchronize()
    a = np.fromfile(TL, dtype=np.uint64).reshape(C, 4)
    t0 = a[:, 0].astype(np.int64)
    t1 = a[:, 1].astype(np.int64)
    base = t0.min()
    hw = (a[:, 2] >> np.uint64(32)).astype(np.int64)
    xcc = (a[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
    return dict(start_us=(t0 - base) / 100.0, end_us=(t1 - base) / 100.0, sim=a[:, 3].astype(np.int64),
                xcc=xcc & 0xf, se=(hw >> 13) & 0x7, cu=(hw >> 8) & 0xf, simd=(hw >> 4) & 0x3,
                qp=out["qp_iters"].cpu().numpy())


def co_resident(T, i):
    """waves that shared slot i's CU (and SIMD) at any time during its life"""
    same_cu = (T["xcc"] == T["xcc"][i]) & (T["se"] == T["se"][i]) & (T["cu"] == T["cu"][i])
    overlap = (T["start_us"] < T["end_us"][i]) & (T["end_us"] > T["start_us"][i])
    m = same_cu & overlap
    m[i] = False
    return int(m.sum()), int((m & (T["simd"] == T["simd"][i])).sum())


def main():
    rep = {}
    full = run(np.arange(4096))
    span = full["end_us"].max()
    dur = full["end_us"] - full["start_us"]
    last = np.argsort(-full["end_us"])[:16]
    rep["launch_span_us"] = float(span)
    rep["first_round_slots"] = int((full["start_us"] < 5.0).sum())
    rep["duration_us_quantiles"] = {q: float(np.quantile(dur, q)) for q in (0.5, 0.9, 0.99, 1.0)}
    rep["latest_finishers"] = [dict(slot=int(i), sim=int(full["sim"][i]), start_us=float(full["start_us"][i]),
                                    dur_us=float(dur[i]), qp_iters=int(full["qp"][full["sim"][i]]),
                                    co_cu_simd=co_resident(full, i)) for i in last]
    print(json.dumps({k: v for k, v in rep.items() if k != "latest_finishers"}, indent=1))
    for e in rep["latest_finishers"]:
        print(e)
    # the 256 heaviest (first slots) alone, one per CU, against their duration in the full launch
    heavy = full["sim"][np.argsort(full["start_us"], kind="stable")[:256]]
    alone = run(heavy)
    d_alone = dict(zip(alone["sim"].tolist(), (alone["end_us"] - alone["start_us"]).tolist()))
    d_full = dict(zip(full["sim"].tolist(), dur.tolist()))
    # alone[] numbers the sims 0..255 of the sub-batch; map back through `heavy`
    ratio = np.array([d_full[int(heavy[s])] / dd for s, dd in d_alone.items()])
    rep["heavy256_alone_span_us"] = float(alone["end_us"].max())
    rep["heavy256_stretch_in_full"] = {q: float(np.quantile(ratio, q)) for q in (0.1, 0.5, 0.9)}
    print("heavy 256 alone span %.0f us; duration in the full launch / alone: p10 %.2f p50 %.2f p90 %.2f" % (
        rep["heavy256_alone_span_us"], *rep["heavy256_stretch_in_full"].values()))
    # time profile: waves resident over the launch
    grid = np.linspace(0, span, 41)
    rep["resident_waves"] = [int(((full["start_us"] <= g) & (full["end_us"] > g)).sum()) for g in grid]
    print("resident waves every %.0f us:" % (span / 40), rep["resident_waves"])
    if "--out" in sys.argv:
        with open(sys.argv[sys.argv.index("--out") + 1], "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
