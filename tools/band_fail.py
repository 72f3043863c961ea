"""Config-3 failure census: score the 65,536-candidate Shell 7x5 grid, tabulate nonzero status by
(N2, Nu), then re-run a sample of failing candidates singly with trajectories (saved to
gpurun_out/band_fail.npz for an oracle replay on the CPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402,F401

from bench_config3 import grid  # noqa: E402
from mpct.engine import eval_batch  # noqa: E402
from mpct.scenarios import shell7x5  # noqa: E402


def main():
    sc, r, v, yref = shell7x5(n2_max=127, nu_max=15)
    N2, Nu, D, L = grid(1024)
    mq = int(os.environ.get("MAXQP", "0"))
    res = eval_batch(sc, N2, Nu, D, L, r[None], v=v[None], device=0, max_qp_iter=mq)
    st = res.status
    print("nonzero:", int(np.sum(st != 0)), "of", st.size)
    for n2 in np.unique(N2):
        row = []
        for nu in np.unique(Nu):
            m = (N2 == n2) & (Nu == nu)
            row.append("%4d" % int(np.sum(st[m] != 0)))
        print("N2=%3d" % n2, " ".join(row))
    bad = np.flatnonzero(st != 0)
    rng = np.random.default_rng(1)
    pick = np.sort(rng.choice(bad, size=min(8, bad.size), replace=False)) if bad.size else bad
    # smallest-horizon failures first: cheapest oracle replays
    small = bad[np.argsort(N2[bad] * 100 + Nu[bad], kind="stable")][:8]
    pick = np.unique(np.concatenate([pick, small]))
    sub = eval_batch(sc, N2[pick], Nu[pick], D[pick], L[pick], r[None], v=v[None], want_traj=True, device=0, max_qp_iter=mq)
    print("picked", pick.tolist(), "status", sub.status.tolist(), "iters", sub.qp_iters.tolist())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "band_fail.npz"), status=st, iters=res.qp_iters,
                        pick=pick, N2=N2[pick], Nu=Nu[pick], L=L[pick], u=sub.u, y=sub.y, sub_status=sub.status)


if __name__ == "__main__":
    main()
