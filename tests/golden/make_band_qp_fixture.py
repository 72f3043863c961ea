"""Writes band_qp_near_dependent.npz: the equilibrated toolbox QP (W, c, A, b) of config-3 grid
candidate 17703 (tools/bench_config3.grid: N2 = 32, Nu = 3, delta = 0) at the step where the
measured disturbance enters, captured from the oracle's own closed loop (oracle/toolbox_band.py).
Run from the repo root:  python tests/golden/make_band_qp_fixture.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]

import oracle.toolbox_band as tb  # noqa: E402
from bench_config3 import grid  # noqa: E402
from oracle.scenarios import shell7x5  # noqa: E402

STEP = 19


def main():
    sc, r, v, yref, fx = shell7x5()
    N2, Nu, D, L = grid(1024)
    k = 17703
    caps = []
    orig = tb.qp_dual_dense

    def spy(W, c, A, b, **kw):
        caps.append((W, c, A, b))
        return orig(W, c, A, b, **kw)

    tb.qp_dual_dense = spy
    try:
        tb.closedloop_band(sc, r[:, :STEP + 1], v[:, :STEP + 1], int(N2[k]), int(Nu[k]), D[k], L[k], STEP + 1,
                           open_loop=False)
    finally:
        tb.qp_dual_dense = orig
    W, c, A, b = caps[STEP]
    np.savez(os.path.join(os.path.dirname(os.path.abspath(__file__)), "band_qp_near_dependent.npz"),
             W=W, c=c, A=A, b=b)
    print("rows", A.shape, "from candidate", k, "step", STEP)


if __name__ == "__main__":
    main()
