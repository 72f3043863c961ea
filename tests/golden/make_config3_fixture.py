"""Generates tests/golden/config3_cband.npz: config-3 (Shell 7x5 band-mode MPC) costs
scored by the oracle's C restatement (oracle/cband.c, restating oracle/toolbox_band.py, which
restates closedloop_toolbox.m:36-100 for Shell7x5.m:98-196).

  J1_strat  (8192, 7)  per-output J1 (GAM_fun.m:110-111) of the stratified sample: the first 128
                       lambda draws of each of the 64 (N2, Nu) cells (mpct.scenarios.config3_stratified)
  F_full    (65536,)   the Pareto-weighted GAM cost J1 @ SHELL7_W (Shell7x5.m:202) of the whole grid
  st_full   (65536,)   oracle status (0 = every QP solved and feasible)
  it_strat  (8192,)    oracle dual-method iterations of the sample

Inputs: mpct.scenarios.config3_grid (N2 x Nu x 1024 lambda draws, seed 20250307, delta = 0),
r = 0, v = the measured disturbance step, nit = 200, GAM mode (no open-loop leg).
Run:  python tests/golden/make_config3_fixture.py [--threads 8]   (≈15 min on 8 cores).

--warm writes tests/golden/config3_cband_warm.npz instead: the same grid scored by the C
restatement's second, equally valid QP path (each step's dual method warm-started from the previous
step's final active set, cband.c cb_scen.qp_warm; F_full, st_full).  Its distance to the cold
fixture is the C-vs-C floor of the config-3 parity (tools/config3_floor.py)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-tuning_amd")]

from mpct.scenarios import SHELL7_W, config3_grid, config3_stratified  # noqa: E402
from oracle.cband import CBand  # noqa: E402
from oracle.scenarios import shell7x5  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config3_cband.npz")
OUT_WARM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config3_cband_warm.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--warm", action="store_true")
    a = ap.parse_args()
    sc, r, v, yref, fx = shell7x5()
    cb = CBand(sc, 200, yref, warm=a.warm)
    N2, Nu, D, L = config3_grid(1024)
    C = N2.size
    J1 = np.zeros((C, 7))
    st = np.zeros(C, np.int32)
    it = np.zeros(C, np.int64)
    t0 = time.time()
    # heavy cells interleaved with light ones keep the OpenMP chunks even
    order = np.argsort((np.arange(C) * 7919) % C, kind="stable")
    for k in range(0, C, a.chunk):
        idx = order[k:k + a.chunk]
        o = cb.eval(N2[idx], Nu[idx], D[idx], L[idx], r[None], v[None], threads=a.threads)
        J1[idx], st[idx], it[idx] = o["J1"], o["status"], o["qp_iters"]
        print("%d / %d  %.0f s" % (k + idx.size, C, time.time() - t0), flush=True)
    if a.warm:
        np.savez_compressed(OUT_WARM, F_full=J1 @ SHELL7_W, st_full=st.astype(np.int8))
        print("wrote", OUT_WARM, "status != 0:", int(np.sum(st != 0)))
        return
    s = config3_stratified(128)
    np.savez_compressed(OUT, J1_strat=J1[s], it_strat=it[s], F_full=J1 @ SHELL7_W, st_full=st.astype(np.int8))
    print("wrote", OUT, "status != 0:", int(np.sum(st != 0)))


if __name__ == "__main__":
    main()
