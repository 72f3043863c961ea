"""CPU oracle for the batched closed-loop GPC scoring path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import,
call, link or execute anything in this directory, and only as the checker / baseline.  The
product (``model-predictive-control-tuning_amd/``) never imports it and fails loudly when its
HIP library is missing.

Contents
  matlab.py      restated MATLAB builtins the reference calls (c2d ZOH with fractional delay,
                 step, lsim, roots/poly, round(x,4), conv, de2bi)
  dtcgpc.py      restated DTC-GPC primitives (descompMPC, BA_MIMO, diophantine(MIMO), MatG,
                 deltaUFree, cell2mat2, OptimalPredictor2, filtro_siso, mimofilter) and the
                 config-1 WoodBerry DTC-GPC loop (DTC_GPC_WW.m) in its reference structure
  toolbox_gpc.py the toolbox-equivalent constrained GPC closed loop that replaces
                 closedloop_toolbox.m (A1/A2): Diophantine free response + MatG forced response
                 + a primal active-set QP, the open-loop first-move prediction, and the costs
  objectives.py  GAM_fun J1 (A12), VNS2 objective (A13), PreCon (A15)
  scenarios.py   the Shell 3x3 / WoodBerry scenario definitions transcribed from the drivers
  cgpc.c         the same closed loop restated in plain C (the timed CPU baseline, "port")

Pinning status:
  * c2d / descompMPC / scaling / bounds: pinned by the reference's committed MAT files
    (tests/golden/tuning_parameters_mat.json, decoded by tests/golden/make_mat_fixtures.py).
  * per-candidate closed-loop trajectories and costs against MATLAB's MPC Toolbox:
    **parity unpinned** — the reference commits no trajectories or per-candidate costs, and
    neither MATLAB nor the closed-source toolbox exists here.  The oracle is pinned instead by
    the reference's own algebraic identities (Diophantine identity, MatG == E*B forced part,
    KKT optimality of every QP) tested in tests/test_oracle_*.py.
"""
