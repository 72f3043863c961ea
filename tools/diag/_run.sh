#!/bin/bash
# gpc_small_kernel scheduling on top of max-ilp: pre-RA top-down, post-RA bottom-up (interleaved, bitwise J1 check)
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r05i2"; mkdir -p "$O"; C="$R/model-predictive-control-tuning_amd/csrc"
for rep in 1 2 3; do
  for L in libmpct.so libmpct_td.so libmpct_pbu.so; do
    MPCT_LIB=$C/$L QAB_DUMP=$O/${L%.so}.npz timeout -k 10 120 python3 tools/qab.py 4096 h256 2>&1 | grep kernel || exit 1
  done
done
python3 - "$O" <<'PY'
import numpy as np, sys
a = np.load(sys.argv[1] + "/libmpct.npz")
for v in ("libmpct_td", "libmpct_pbu"):
    b = np.load(sys.argv[1] + "/%s.npz" % v)
    print(v, "J1 bitwise equal:", np.array_equal(a["J1"], b["J1"]), "iters equal:", np.array_equal(a["it"], b["it"]))
PY
