#!/bin/bash
# A/B of config-3 (band) kernel time for libmpct variants: bash tools/ab3.sh lib1.so lib2.so ...
R="${GRAFT_REPO_ROOT:-$(pwd)}"; C=$R/model-predictive-control-tuning_amd/csrc
for lib in "$@"; do
  echo -n "$lib: "
  MPCT_LIB=$C/$lib timeout -k 10 200 python3 $R/tools/bench_config3.py --reps 2 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['kernel_ms'],1), d['status_nonzero'])" || exit 1
done
