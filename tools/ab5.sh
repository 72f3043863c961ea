#!/bin/bash
# A/B of config-5 (NMPC) kernel time for libmpct variants: bash tools/ab5.sh lib1.so lib2.so ...
R="${GRAFT_REPO_ROOT:-$(pwd)}"; C=$R/model-predictive-control-tuning_amd/csrc
for lib in "$@"; do
  echo "$lib"
  MPCT_LIB=$C/$lib timeout -k 10 200 python3 $R/tools/bench_config5.py --reps 2 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 || exit 1
done
