#!/bin/bash
# A/B kernel time of every csrc/libmpct*.so variant given on the command line
R="${GRAFT_REPO_ROOT:-$(pwd)}"; C=$R/model-predictive-control-tuning_amd/csrc
for lib in "$@"; do
  MPCT_LIB=$C/$lib timeout -k 10 120 python3 $R/tools/ab.py 2>&1 | grep -v amdgpu.ids || exit 1
done
