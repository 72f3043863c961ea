#!/bin/bash
# GPU-box A/B of libmpct variant builds (tools/variant.sh): metric-grid parity against the C port
# and kernel time at several batch sizes.  Usage: bash tools/ab_variants.sh NAME... ("-" = libmpct.so)
set -eo pipefail
L=$PWD/model-predictive-control-tuning_amd/csrc
for V in "$@"; do
  if [ "$V" = "-" ]; then LIB=$L/libmpct.so; else LIB=$L/libmpct_$V.so; fi
  echo "== $V"
  MPCT_LIB=$LIB timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -s -k metric_instance_full_grid \
    --timeout 150 --timeout-method thread 2>&1 | grep -E "J1 max rel|passed|failed"
  MPCT_LIB=$LIB timeout -k 10 120 python3 tools/qab.py ${CS:-1024 4096 8192}
done
