#!/bin/bash
# scatter unpermute (no invert_perm launch) vs the same without result staging: parity + step time
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r05w"; mkdir -p "$O"
C="$R/model-predictive-control-tuning_amd/csrc"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_c_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2; do
  for L in libmpct.so libmpct_nostage.so; do
    MPCT_LIB=$C/$L timeout -k 10 120 python3 tools/qab.py 4096 8192 2>&1 | grep kernel || exit 1
  done
done
