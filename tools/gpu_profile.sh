#!/bin/bash
# GPU-box evidence pass: parity tests, the bench line, a rocprofv3 kernel-trace --stats summary
# and separate FETCH_SIZE / WRITE_SIZE counter passes (never combined with other traces).
# Usage (from the repo root on the GPU box):  bash tools/gpu_profile.sh [tag]
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r01}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline)
sha256sum "$R/model-predictive-control-tuning_amd/csrc/libmpct.so" > "$O/lib_sha256.txt"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  (cd "$R" && timeout -k 10 420 python3 -m pytest tests -m gpu -x -q > "$O/pytest_gpu.log" 2>&1) \
    || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
timeout -k 10 420 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- "${BENCH[@]}" \
  > "$O/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o fetch -- "${BENCH[@]}" \
  > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o write -- "${BENCH[@]}" \
  > "$O/write.log" 2>&1
find "$O" -name "*.csv" | sort
