#!/bin/bash
# GPU-box check: parity tests, the bench line, the config-3 (Shell 7x5) bench.
# Usage (repo root on the GPU box): bash tools/gpu_check.sh [tag]
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
TAG="${1:-chk}"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
if [ "${CONFIG3:-1}" = "1" ]; then
  timeout -k 10 300 python3 tools/bench_config3.py --out "$O/config3.json" > "$O/config3.log" 2>&1 \
    || { tail -20 "$O/config3.log"; exit 1; }
  tail -2 "$O/config3.log"
fi
if [ "${CONFIG5:-1}" = "1" ]; then
  timeout -k 10 300 python3 tools/bench_config5.py --out "$O/config5.json" > "$O/config5.log" 2>&1 \
    || { tail -20 "$O/config5.log"; exit 1; }
  tail -1 "$O/config5.log"
fi
