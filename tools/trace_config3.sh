#!/bin/bash
# rocprofv3 kernel trace of one config-3 run: per-dispatch start / duration / LDS of the class launches
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/${1:-c3trace}"; mkdir -p "$O"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O" -o c3 -- \
  python3 "$R/tools/bench_config3.py" --reps 1 > "$O/c3.log" 2>&1
