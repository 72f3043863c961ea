#!/bin/bash
# rocprofv3 kernel-trace summaries of the config-3 (mdband) and config-5 (nmpc) kernels.
# Usage (repo root on the GPU box): bash tools/gpu_profile_configs.sh [tag]
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-cfg}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c3" -o c3 -- \
  python3 "$R/tools/bench_config3.py" --reps 1 > "$O/c3.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5" -o c5 -- \
  python3 "$R/tools/bench_config5.py" --reps 1 > "$O/c5.log" 2>&1
find "$O" -name "*kernel_stats.csv" | sort
