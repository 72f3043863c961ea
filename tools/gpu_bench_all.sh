#!/bin/bash
# GPU-box evidence pass over every SURVEY §8d workload: the bench line of each (roofline +
# cpu_baseline) and a rocprofv3 --kernel-trace --stats summary of each (separate runs, no PMC).
# Usage (repo root on the GPU box): bash tools/gpu_bench_all.sh [tag]
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-all}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 "$R/bench.py" > "$O/bench_shell3x3.json" 2> "$O/bench_shell3x3.err" || { tail -20 "$O/bench_shell3x3.err"; exit 1; }
cat "$O/bench_shell3x3.json"
for W in shell7x5 vandevusse dtc-mc; do
  timeout -k 10 300 python3 "$R/bench.py" --workload $W --cpu-seconds 10 > "$O/bench_$W.json" 2> "$O/bench_$W.err" \
    || { tail -20 "$O/bench_$W.err"; exit 1; }
  cat "$O/bench_$W.json"
done
for W in shell3x3 shell7x5 vandevusse dtc-mc; do
  S=1; [ "$W" = "shell3x3" ] && S=5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$W" -o kt -- \
    python3 "$R/bench.py" --workload $W --steps $S --warmup 1 --no-cpu-baseline > "$O/kt_$W.log" 2>&1 \
    || { tail -20 "$O/kt_$W.log"; exit 1; }
done
find "$O" -name "*kernel_stats.csv" | sort
