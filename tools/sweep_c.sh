#!/bin/bash
# Kernel time vs candidates per launch (wave quantisation / occupancy probe).
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
for c in 256 1024 2048 3072 3584 4096 6144 8192; do
  timeout -k 10 120 python3 bench.py --candidates $c --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print($c, round(d['roofline']['kernel_ms'],3), round(d['value']))" || exit 1
done
