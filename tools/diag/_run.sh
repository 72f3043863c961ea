#!/bin/bash
# r06e: the NMPC kernel's FP64 split (profile build, config 5 grid) and config 5's bench line
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06e}; O="gpurun_out/$T"; mkdir -p "$O"
bash tools/gpu_steps.sh "$O" \
  "300 split python3 tools/nmpc_fp64_split.py 4096 --out $O/nmpc_fp64_split.json" \
  "200 bench5 python3 bench.py --workload vandevusse --no-cpu-baseline"
