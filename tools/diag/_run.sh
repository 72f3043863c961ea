#!/bin/bash
# r06b: the QP-cap fault tests again (band batch: no clean simulation), the config-3 LPT plan sweep
# from the committed cell table, and the metric's heaviest-256 profile with the warm start split
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06b}; O="gpurun_out/$T"; mkdir -p "$O"
bash tools/gpu_steps.sh "$O" \
  "300 pytest python3 -u -m pytest tests/test_qp_caps.py tests/test_not_run.py -m gpu -x -v --timeout 240 --timeout-method thread" \
  "300 plans python3 tools/shard_balance.py --only shell7x5 --plans 1:none,0.4:none,0.3:none,0.5:none,0.4:100,0.4:80 --out $O/shard_plans.json" \
  "120 kprof env MPCT_PROF_OUT=$O/prof_heavy256.bin python3 tools/kprof.py 256 heavy"
