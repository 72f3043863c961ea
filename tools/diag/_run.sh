#!/bin/bash
# end-of-round keyed pass: the workload PMC pass and the four bench lines read back against the committed
# metric PMC / latency model (tools/diag/_keyed.sh), the 8-rank config-3 plans on one GPU, and the
# 400-iteration Van de Vusse tuning run
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06ac}; O="$R/gpurun_out/$T"; mkdir -p "$O"
bash tools/diag/_keyed.sh $T
timeout -k 10 400 python3 tools/shard_balance.py --only shell7x5 --plans 0.54:none --out "$O/shard_plans.json" \
  > "$O/shard_plans.log" 2>&1 || { tail -20 "$O/shard_plans.log"; exit 1; }
timeout -k 10 300 python3 tools/tune_vandevusse.py "$O/vdv_tuning.mat" > "$O/tune_vandevusse.log" 2>&1 \
  || { tail -20 "$O/tune_vandevusse.log"; exit 1; }
echo all done
