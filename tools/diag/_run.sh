#!/bin/bash
# r06c: metric variants (bounds in LDS, merged drop shifts, R_A(jj,jj) by readlane) A/B, three
# interleaved rounds with bitwise dumps; config-3 plans at the fitted overlap
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06c}; O="gpurun_out/$T"; mkdir -p "$O"
AB=()
for rep in 1 2 3; do
  for v in base mrg bnd bm bma ma; do
    AB+=("45 ab_${v}_$rep env MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so QAB_DUMP=$O/ab_$v.npz python3 tools/qab.py h256 4096 8192")
  done
done
bash tools/gpu_steps.sh "$O" "${AB[@]}" \
  "200 plans python3 tools/shard_balance.py --only shell7x5 --plans 0.54:none,0.5:none --out $O/shard_plans.json"
