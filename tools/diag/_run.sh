#!/bin/bash
# r06f: the metric QP drop's Givens chain without per-rotation hand-offs (nos), with R_A(jj,jj) by
# readlane (areg), with R_A's row and B's column carried in registers (carry): A/B, three
# interleaved runs with bitwise dumps
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06f}; O="gpurun_out/$T"; mkdir -p "$O"
AB=()
for rep in 1 2 3; do
  for v in base nos areg carry; do
    AB+=("45 ab_${v}_$rep env MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so QAB_DUMP=$O/ab_$v.npz python3 tools/qab.py h256 4096 8192")
  done
done
bash tools/gpu_steps.sh "$O" "${AB[@]}"
