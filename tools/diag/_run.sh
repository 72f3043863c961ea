#!/bin/bash
# r06d: the GPU suite with dtc_small_kernel (config 4's cost-only launches), the dtc-mc bench line
# for three occupancy variants of that kernel, interleaved, and the metric bench line
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06d}; O="gpurun_out/$T"; mkdir -p "$O"
AB=()
for rep in 1 2; do
  for v in dw1 dw5 dw6; do
    AB+=("90 dtc_${v}_$rep env MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so python3 bench.py --workload dtc-mc --no-cpu-baseline")
  done
done
bash tools/gpu_steps.sh "$O" \
  "420 pytest python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread" \
  "${AB[@]}" \
  "200 bench python3 bench.py --no-cpu-baseline"
