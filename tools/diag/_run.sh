#!/bin/bash
# r06aa: the GPU suite on the no-select prologue build (8a6d257b), then config 4 with dtc_small_kernel's prologue
# blocks of 4 (release), 8 and 12 rows, three interleaved bench rounds
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06aa}; O="gpurun_out/$T"; mkdir -p "$O"
C=$R/model-predictive-control-tuning_amd/csrc
AB=("600 pytest python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread")
for rep in 1 2 3; do
  for v in base dh8 dh12; do
    AB+=("120 c4_${v}_$rep env MPCT_LIB=$C/libmpct_$v.so python3 bench.py --workload dtc-mc --steps 5 --warmup 2 --no-cpu-baseline")
  done
done
bash tools/gpu_steps.sh "$O" "${AB[@]}"
