#!/bin/bash
# r06q: NMPC packed layouts on config 5 (bench, three interleaved rounds) and the small-batch latency:
# base (822bf19b), lx (40 KB tier, packed R / R^-1), pra (lx + packed R_A: the release candidate);
# the NMPC, tuning and not-run GPU tests on pra
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06q}; O="gpurun_out/$T"; mkdir -p "$O"
C=$R/model-predictive-control-tuning_amd/csrc
AB=()
for rep in 1 2 3; do
  for v in base lx pra; do
    AB+=("120 c5_${v}_$rep env MPCT_LIB=$C/libmpct_$v.so python3 bench.py --workload vandevusse --steps 3 --warmup 1 --no-cpu-baseline")
  done
done
for v in base lx pra; do
  AB+=("120 lat_$v env MPCT_LIB=$C/libmpct_$v.so python3 tools/nmpc_latency.py")
done
AB+=("500 nm_pra env MPCT_LIB=$C/libmpct_pra.so python3 -u -m pytest tests/test_nmpc.py tests/test_tuning.py tests/test_not_run.py -m gpu -x -q --timeout 300 --timeout-method thread")
bash tools/gpu_steps.sh "$O" "${AB[@]}"
