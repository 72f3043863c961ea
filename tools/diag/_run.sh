#!/bin/bash
# r06i: dtc_small_kernel occupancy x prologue block size (kHB 8 / 4) on config 4 (bench.py --workload
# dtc-mc), two interleaved runs, plus a WRITE_SIZE pass of each build
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06i}; O="$R/gpurun_out/$T"; mkdir -p "$O"
AB=()
for rep in 1 2; do
  for v in w1h8 w5h8 w5h4 w4h4; do
    AB+=("90 dtc_${v}_$rep env MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so python3 bench.py --workload dtc-mc --no-cpu-baseline")
  done
done
bash tools/gpu_steps.sh "$O" "${AB[@]}" || exit 1
export TMPDIR=/tmp; cd /tmp
for v in w1h8 w5h8 w5h4 w4h4; do
  MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o w -- python3 $R/bench.py --workload dtc-mc --steps 1 --warmup 1 --no-cpu-baseline > $O/w_$v.log 2>&1 || exit 1
done
echo done
