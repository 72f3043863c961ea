#!/bin/bash
# r06x: NMPC streamed QR with both output rows in flight (qr2, -DMPCT_NM_QR2) against the release (base,
# 628c0cd4) and the same source without it (ref): config-5 bench, three interleaved rounds, the small-batch
# latency, and the NMPC GPU tests on qr2
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06x}; O="gpurun_out/$T"; mkdir -p "$O"
C=$R/model-predictive-control-tuning_amd/csrc
AB=()
for rep in 1 2 3; do
  for v in base ref qr2; do
    AB+=("120 c5_${v}_$rep env MPCT_LIB=$C/libmpct_$v.so python3 bench.py --workload vandevusse --steps 3 --warmup 1 --no-cpu-baseline")
  done
done
for v in base qr2; do
  AB+=("120 lat_$v env MPCT_LIB=$C/libmpct_$v.so python3 tools/nmpc_latency.py")
done
AB+=("400 nm_qr2 env MPCT_LIB=$C/libmpct_qr2.so python3 -u -m pytest tests/test_nmpc.py -m gpu -x -q --timeout 300 --timeout-method thread")
bash tools/gpu_steps.sh "$O" "${AB[@]}"
