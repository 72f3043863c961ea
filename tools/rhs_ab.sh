# NMPC variants: config 5 throughput and small-batch latency per libmpct variant (tools/variant.sh)
# usage: bash tools/rhs_ab.sh NAME... ("-" = libmpct.so)
for v in "$@"; do
  if [ "$v" != "-" ]; then export MPCT_LIB=$PWD/model-predictive-control-tuning_amd/csrc/libmpct_$v.so; else unset MPCT_LIB; fi
  echo "== variant $v"
  timeout -k 10 120 python3 tools/bench_config5.py --reps 3 > gpurun_out/c5.json || exit 1
  tail -1 gpurun_out/c5.json | cut -c1-190
  timeout -k 10 120 python3 tools/nmpc_latency.py > gpurun_out/lat.txt || exit 1
  head -2 gpurun_out/lat.txt
done
