set -o pipefail
L=$PWD/model-predictive-control-tuning_amd/csrc
CS="1024 4096" bash tools/ab_variants.sh - fd || exit 1
MPCT_LIB=$L/libmpct.so timeout -k 10 200 python3 tools/diag/band_ab.py base || exit 1
MPCT_LIB=$L/libmpct_fd.so timeout -k 10 200 python3 tools/diag/band_ab.py fd base || exit 1
for v in libmpct.so libmpct_fd.so; do
  echo "== config3 $v"; MPCT_LIB=$L/$v timeout -k 10 200 python3 tools/bench_config3.py 2>&1 | tail -1 | cut -c1-200 || exit 1
  echo "== config5 $v"; MPCT_LIB=$L/$v timeout -k 10 200 python3 tools/bench_config5.py --reps 3 | tail -1 | cut -c1-200 || exit 1
done
