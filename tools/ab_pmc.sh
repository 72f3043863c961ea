# GPU-box A/B of libmpct.so against one variant build (tools/variant.sh): metric parity and kernel
# time at 1024 / 4096 / 8192 candidates (tools/ab_variants.sh), then one WRITE_SIZE and one
# FETCH_SIZE pass of the 4096-candidate batch (tools/ab.py) per build -> gpurun_out/TAG/.
# Usage (repo root): bash tools/ab_pmc.sh VARIANT TAG
set -o pipefail
V=$1; O=$PWD/gpurun_out/$2; mkdir -p $O
R=$PWD; L=$R/model-predictive-control-tuning_amd/csrc
CS="1024 4096 8192" timeout -k 10 500 bash tools/ab_variants.sh - $V - $V > $O/ab_$V.txt 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
for B in - $V; do
  if [ "$B" = "-" ]; then LIB=$L/libmpct.so; T=base; else LIB=$L/libmpct_$B.so; T=$B; fi
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$T -o w -- python3 $R/tools/ab.py > $O/w_$T.log 2>&1 || exit 1
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$T -o f -- python3 $R/tools/ab.py > $O/f_$T.log 2>&1 || exit 1
done
