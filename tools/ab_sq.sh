#!/bin/bash
# GPU-box A/B of variant builds (tools/variant.sh) with one SQ pass each: metric parity and kernel
# time (tools/ab_variants.sh, CS batch sizes; hC = the C heaviest candidates), then the LDS bank
# conflict / instruction-mix counters of the 4096-candidate batch (tools/ab.py) -> gpurun_out/TAG/.
# Usage (repo root): CS="4096 h256" bash tools/ab_sq.sh TAG VARIANT...   ("-" = libmpct.so)
set -o pipefail
O=$PWD/gpurun_out/$1; shift; mkdir -p $O
R=$PWD; L=$R/model-predictive-control-tuning_amd/csrc
timeout -k 10 600 bash tools/ab_variants.sh "$@" "$@" > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
export TMPDIR=/tmp
cd /tmp
for B in "$@"; do
  if [ "$B" = "-" ]; then LIB=$L/libmpct.so; T=base; else LIB=$L/libmpct_$B.so; T=$B; fi
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/sq_$T -o sq \
    -- python3 $R/tools/ab.py > $O/sq_$T.log 2>&1 || exit 1
done
python3 $R/tools/pmc_kernels.py $O/sq.json $O/sq_*/ || true
