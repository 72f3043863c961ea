set -o pipefail
O=$PWD/gpurun_out/r03f; mkdir -p $O
R=$PWD; L=$R/model-predictive-control-tuning_amd/csrc
CS="1024 4096 8192" timeout -k 10 500 bash tools/ab_variants.sh - w2 - w2 > $O/ab_w2.txt 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
for V in - nostage; do
  if [ "$V" = "-" ]; then LIB=$L/libmpct.so; T=stage; else LIB=$L/libmpct_$V.so; T=$V; fi
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$T -o w -- python3 $R/tools/ab.py > $O/w_$T.log 2>&1 || exit 1
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$T -o f -- python3 $R/tools/ab.py > $O/f_$T.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/clk -o clk -- python3 $R/tools/qab.py 256 1024 4096 > $O/clk.log 2>&1 || exit 1
