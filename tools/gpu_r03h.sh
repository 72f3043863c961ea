set -o pipefail
O=$PWD/gpurun_out/r03h; mkdir -p $O
R=$PWD; L=$R/model-predictive-control-tuning_amd/csrc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
CS="1024 4096 8192" timeout -k 10 500 bash tools/ab_variants.sh - nostage - nostage > $O/ab_nostage.txt 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
for V in - nostage; do
  if [ "$V" = "-" ]; then LIB=$L/libmpct.so; T=stage; else LIB=$L/libmpct_$V.so; T=$V; fi
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$T -o w -- python3 $R/tools/ab.py > $O/w_$T.log 2>&1 || exit 1
  MPCT_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$T -o f -- python3 $R/tools/ab.py > $O/f_$T.log 2>&1 || exit 1
done
