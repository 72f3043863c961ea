set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
MPCT_LIB=$L/libmpct_pol0.so timeout -k 10 240 python3 -u tools/config3_ab.py >> $O/config3_ab.jsonl 2>> $O/config3_ab.err || { tail -20 $O/config3_ab.err; exit 1; }
cat $O/config3_ab.jsonl
cd tools && timeout -k 10 1000 python3 -u tune_vandevusse.py > ../$O/tune_vandevusse.log 2>&1 || { tail -20 ../$O/tune_vandevusse.log; exit 1; }
tail -4 ../$O/tune_vandevusse.log
echo diag done
