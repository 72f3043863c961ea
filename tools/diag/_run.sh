set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
for v in _base _kraw ""; do
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 240 python3 -u tools/config3_ab.py >> $O/config3_ab.jsonl 2>> $O/config3_ab.err || { tail -20 $O/config3_ab.err; exit 1; }
done
cat $O/config3_ab.jsonl
MPCT_LIB=$L/libmpct_bprof.so timeout -k 10 120 python3 -u tools/diag/band_step_debug.py 8015 $O/slow.npz > $O/band_prof_8015.txt 2>&1 || { tail -20 $O/band_prof_8015.txt; exit 1; }
grep -v amdgpu $O/band_prof_8015.txt | head -15
echo diag done
