set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
L=model-predictive-control-tuning_amd/csrc
MPCT_LIB=$L/libmpct_dbg53.so timeout -k 10 120 python -u tools/diag/band_step_debug.py 63531 $O/c63531.npz > $O/c63531.txt 2>&1 || exit 1
MPCT_LIB=$L/libmpct_dbg80.so timeout -k 10 120 python -u tools/diag/band_step_debug.py 46107 $O/c46107.npz > $O/c46107.txt 2>&1 || exit 1
MPCT_LIB=$L/libmpct_dbg19.so timeout -k 10 120 python -u tools/diag/band_step_debug.py 62507 $O/c62507.npz > $O/c62507.txt 2>&1 || exit 1
