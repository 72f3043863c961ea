set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 60 ./tools/diag/xlane_latency > $O/xlane_latency.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/config3_parity.py --out $O/parity_tol_default.json --dump $O/dump_default.npz > $O/p0.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/config3_parity.py --feas-tol 1e-12 --out $O/parity_tol_1e12.json --dump $O/dump_1e12.npz > $O/p1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/config3_parity.py --feas-tol 1e-13 --out $O/parity_tol_1e13.json > $O/p2.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/scalar_latency.py --out $O/scalar_latency.json > $O/scalar.log 2>&1 || exit 1
cd tools
timeout -k 10 120 python -u tune_shell3x3.py ../$O/s3_last.mat > ../$O/tune_shell3x3_last_eval.log 2>&1 || exit 1
MPCT_FGAM_FROM=returned MPCT_STALE_ROWS=0 timeout -k 10 120 python -u tune_shell3x3.py ../$O/s3_ret.mat > ../$O/tune_shell3x3_returned.log 2>&1 || exit 1
timeout -k 10 300 python -u tune_vandevusse.py ../$O/vdv_spec.mat > ../$O/tune_vandevusse_spec.log 2>&1 || exit 1
MPCT_GAM_SPECULATE=0 timeout -k 10 300 python -u tune_vandevusse.py ../$O/vdv_nospec.mat > ../$O/tune_vandevusse_nospec.log 2>&1 || exit 1
