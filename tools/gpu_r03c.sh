set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
cd tools
timeout -k 10 300 python -u tune_vandevusse.py ../$O/vdv_l3.mat > ../$O/tune_vandevusse_ladder3.log 2>&1 || exit 1
MPCT_GAM_LADDER=6 timeout -k 10 300 python -u tune_vandevusse.py ../$O/vdv_l6.mat > ../$O/tune_vandevusse_ladder6.log 2>&1 || exit 1
MPCT_GAM_SPECULATE=0 timeout -k 10 300 python -u tune_vandevusse.py ../$O/vdv_nospec.mat > ../$O/tune_vandevusse_nospec.log 2>&1 || exit 1
timeout -k 10 120 python -u tune_shell3x3.py ../$O/s3.mat > ../$O/tune_shell3x3.log 2>&1 || exit 1
MPCT_GAM_SPECULATE=0 timeout -k 10 120 python -u tune_shell3x3.py ../$O/s3n.mat > ../$O/tune_shell3x3_nospec.log 2>&1 || exit 1
