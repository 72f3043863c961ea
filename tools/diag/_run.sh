#!/bin/bash
# r06m: metric LDS bank variants (A-row rotation, B block swizzle, both) A/B against the release library:
# three interleaved qab rounds with bitwise dumps, one LDS PMC pass each; the metric parity tests on
# the combined build; the NMPC tests on the 40 KB-tier build
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06m}; O="gpurun_out/$T"; mkdir -p "$O"
C=$R/model-predictive-control-tuning_amd/csrc
AB=()
for rep in 1 2 3; do
  for v in base arot bswz ba; do
    AB+=("45 ab_${v}_$rep env MPCT_LIB=$C/libmpct_$v.so QAB_DUMP=$O/ab_$v.npz python3 tools/qab.py h256 4096 8192")
  done
done
for v in base arot bswz ba; do
  AB+=("90 lds_$v export TMPDIR=/tmp; MPCT_LIB=$C/libmpct_$v.so timeout -s KILL 80 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/lds_$v -o p -- python3 tools/qab.py 4096")
done
AB+=("300 par_ba env MPCT_LIB=$C/libmpct_ba.so python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread")
AB+=("300 nm_cap40 env MPCT_LIB=$C/libmpct_cap40.so python3 -u -m pytest tests/test_nmpc.py -m gpu -x -q --timeout 240 --timeout-method thread")
bash tools/gpu_steps.sh "$O" "${AB[@]}"
