set -o pipefail
O=gpurun_out/r04zp; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
for v in _head "" _head ""; do
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 240 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/b$v.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$v.json')); print('$v', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done

timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_dtc.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 && grep order_keys_gpc $GRAFT_REPO_ROOT/$O/kt/kt_kernel_stats.csv | cut -c1-40,150-260
echo diag done
