set -o pipefail
O=gpurun_out/r04zt; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_dtc.py tests/test_gpu_tuning.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in _head "" _head ""; do
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 240 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/b$v.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$v.json')); print('$v', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done
echo diag done
