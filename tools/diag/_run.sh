set -o pipefail
O=gpurun_out/r04zs; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
for v in _head "" _head ""; do
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 240 python3 -u tools/config3_ab.py >> $O/config3_ab.jsonl 2>> $O/config3_ab.err || { tail -20 $O/config3_ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/config3_ab.jsonl'):
    d=json.loads(l); print(d['lib'], round(d['grid_s'],3), round(d['slowest']['alone_ms'],1), d['F_beyond_1e-6'], d['rank'], d['status_nonzero'])"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_band.py > $O/pytest_band.log 2>&1 || { tail -30 $O/pytest_band.log; exit 1; }
tail -1 $O/pytest_band.log
echo diag done
