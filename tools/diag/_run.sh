set -o pipefail
O=gpurun_out/r04za; mkdir -p $O
L=$PWD/model-predictive-control-tuning_amd/csrc
for v in _base ""; do
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 240 python3 -u tools/config3_ab.py >> $O/config3_ab.jsonl 2>> $O/config3_ab.err || { tail -20 $O/config3_ab.err; exit 1; }
  MPCT_LIB=$L/libmpct$v.so timeout -k 10 120 python3 -u tools/nmpc_latency.py 2>&1 | grep "C=1" | head -2 >> $O/nmpc.txt || { tail -5 $O/nmpc.txt; exit 1; }
done
python3 -c "
import json
for l in open('$O/config3_ab.jsonl'):
    d=json.loads(l); print(d['lib'], round(d['grid_s'],3), round(d['slowest']['alone_ms'],1), d['F_beyond_1e-6'], d['rank'], d['status_nonzero'])"
cat $O/nmpc.txt
echo diag done
