set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 240 python3 -u tools/config3_ab.py > $O/config3_ab.jsonl 2> $O/config3_ab.err || { tail -20 $O/config3_ab.err; exit 1; }
cat $O/config3_ab.jsonl
timeout -k 10 180 python3 -u tools/nmpc_latency.py > $O/nmpc_latency.txt 2>&1 || { tail -20 $O/nmpc_latency.txt; exit 1; }
grep "C=1" $O/nmpc_latency.txt
timeout -k 10 180 python3 -u tools/bench_config5.py > $O/bench_config5.txt 2>&1 || { tail -20 $O/bench_config5.txt; exit 1; }
tail -1 $O/bench_config5.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -u tools/diag/gam_calls.py 60 > $O/gam_calls.txt 2>&1 || { tail -20 $O/gam_calls.txt; exit 1; }
tail -4 $O/gam_calls.txt
echo diag done
