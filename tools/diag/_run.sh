set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 180 python3 -u tools/diag/nmpc_order.py > $O/nmpc_order.txt 2>&1 || { tail -20 $O/nmpc_order.txt; exit 1; }
cat $O/nmpc_order.txt
timeout -k 10 180 python3 -u tools/nmpc_latency.py > $O/nmpc_latency.txt 2>&1 || { tail -20 $O/nmpc_latency.txt; exit 1; }
cat $O/nmpc_latency.txt
timeout -k 10 400 python3 -u -m pytest tests/test_nmpc.py tests/test_tuning.py tests/test_gpu_tuning.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_nmpc.log 2>&1 || { tail -40 $O/pytest_nmpc.log; exit 1; }
tail -2 $O/pytest_nmpc.log
timeout -k 10 180 python3 -u tools/bench_config5.py > $O/bench_config5.txt 2>&1 || { tail -20 $O/bench_config5.txt; exit 1; }
tail -5 $O/bench_config5.txt
echo diag done
