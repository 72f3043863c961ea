set -o pipefail
timeout -k 10 200 python3 tools/diag/order_key_probe.py work est > gpurun_out/okp2.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_dtc.py -m gpu -x -q --timeout 250 --timeout-method thread >> gpurun_out/okp2.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/okp2.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload dtc-mc --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/okp2.log 2>&1 || exit 1
