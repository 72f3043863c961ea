set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u tools/shard_balance.py --out $O/shard_balance.json > $O/shard.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
