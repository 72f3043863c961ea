set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ktk2 -o kt -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ktk2.log 2>&1 || exit 1
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_dtc.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/okp3.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/okp3.log 2>&1
