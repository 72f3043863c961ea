#!/bin/bash
# workload PMC pass (tools/pmc_workloads.sh), then the four bench lines read back against the committed
# metric PMC / latency model and this pass's workload summary (copied into profiles/ on the box only)
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r05m}; O="$R/gpurun_out/$T"; mkdir -p "$O"
bash tools/pmc_workloads.sh $T > "$O/pmcw.log" 2>&1 || { tail -30 "$O/pmcw.log"; exit 1; }
cp "$O/pmcw/summary.json" profiles/pmc_workloads_latest.json
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
for W in shell7x5 vandevusse dtc-mc; do
  timeout -k 10 300 python3 bench.py --workload $W --cpu-seconds 10 > "$O/bench_$W.json" 2> "$O/bench_$W.err" \
    || { tail -20 "$O/bench_$W.err"; exit 1; }
done
for f in "$O"/bench*.json; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']), round(d['ms_per_step'],3), r.get('traffic'), r.get('fp64_counter_tflops'), r.get('latency_frac'))" "$f"; done
