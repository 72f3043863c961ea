#!/bin/bash
# end-of-round evidence pass: tools/gpu_evidence.sh (GPU suite, smoke, metric bench line, kernel
# trace, FETCH_SIZE / WRITE_SIZE and two SQ passes of the metric), the latency probe, the
# heaviest-256 section profile of the -DMPCT_PROFILE build, the SQ counters of the heaviest 256, and
# every workload's bench line with a kernel trace each
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; T=${1:-r06ab}; O="$R/gpurun_out/$T"; mkdir -p "$O"
bash tools/gpu_evidence.sh $T
timeout -k 10 60 tools/latency_probe > "$O/probe.json"
MPCT_PROF_OUT="$O/prof_heavy256.bin" timeout -k 10 120 python3 tools/kprof.py 256 heavy > "$O/kprof.txt" 2>&1
bash tools/sq_heavy.sh
cp gpurun_out/sqh/summary.json "$O/sq_heavy.json"
bash tools/gpu_bench_all.sh ${T}_all > "$O/bench_all.log" 2>&1
echo all done
