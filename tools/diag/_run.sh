#!/bin/bash
# key with the Gram tables and register jump vectors: GPU parity tests, metric timing, bench, key time
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r05v"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 200 python3 tools/qab.py 4096 h256 > "$O/qab.txt" 2>&1 || exit 1; cat "$O/qab.txt"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || exit 1; cut -c1-330 "$O/bench.json"
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$O/kt.log" 2>&1 || exit 1
python3 - "$O/kt" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:40], r["Calls"], r["AverageNs"])
PY
