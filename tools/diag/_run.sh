#!/bin/bash
# counting rank (order key sort + ranking): GPU suite, metric timing, bench, kernel list
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r05y3"; mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 200 python3 tools/qab.py 4096 4096 h256 > "$O/qab.txt" 2>&1 || exit 1; cat "$O/qab.txt"
for k in 1 2; do timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$O/bench$k.json" 2> "$O/bench$k.err" || exit 1; cut -c1-330 "$O/bench$k.json"; done
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$O/kt.log" 2>&1 || exit 1
python3 - "$O/kt" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:40], r["Calls"], r["AverageNs"])
PY
