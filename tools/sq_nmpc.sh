#!/bin/bash
# SQ issue / instruction-fetch counters of the NMPC kernel over config 5, per libmpct variant
# (one --pmc pass each, kernel-trace only).  usage: bash tools/sq_nmpc.sh NAME... ("-" = libmpct.so)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/sqn; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 100 rocprofv3 -L > $O/avail.txt 2>&1
grep -iE "IFETCH|ICACHE|SQC_" $O/avail.txt | head -20
for v in "$@"; do
  if [ "$v" != "-" ]; then export MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so; else unset MPCT_LIB; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH --output-format csv -d $O/$v -o p -- python3 $R/tools/bench_config5.py --reps 1 > $O/$v.log 2>&1 || { echo "pmc pass $v failed"; tail -5 $O/$v.log; exit 1; }
  python3 - "$O/$v" "$v" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "nmpc_closed_loop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("==", sys.argv[2])
for k, v in sorted(agg.items()):
    print("%-22s sum %.4g over %d dispatches" % (k, sum(v), len(v)))
PY
done
