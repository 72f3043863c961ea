#!/bin/bash
# SQ issue/stall counters of the closed-loop kernel (two PMC passes, kernel-trace only; no
# other traces are combined with --pmc).  Output: gpurun_out/sq/*/..._counter_collection.csv
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/sq; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/ab.py > $O/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o p2 -- python3 $R/tools/ab.py > $O/p2.log 2>&1
python3 - <<'PY'
import csv, glob, collections, os
O=os.environ.get("GRAFT_REPO_ROOT", os.getcwd()) + "/gpurun_out/sq"
for f in sorted(glob.glob(O + "/*/*counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gpc_closed_loop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print("%-26s %.4g (median of %d)" % (k, sorted(v)[len(v) // 2], len(v)))
PY
