#!/bin/bash
# One PMC pass (8 SQ counters, kernel-trace only) over the metric launch: LDS bank conflicts,
# LDS-array cycles, instruction mix.  Summary -> gpurun_out/sq_lds/summary.json
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/sq_lds; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/p -o p -- python3 $R/tools/ab.py > $O/p.log 2>&1
python3 - <<'PY'
import csv, glob, collections, json, os
O = os.environ.get("GRAFT_REPO_ROOT", os.getcwd()) + "/gpurun_out/sq_lds"
agg = collections.defaultdict(list)
for f in glob.glob(O + "/p/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "gpc_closed_loop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
med = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
steps = 4096 * 500
out = dict(per_launch=med, dispatches=len(agg.get("SQ_WAVES", [])),
           per_sim_step={k: med[k] / steps for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_FMA_F64") if k in med},
           lds_bank_conflict_share=med.get("SQ_LDS_BANK_CONFLICT", 0) / max(med.get("SQ_LDS_IDX_ACTIVE", 1), 1))
json.dump(out, open(O + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
