#!/bin/bash
# SQ issue / stall counters of the metric kernel on the heaviest 256 simulations alone (one wave per
# CU: tools/qab.py h256), where the launch time is one simulation's own latency.  Two PMC passes,
# kernel-trace only (no other trace is combined with --pmc), each under its own time limit.
# SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; WAIT_ANY + WAIT_INST_ANY +
# ACTIVE_INST_ANY ~ WAVE_CYCLES (MI355X_MICROARCH.md).  Output: gpurun_out/sqh/summary.json
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/sqh; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o p1 -- python3 $R/tools/qab.py h256 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o p2 -- python3 $R/tools/qab.py h256 > $O/p2.log 2>&1
python3 - "$O" <<'PY'
import collections, csv, glob, json, sys
O = sys.argv[1]
out = {}
for f in sorted(glob.glob(O + "/*/*counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gpc_small_kernel" in r["Kernel_Name"] and int(r.get("Grid_Size", 0) or 0) == 256 * 64:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sorted(v)[len(v) // 2]
w = out.get("SQ_WAVES") or 256.0
per = {k: v / w for k, v in out.items() if k != "SQ_WAVES"}
rep = {"launch": "gpc_small_kernel, the 256 heaviest simulations of the 4096 grid, one per CU",
       "per_wave_median_over_launches": per}
if "SQ_WAVE_CYCLES" in per:
    wc = per["SQ_WAVE_CYCLES"]
    rep["fractions_of_wave_cycles"] = {k: per[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                       "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                       "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if k in per}
json.dump(rep, open(O + "/summary.json", "w"), indent=1)
print(json.dumps(rep, indent=1))
PY
