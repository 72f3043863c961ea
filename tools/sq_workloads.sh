#!/bin/bash
# PMC passes over the three other workloads: config 3 (mdband_closed_loop_kernel,
# tools/bench_config3.py), config 5 (nmpc_closed_loop_kernel, tools/bench_config5.py) and config 4
# (config 4: dtc_small_kernel since round 6, tools/bench_dtc_mc.py).  Per workload: two SQ passes
# (issue, waits, FP64 mix, LDS bank conflicts) and separate FETCH_SIZE / WRITE_SIZE passes, each its
# own rocprofv3 run, kernel-trace only, under its own time limit.  Summary (sums over the timed
# dispatches of the workload's kernel family): gpurun_out/sqw/summary.json
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/sqw; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
run() {  # name, command...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/$n/p1 -o p1 -- "$@" > $O/$n.p1.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $O/$n/p2 -o p2 -- "$@" > $O/$n.p2.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$n/f -o f -- "$@" > $O/$n.f.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$n/w -o w -- "$@" > $O/$n.w.log 2>&1
}
run config3 python3 $R/tools/bench_config3.py --reps 1
run config5 python3 $R/tools/bench_config5.py --reps 1 --open-loop 0
run config4 python3 $R/tools/bench_dtc_mc.py
python3 - "$O" "$(sha256sum $R/model-predictive-control-tuning_amd/csrc/libmpct.so | cut -c1-64)" <<'PY'
import collections, csv, glob, json, sys
O, sha = sys.argv[1], sys.argv[2]
fam = {"config3": "mdband_closed_loop", "config5": "nmpc_closed_loop", "config4": "dtc_small_kernel"}  # r06: config 4 runs dtc_small_kernel
rep = {"lib_sha256": sha, "units": "sums over every dispatch of the kernel family in one run of the workload; "
       "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles; FETCH_SIZE / WRITE_SIZE in KiB (hbm_*_bytes corrected)"}
for w, k in fam.items():
    agg = collections.defaultdict(float)
    nd = collections.defaultdict(int)
    for f in glob.glob("%s/%s/*/*counter_collection.csv" % (O, w)):
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                nd[r["Counter_Name"]] += 1
    d = dict(agg)
    if d.get("SQ_WAVE_CYCLES"):
        wc = d["SQ_WAVE_CYCLES"]
        d["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / wc
        d["frac_active_any"] = d.get("SQ_ACTIVE_INST_ANY", 0) / wc
        d["frac_active_valu"] = d.get("SQ_ACTIVE_INST_VALU", 0) / wc
    if d.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_frac"] = d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"]
    d["fp64_flops"] = 64.0 * (2 * d.get("SQ_INSTS_VALU_FMA_F64", 0) + d.get("SQ_INSTS_VALU_ADD_F64", 0)
                              + d.get("SQ_INSTS_VALU_MUL_F64", 0))
    if "FETCH_SIZE" in d:  # gfx950 (MI355X_MICROARCH.md HBM section, tools/pmc_summary.py): read = 2 x FETCH_SIZE
        d["hbm_read_bytes"] = 2.0 * d["FETCH_SIZE"] * 1024.0
    if "WRITE_SIZE" in d:
        d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024.0
    d["dispatches"] = max(nd.values()) if nd else 0
    rep[w] = {"kernel": k, **d}
json.dump(rep, open(O + "/summary.json", "w"), indent=1)
print(json.dumps(rep, indent=1))
PY
