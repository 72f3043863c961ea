#!/bin/bash
# HBM traffic and FP64 counters of the three other SURVEY §8d bench lines (traffic
# and fp64_counter_tflops non-null in all four lines).  Each workload is profiled through bench.py
# itself (--steps 1 --warmup 1: exactly two evaluations of the workload's grid), in three separate
# rocprofv3 runs, kernel-trace only, each under its own time limit: FETCH_SIZE, WRITE_SIZE, and the
# FP64 instruction mix.  The summary (profiles/pmc_workloads_latest.json, keyed by this libmpct.so's
# sha256) holds per-evaluation sums over the workload's kernel family; bench.py reads it back.
# Usage (repo root on the GPU box): bash tools/pmc_workloads.sh TAG  -> gpurun_out/TAG/pmcw/
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; T=${1:-pmcw}; O=$R/gpurun_out/$T/pmcw; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
SHA=$(sha256sum $R/model-predictive-control-tuning_amd/csrc/libmpct.so | cut -c1-64)
for W in shell7x5 vandevusse dtc-mc; do
  B=(python3 $R/bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline)
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$W/f -o f -- "${B[@]}" > $O/$W.f.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/$W/w -o w -- "${B[@]}" > $O/$W.w.log 2>&1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
    --output-format csv -d $O/$W/s -o s -- "${B[@]}" > $O/$W.s.log 2>&1
  echo "$W profiled"
done
python3 - "$O" "$SHA" "$T" <<'PY'
import collections, csv, glob, json, sys
O, sha, tag = sys.argv[1], sys.argv[2], sys.argv[3]
fam = {"shell7x5": "mdband_closed_loop", "vandevusse": "nmpc_closed_loop", "dtc-mc": "dtc_small_kernel"}  # r06: config 4 runs dtc_small_kernel
EVALS = 2  # --warmup 1 --steps 1
rep = {"lib_sha256": sha, "tag": tag, "evaluations_profiled": EVALS,
       "units": "per evaluation of the workload's grid (one bench.py step), summed over the kernel family's "
                "dispatches; hbm_read_bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 correction, MI355X_MICROARCH.md "
                "HBM section), hbm_write_bytes = WRITE_SIZE KiB x 1024; fp64_flops = 64 x (2 FMA + ADD + MUL)"}
for w, k in fam.items():
    agg = collections.defaultdict(float)
    nd = collections.defaultdict(int)
    for f in glob.glob("%s/%s/*/*counter_collection.csv" % (O, w)):
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                nd[r["Counter_Name"]] += 1
    d = {c: v / EVALS for c, v in agg.items()}
    e = {"kernel": k, "dispatches_per_evaluation": (max(nd.values()) if nd else 0) / EVALS, "counters": d}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        e["hbm_read_bytes"] = 2.0 * d["FETCH_SIZE"] * 1024.0
        e["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024.0
        e["hbm_bytes_per_evaluation"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
    if "SQ_INSTS_VALU_FMA_F64" in d:
        e["fp64_flops_per_evaluation"] = 64.0 * (2 * d["SQ_INSTS_VALU_FMA_F64"] + d.get("SQ_INSTS_VALU_ADD_F64", 0)
                                                 + d.get("SQ_INSTS_VALU_MUL_F64", 0))
    rep[w] = e
json.dump(rep, open(O + "/summary.json", "w"), indent=1)
print(json.dumps(rep, indent=1))
PY
