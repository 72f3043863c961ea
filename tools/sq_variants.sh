#!/bin/bash
# SQ instruction counters for each libmpct_pv_*.so variant (phase ablations)
R="${GRAFT_REPO_ROOT:-$(pwd)}"; C=$R/model-predictive-control-tuning_amd/csrc; O=$R/gpurun_out/sqv; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for lib in $C/libmpct_pv_*.so; do
  n=$(basename $lib .so)
  MPCT_LIB=$lib timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/$n -o $n -- python3 $R/tools/ab.py > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
O=os.environ.get("GRAFT_REPO_ROOT", os.getcwd()) + "/gpurun_out/sqv"
for d in sorted(glob.glob(O + "/libmpct_pv_*/")):
    f = glob.glob(d + "*counter_collection.csv")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gpc_closed_loop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: sorted(v)[len(v)//2] for k, v in agg.items()}
    W = med["SQ_WAVES"] * 500
    print("%-28s VALU/step %6.0f SALU/step %5.0f LDS/step %5.0f F64FMA/step %4.0f  wave-cyc/step %6.0f" % (
        os.path.basename(d[:-1]), med["SQ_INSTS_VALU"]/W, med["SQ_INSTS_SALU"]/W, med["SQ_INSTS_LDS"]/W,
        med["SQ_INSTS_VALU_FMA_F64"]/W, 4*med["SQ_WAVE_CYCLES"]/W))
PY
