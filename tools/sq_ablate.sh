#!/bin/bash
# Instruction counts per simulation step of the metric kernel, by phase: one SQ --pmc pass
# (kernel-trace only) over the 4096-candidate batch (tools/ab.py) per ablation build
# (tools/variant.sh NAME -DMPCT_EXP_NOQP [-DMPCT_EXP_SKIP=bits]); the differences between builds
# attribute VALU / SALU / LDS instructions to the phases.  Usage: bash tools/sq_ablate.sh TAG NAME...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O=$R/gpurun_out/$1; shift; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
L=$R/model-predictive-control-tuning_amd/csrc
for V in "$@"; do
  if [ "$V" = "-" ]; then LIB=$L/libmpct.so; T=base; else LIB=$L/libmpct_$V.so; T=$V; fi
  MPCT_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --output-format csv -d $O/$T -o sq -- python3 $R/tools/ab.py > $O/$T.log 2>&1 || exit 1
done
python3 - "$O" "$@" <<'PY'
import csv, glob, collections, sys
O = sys.argv[1]
for V in sys.argv[2:]:
    T = "base" if V == "-" else V
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob("%s/%s/*counter_collection.csv" % (O, T))[0])):
        if "gpc_closed_loop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
    steps = med["SQ_WAVES"] * 500.0
    f64 = med["SQ_INSTS_VALU_FMA_F64"] + med["SQ_INSTS_VALU_MUL_F64"] + med["SQ_INSTS_VALU_ADD_F64"]
    print("%-12s per sim-step: VALU %6.1f (f64 %5.1f)  SALU %6.1f  LDS %5.1f  wave-cycles/step %7.0f" % (
        T, med["SQ_INSTS_VALU"] / steps, f64 / steps, med["SQ_INSTS_SALU"] / steps, med["SQ_INSTS_LDS"] / steps,
        med["SQ_WAVE_CYCLES"] / steps))
PY
