# order_keys_gpc duration per ablation build (MPCT_KEY_SKIP): one kernel-trace pass each
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
for v in - "$@"; do
  if [ "$v" != "-" ]; then export MPCT_LIB=$R/model-predictive-control-tuning_amd/csrc/libmpct_$v.so; else unset MPCT_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ka_$v -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ka_$v.log 2>&1 || exit 1
  python3 - "$R/gpurun_out/ka_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "order_keys" in r["Name"] or "gpc_closed_loop" in r["Name"]:
        print("%-5s %-40s avg %9.1f us" % (sys.argv[2], r["Name"][:40], float(r["AverageNs"]) / 1e3))
PY
done
