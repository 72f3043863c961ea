#!/bin/bash
# Run GPU steps one after another on the box, each under its own time limit.  A step that exits
# 0 or 1 (a failed assertion / test) lets the next one run; any other status (a time limit 124 /
# 137, an abort 134, a segfault 139, a GPU fault) ends the script there.
# Usage: bash tools/gpu_steps.sh OUTDIR "SECONDS NAME COMMAND..." ...   (logs: OUTDIR/NAME.log)
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R" || exit 2
O="$1"; shift
mkdir -p "$O"
sha256sum "$R/model-predictive-control-tuning_amd/csrc/libmpct.so" > "$O/lib_sha256.txt"
worst=0
for step in "$@"; do
  read -r secs name cmd <<< "$step"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
