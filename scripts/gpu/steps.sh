#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that FAILS (exit 1: a failed test)
# does not stop the next one, anything worse (a fault, an abort, a time limit, a signal) ends the
# script there.
#   scripts/gpu/steps.sh OUTDIR "SECONDS command..." ["SECONDS command..." ...]
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0; worst=0
for step in "$@"; do
  i=$((i + 1))
  lim=${step%% *}; cmd=${step#* }
  echo "== step $i (limit ${lim}s): $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/step$i.log" 2>&1
  rc=$?
  tail -4 "$OUT/step$i.log"
  echo "== step $i rc=$rc"
  if [ $rc -gt 1 ]; then echo "stopping: step $i rc=$rc"; exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
