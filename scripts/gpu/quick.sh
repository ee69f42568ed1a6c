#!/bin/bash
# Quick GPU round trip: selected tests (pytest -k expression or files) + flagship bench.
#   scripts/gpu/quick.sh TAG "<pytest args>" ["<bench args>"]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; TARGS=$2; BARGS=${3:---steps 20 --warmup 5}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "$TARGS" ]; then
  timeout -k 10 400 python -u -m pytest $TARGS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
  s=$?; tail -4 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
fi
timeout -k 10 400 python bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
