#!/bin/bash
# One GPU round trip (run through gpurun): GPU test suite, flagship bench, rocprofv3 kernel stats.
#   scripts/gpu/check.sh TAG [--no-tests] [--no-prof] [--bench-args "..."]
# Writes gpurun_out/TAG/{tests.log,bench.json,kernel_stats.txt}.  Each GPU step has its own time
# limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-check}; shift || true
TESTS=1; PROF=1; BARGS="--steps 10 --warmup 3"
while [ $# -gt 0 ]; do
  case "$1" in
    --no-tests) TESTS=0 ;;
    --no-prof) PROF=0 ;;
    --bench-args) BARGS="$2"; shift ;;
  esac
  shift
done
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
fi
timeout -k 10 400 python bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ $PROF = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --also-batch 0 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
  python scripts/kernel_stats.py "$OUT/prof" --steps 7 > "$OUT/kernel_stats.txt" && head -25 "$OUT/kernel_stats.txt"
fi
