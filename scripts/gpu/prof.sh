#!/bin/bash
# rocprofv3 kernel trace of a short bench run + one-step breakdown.   scripts/gpu/prof.sh TAG "ENV" ["bench args"]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; E=${2:-X=1}; BARGS=${3:---steps 4 --warmup 2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
export $E
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py $BARGS > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
python scripts/step_breakdown.py "$OUT/prof/run_kernel_trace.csv" 45 > "$OUT/step.txt" && head -30 "$OUT/step.txt"
