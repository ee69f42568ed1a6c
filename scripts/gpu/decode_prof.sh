#!/bin/bash
# decode kernel trace: per-grid durations of gemv / decode attention  (scripts/gpu/decode_prof.sh TAG)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-dec}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
NEW=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o d -- python3 bench/decode_timing.py > "$OUT/prof.log" 2>&1 || { tail "$OUT/prof.log"; exit 1; }
python scripts/decode_kernel_table.py "$OUT/prof"
