#!/bin/bash
# gpt2-xl (BASELINE config #5) on one GPU: bench at B = 16 (+ B = 32 in 'extra') and rocprofv3
# kernel stats of the B = 16 step.   scripts/gpu/xl_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-xl}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --model gpt2-xl --batch 16 --also-batch 32 --steps 6 --warmup 2 > "$OUT/xl.json" 2> "$OUT/xl.err" || { tail -20 "$OUT/xl.err"; exit 1; }
tail -1 "$OUT/xl.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --model gpt2-xl --batch 16 --also-batch 0 --steps 3 --warmup 1 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
python scripts/kernel_stats.py "$OUT/prof" --steps 4 > "$OUT/kernel_stats.txt" && head -32 "$OUT/kernel_stats.txt"
