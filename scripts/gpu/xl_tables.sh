#!/bin/bash
# gpt2-xl B = 16 on one GPU: bench and rocprofv3 kernel table with the weight-gradient side stream
# (default "auto": on at 16k tokens) and single-stream (MINGPT_WGRAD_STREAM=0), so the in-step
# inflation of kernels that co-run with the side-stream GEMMs can be read off the pure table.
#   scripts/gpu/xl_tables.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-xlt}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for mode in auto 0; do
  MINGPT_WGRAD_STREAM=$mode timeout -k 10 400 python bench.py --model gpt2-xl --batch 16 --also-batch 0 --steps 6 --warmup 2 \
    > "$OUT/xl_$mode.json" 2> "$OUT/xl_$mode.err" || { tail -20 "$OUT/xl_$mode.err"; exit 1; }
  tail -1 "$OUT/xl_$mode.json" | cut -c1-200
  MINGPT_WGRAD_STREAM=$mode timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$mode" -o run -- \
    python3 bench.py --model gpt2-xl --batch 16 --also-batch 0 --steps 3 --warmup 1 > "$OUT/prof_$mode.log" 2>&1 \
    || { tail -20 "$OUT/prof_$mode.log"; exit 1; }
  python scripts/kernel_stats.py "$OUT/prof_$mode" --steps 4 > "$OUT/kernel_stats_$mode.txt" && head -24 "$OUT/kernel_stats_$mode.txt"
done
