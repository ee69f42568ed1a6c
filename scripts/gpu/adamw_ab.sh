#!/bin/bash
# AdamW step alone (bench/dev/adamw_time.py, gpt2-xl and GPT-2) for several extension builds,
# interleaved.   scripts/gpu/adamw_ab.sh TAG so1 so2 ...   ("tree" = in-tree build)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for so in "$@"; do
    if [ "$so" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$so; fi
    for m in gpt2-xl gpt2; do
      timeout -k 10 200 python bench/dev/adamw_time.py --model $m 2> "$OUT/err_$r.txt" | tee -a "$OUT/adamw.jsonl" || { tail -5 "$OUT/err_$r.txt"; exit 1; }
    done
  done
done
