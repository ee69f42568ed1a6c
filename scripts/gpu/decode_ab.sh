#!/bin/bash
# Decode A/B on one box: GEMV weight-load policy (MINGPT_GEMV_NT) x LM-head grid
# (MINGPT_GEMV_WIDE_GRID), two interleaved rounds.   scripts/gpu/decode_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-dab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for i in 1 2; do
  for nt in 1 0; do
    for gr in 512 1024; do
      VARIANT="nt$nt.grid$gr.r$i" MINGPT_GEMV_NT=$nt MINGPT_GEMV_WIDE_GRID=$gr timeout -k 10 120 \
        python bench/decode_ab.py >> "$OUT/decode_ab.jsonl" 2> "$OUT/decode_ab.err" || { tail -20 "$OUT/decode_ab.err"; exit 1; }
      tail -1 "$OUT/decode_ab.jsonl"
    done
  done
done
