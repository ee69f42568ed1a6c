#!/bin/bash
# Quick kernel-level A/B of extension builds: attention (B = 128) and the step's epilogue GEMMs,
# each build twice, interleaved.   scripts/gpu/so_quick_ab.sh TAG so1 so2 ...  ("tree" = in-tree)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
use() { if [ "$1" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$1; fi; }
for rep in 1 2; do
  for so in "$@"; do
    use "$so"
    ATTN_B=128 timeout -k 10 200 python bench/attn_ab.py >> "$OUT/attn.jsonl" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    echo "{\"so\": \"$so\"}" >> "$OUT/gemm.jsonl"
    VARIANTS=0 timeout -k 10 200 python bench/dev/gemm_epi_variants.py >> "$OUT/gemm.jsonl" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  done
done
cat "$OUT/attn.jsonl" "$OUT/gemm.jsonl"
