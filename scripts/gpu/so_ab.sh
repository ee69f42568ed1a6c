#!/bin/bash
# One-box A/B of extension builds: attention microbench (B = 128), the epilogue GEMMs, and the
# flagship bench, alternating builds.   scripts/gpu/so_ab.sh TAG so1 so2 ...  ("tree" = in-tree)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
use() { if [ "$1" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$1; fi; }
for rep in ${ATTN_REPS:-2}; do
  for so in "$@"; do
    use "$so"
    ATTN_B=128 timeout -k 10 200 python bench/attn_ab.py >> "$OUT/attn.jsonl" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
  done
done
cat "$OUT/attn.jsonl"
for so in "$@"; do
  use "$so"
  echo "{\"so\": \"$so\"}" >> "$OUT/gemm.jsonl"
  VARIANTS=0 timeout -k 10 200 python bench/dev/gemm_epi_variants.py >> "$OUT/gemm.jsonl" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
done
cat "$OUT/gemm.jsonl"
for rep in 1 2; do
  for so in "$@"; do
    use "$so"
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_tmp.json" 2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/bench_tmp.json').read().strip().splitlines()[-1]); print(json.dumps({'so': '$so', 'tok_s': d['value'], 'ms': d['ms_per_step'], 'b64': d['extra'].get('batch64', {}).get('value')}))" | tee -a "$OUT/bench.jsonl"
  done
done
