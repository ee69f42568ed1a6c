#!/bin/bash
# Decode experiments: weight-load cache policy (nt vs default, the ~250 MB of GPT-2 weights vs the
# 256 MB Infinity Cache) and the per-kernel decode table.   scripts/gpu/decode_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-dec}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for nt in 1 0; do
    MINGPT_GEMV_NT=$nt NEW=256 timeout -k 10 200 python bench/decode_timing.py > "$OUT/dec_nt${nt}_r${rep}.jsonl" 2>&1 || { tail "$OUT/dec_nt${nt}_r${rep}.jsonl"; exit 1; }
    echo "nt=$nt rep=$rep: $(grep bfloat16 $OUT/dec_nt${nt}_r${rep}.jsonl | tr '\n' ' ')"
  done
done
NEW=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o d -- python3 bench/decode_timing.py > "$OUT/prof.log" 2>&1 || { tail "$OUT/prof.log"; exit 1; }
python scripts/decode_kernel_table.py "$OUT/prof" | tee "$OUT/decode_table.txt"
