#!/bin/bash
# attention numerics + microbench (B=32 GPT-2 shape and the B=16 one) -> gpurun_out/TAG/
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attn}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -q -x -p no:cacheprovider > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench/bench_attention.py --B 32 > "$OUT/attn_b32.jsonl" 2>&1 || { tail "$OUT/attn_b32.jsonl"; exit 1; }
cat "$OUT/attn_b32.jsonl" | grep -v amdgpu.ids
