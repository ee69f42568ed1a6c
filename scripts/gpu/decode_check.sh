#!/bin/bash
# Decode change check: attention / model GPU tests, then greedy decode throughput (B = 1, 2, 8).
#   TAG=x scripts/gpu/decode_check.sh
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-dec}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_model_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -5 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench/bench_generate.py --batches 1,2,8 > "$OUT/generate.jsonl" 2> "$OUT/generate.err" || { tail -20 "$OUT/generate.err"; exit 1; }
cat "$OUT/generate.jsonl"
