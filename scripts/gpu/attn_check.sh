#!/bin/bash
# attention numerics + microbench at the bench shape + flagship step:  scripts/gpu/attn_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attn}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 python bench/bench_attention.py --B 64 > "$OUT/attn_bench.log" 2>&1 || { tail "$OUT/attn_bench.log"; exit 1; }
grep '^{' "$OUT/attn_bench.log"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
