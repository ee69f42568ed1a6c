#!/bin/bash
# GEMM numerics + microbench (all tile configs, GPT-2 B=32 shapes) -> gpurun_out/TAG/
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-gemm}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider > "$OUT/tests.log" 2>&1
s=$?; tail -2 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python bench/bench_gemm.py --tokens 32768 > "$OUT/gemm.jsonl" 2>&1 || { tail -30 "$OUT/gemm.jsonl"; exit 1; }
grep -v amdgpu.ids "$OUT/gemm.jsonl" | tail -5
