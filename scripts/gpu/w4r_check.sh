#!/bin/bash
# W4R (forward GEMM with B fragments in registers) check: GEMM / model GPU tests, per-shape GEMM
# times for every tile config (bench/bench_gemm.py at 131k tokens), the epilogue table and the
# step A/B of a W4R-default build against the W4 default.   TAG=x scripts/gpu/w4r_check.sh
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-w4r}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_bench_scale_gpu.py -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python bench/bench_gemm.py --tokens 131072 > "$OUT/gemm.jsonl" 2> "$OUT/gemm.err" || { tail "$OUT/gemm.err"; exit 1; }
tail -2 "$OUT/gemm.jsonl"
TAG=${TAG:-w4r}/ab bash scripts/gpu/so_bench_ab.sh build/ab/w4def/_C.so build/ab/w4rdef/_C.so
