#!/bin/bash
# GEMM change check: GEMM + model numerics tests, W4 epilogue stamps at K = 768, the step's epilogue
# GEMMs, the flagship bench.   scripts/gpu/gemm_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${1:-gemm}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_bench_scale_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
s=$?; tail -3 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
if [ -x build/bin/gemm_epi_stamps ]; then
  for sh in "131072 3072 768" "65536 50304 768"; do timeout -k 10 60 build/bin/gemm_epi_stamps $sh 5 | grep -E "variant|per tile|epilogue:" || exit 1; done
fi
VARIANTS=0 LMHEAD=1 timeout -k 10 200 python bench/dev/gemm_epi_variants.py | tee "$OUT/epi.jsonl" || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json"
