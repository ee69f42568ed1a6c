#!/bin/bash
# 64-bit GEMM operand extents (no row-chunked LM-head launches): GEMM / model tests, then the
# flagship bench and kernel stats.   scripts/gpu/s11_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-s11}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_bench_scale_gpu.py \
  tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
s=$?; tail -4 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench.$i.json" 2> "$OUT/bench.$i.err" || { tail -20 "$OUT/bench.$i.err"; exit 1; }
  echo "run $i: $(tail -1 "$OUT/bench.$i.json" | cut -c1-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
python scripts/kernel_stats.py "$OUT/prof" --steps 7 > "$OUT/kernel_stats.txt" && head -16 "$OUT/kernel_stats.txt" | cut -c1-160
