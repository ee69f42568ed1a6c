#!/bin/bash
# Session-9 check: kernels touched (GEMM dbias epilogue, attention dbias / finalize, decode
# attention, GEMV grid), then the flagship bench (B = 128 default) interleaved with the bias
# fusions off, and the decode A/B script.   scripts/gpu/s9_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-s9}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_attention_gpu.py tests/test_model_gpu.py \
  tests/test_bench_scale_gpu.py tests/test_pretrained_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
s=$?; tail -4 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  for v in 1 0; do
    MINGPT_FC_DBIAS_FUSED=$v MINGPT_QKV_DBIAS_FUSED=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 \
      > "$OUT/bench_fused$v.$i.json" 2> "$OUT/bench_fused$v.$i.err" || { tail -20 "$OUT/bench_fused$v.$i.err"; exit 1; }
    echo "fused=$v run $i: $(tail -1 "$OUT/bench_fused$v.$i.json")"
  done
done
for i in 1 2; do
  VARIANT="new.r$i" timeout -k 10 120 python bench/decode_ab.py >> "$OUT/decode.jsonl" 2> "$OUT/decode.err" || { tail -20 "$OUT/decode.err"; exit 1; }
  tail -1 "$OUT/decode.jsonl"
done
