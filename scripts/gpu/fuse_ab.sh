#!/bin/bash
# Bias-gradient fusion check: the affected GPU tests, then the flagship bench interleaved with the
# fusions switched off (MINGPT_{FC,QKV}_DBIAS_FUSED=0) on the same box.
#   scripts/gpu/fuse_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-fab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_attention_gpu.py tests/test_model_gpu.py \
  tests/test_bench_scale_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
s=$?; tail -4 "$OUT/tests.log"; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  for v in 1 0; do
    MINGPT_FC_DBIAS_FUSED=$v MINGPT_QKV_DBIAS_FUSED=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      > "$OUT/bench_fused$v.$i.json" 2> "$OUT/bench_fused$v.$i.err" || { tail -20 "$OUT/bench_fused$v.$i.err"; exit 1; }
    echo "fused=$v run $i: $(python -c "import json,sys; d=json.loads(open('$OUT/bench_fused$v.$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
