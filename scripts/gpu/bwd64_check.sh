#!/bin/bash
# hd = 64 attention backward (attn_bwd64_kernel): numerics (fp32 reference + bitwise vs the general
# kernel), model-level dropout gradients, then kernel times against the general kernel on one box.
#   scripts/gpu/bwd64_check.sh TAG [rounds]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-bwd64}; R=${2:-2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/attn_tests.log" 2>&1 || { tail -30 "$OUT/attn_tests.log"; exit 1; }
tail -2 "$OUT/attn_tests.log"
timeout -k 10 300 python -u -m pytest tests/test_dropout_grad_gpu.py -x -v -s --timeout 200 --timeout-method thread \
  > "$OUT/dgrad_tests.log" 2>&1 || { tail -30 "$OUT/dgrad_tests.log"; exit 1; }
tail -2 "$OUT/dgrad_tests.log"
bash scripts/gpu/so_attn_stats.sh "$TAG/ab" "$R" tree tree@MINGPT_ATTN_BWD64=0
