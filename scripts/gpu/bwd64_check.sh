#!/bin/bash
# hd = 64 attention backward (attn_bwd64_kernel): numerics (fp32 reference + bitwise vs the general
# kernel), model-level dropout gradients, then kernel times against the general kernel on one box.
#   scripts/gpu/bwd64_check.sh TAG [rounds]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-bwd64}; R=${2:-2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for on in 1 0; do  # default (bwd64) and the general kernel it replaces
  MINGPT_ATTN_BWD64=$on timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/attn_tests_$on.log" 2>&1 || { tail -30 "$OUT/attn_tests_$on.log"; exit 1; }
  tail -1 "$OUT/attn_tests_$on.log"
done
timeout -k 10 300 python -u -m pytest tests/test_dropout_grad_gpu.py -x -v -s --timeout 200 --timeout-method thread \
  > "$OUT/dgrad_tests.log" 2>&1 || { tail -30 "$OUT/dgrad_tests.log"; exit 1; }
tail -2 "$OUT/dgrad_tests.log"
# AB_EXTRA: more builds to time beside the tree (e.g. build/ab/prev/_C.so)
bash scripts/gpu/so_attn_stats.sh "$TAG/ab" "$R" tree $AB_EXTRA tree@MINGPT_ATTN_BWD64=0
