#!/bin/bash
# Round checkpoint (round_check.sh) followed by a per-GPU batch sweep of the flagship step and the
# torch-eager self-baseline at the larger batch.   scripts/gpu/round_plus_batch.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-rb}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
bash scripts/gpu/round_check.sh "$TAG" || exit $?
bash scripts/gpu/batch_sweep.sh "$TAG/batch" 64 96 128 || exit $?
timeout -k 10 400 python bench/baseline_torch.py --batch 128 --attn sdpa --steps 5 --warmup 2 \
  > "$OUT/baseline_b128.json" 2> "$OUT/baseline_b128.err" || { tail -5 "$OUT/baseline_b128.err"; exit 1; }
tail -1 "$OUT/baseline_b128.json"
