#!/bin/bash
# Round checkpoint: GPU suite + bench + kernel stats (check.sh), then the bench with the LM-head
# forward on hipBLASLt (the one library option left) and the decode benchmark.
#   scripts/gpu/round_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-rc}; OUT=gpurun_out/$TAG
bash scripts/gpu/check.sh "$TAG" || exit $?
MINGPT_LMHEAD_BLAS=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 \
  > "$OUT/bench_lmhead_blas.json" 2> "$OUT/bench_lmhead_blas.err" || { tail -20 "$OUT/bench_lmhead_blas.err"; exit 1; }
cat "$OUT/bench_lmhead_blas.json"
timeout -k 10 300 python bench/bench_generate.py > "$OUT/generate.jsonl" 2> "$OUT/generate.err" || { tail -20 "$OUT/generate.err"; exit 1; }
cat "$OUT/generate.jsonl"
