#!/bin/bash
# Round checkpoint: GPU suite + bench + kernel stats (check.sh), then the decode benchmark.
#   scripts/gpu/round_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-rc}; OUT=gpurun_out/$TAG
bash scripts/gpu/check.sh "$TAG" || exit $?
timeout -k 10 300 python bench/bench_generate.py > "$OUT/generate.jsonl" 2> "$OUT/generate.err" || { tail -20 "$OUT/generate.err"; exit 1; }
cat "$OUT/generate.jsonl"
