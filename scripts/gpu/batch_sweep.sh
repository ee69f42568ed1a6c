#!/bin/bash
# flagship step at several per-GPU batches: scripts/gpu/batch_sweep.sh TAG B1 B2 ...
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for B in "$@"; do
  timeout -k 10 300 python bench.py --batch "$B" --steps 10 --warmup 3 > "$OUT/b$B.json" 2> "$OUT/b$B.err" || { tail -5 "$OUT/b$B.err"; exit 1; }
  echo "B=$B $(tail -1 "$OUT/b$B.json")"
done
