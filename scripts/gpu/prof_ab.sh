#!/bin/bash
# kernel stats of the flagship step under two environments on one box: prof_ab.sh TAG "ENV_A" "ENV_B"
# (e.g. "MINGPT_EXT_SO=build/ab/base/_C.so" "MINGPT_ATTN_BWD_MODE=2")
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
k=0
for E in "$2" "$3"; do
  k=$((k+1))
  ( export $E; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$k" -o run -- \
    python3 bench.py --steps 5 --warmup 2 > "$OUT/p$k.log" 2>&1 ) || { tail -20 "$OUT/p$k.log"; exit 1; }
  echo "== $E"; python scripts/kernel_stats.py "$OUT/p$k" --steps 7 --top 30 > "$OUT/ks$k.txt" && head -14 "$OUT/ks$k.txt"
done
