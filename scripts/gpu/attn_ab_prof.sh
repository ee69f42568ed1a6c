#!/bin/bash
# per-kernel times of bench/attn_ab.py for two environments: attn_ab_prof.sh TAG "ENV_A" "ENV_B"
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
k=0
for E in "$2" "$3"; do
  k=$((k+1))
  ( export $E; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p$k" -o run -- \
    python3 bench/attn_ab.py > "$OUT/p$k.log" 2>&1 ) || { tail -20 "$OUT/p$k.log"; exit 1; }
  echo "== $E"; cat "$OUT/p$k.log"; python scripts/kernel_stats.py "$OUT/p$k" --steps 1 --top 8 | cut -c1-120
done
