#!/bin/bash
# A/B(/C..) on ONE box (box-to-box clocks differ by a few %): each env config is benched twice,
# interleaved.   scripts/gpu/ab.sh TAG "bench args" "ENV_A" "ENV_B" ...   (use "X=1" as a no-op env)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; BARGS=${2:---steps 20 --warmup 5}; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  k=0
  for E in "$@"; do
    k=$((k+1)); f=$OUT/c${k}_r$rep
    env $E timeout -k 10 300 python bench.py $BARGS > "$f.json" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
    echo "c$k r$rep [$E] $(tail -1 $f.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])")"
  done
done
