#!/bin/bash
# gpt2-xl one-box A/B of extension builds: T128 / W4 weight-gradient microbench at 16k tokens,
# then the B = 16 (+ B = 32) bench, interleaved over ROUNDS.
#   scripts/gpu/xl_so_ab.sh TAG ROUNDS so1 so2 ...   ("tree" = the in-tree build)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
use() { if [ "$1" = tree ]; then unset MINGPT_EXT_SO; else export MINGPT_EXT_SO=$1; fi; }
for so in "$@"; do
  use "$so"; echo "== $so"
  timeout -k 10 200 python bench/bench_wgrad.py --tokens 16384 --D 1600 --variants 1,1,5 || exit 1
done
for r in $(seq 1 "$ROUNDS"); do
  for so in "$@"; do
    use "$so"
    timeout -k 10 300 python bench.py --model gpt2-xl --batch 16 --also-batch 32 --steps 6 --warmup 2 \
      > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['extra']['batch32']['value'])" "$OUT/b.json" "$so" "$r"
  done
done
