#!/bin/bash
# One-box A/B of extension builds: an optional microbenchmark per build, then bench.py per build
# (two interleaved rounds).   TAG=x MICRO=bench/dev/ln_shapes.py scripts/gpu/so_bench_ab.sh A.so B.so ...
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/${TAG:-sobench}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "$MICRO" ]; then
  for so in "$@"; do
    n=$(basename $(dirname $so))
    echo "== $n"; MINGPT_EXT_SO=$so timeout -k 10 200 python $MICRO 2>/dev/null | tee "$OUT/micro_$n.jsonl" || exit 1
  done
fi
for rep in 1 2; do
  for so in "$@"; do
    n=$(basename $(dirname $so))
    MINGPT_EXT_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/bench_${n}_r$rep.json" 2> "$OUT/bench_${n}_r$rep.err" || { tail "$OUT/bench_${n}_r$rep.err"; exit 1; }
    grep '^{' "$OUT/bench_${n}_r$rep.json" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$n r$rep', j['value'], j['ms_per_step'], j['extra']['batch64']['value'])"
  done
done
