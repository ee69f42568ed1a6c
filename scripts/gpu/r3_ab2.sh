#!/bin/bash
# Round-3 A/B: GEMM + attention GPU tests on the tree build, weight-gradient timings at gpt2-xl
# shapes, attention kernel times for BASE / tree / PK builds, and the gpt2 / gpt2-xl benches on
# BASE vs tree.   scripts/gpu/r3_ab2.sh TAG BASE_SO PK_SO
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; BASE=$2; PK=$3; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_attention_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
timeout -k 10 200 python bench/bench_wgrad.py --D 1600 --tokens 16384 --variants 0,1,5 > "$OUT/wgrad_1600.txt" 2>&1 || { tail -20 "$OUT/wgrad_1600.txt"; exit 1; }
grep wgrad "$OUT/wgrad_1600.txt"
bash scripts/gpu/attn_ab_stats.sh "$TAG/attn" "$BASE" tree "$PK" || exit 1
for v in base tree; do
  if [ $v = base ]; then export MINGPT_EXT_SO=$BASE; else unset MINGPT_EXT_SO; fi
  timeout -k 10 500 python bench.py --model gpt2-xl --batch 16 --also-batch 32 --steps 6 --warmup 2 > "$OUT/xl_$v.json" 2> "$OUT/xl_$v.err" || { tail -20 "$OUT/xl_$v.err"; exit 1; }
  echo "xl $v"; tail -1 "$OUT/xl_$v.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('extra',{}).get('batch32'))"
  timeout -k 10 300 python bench.py --also-batch 0 --steps 10 --warmup 3 > "$OUT/gpt2_$v.json" 2> "$OUT/gpt2_$v.err" || { tail -20 "$OUT/gpt2_$v.err"; exit 1; }
  echo "gpt2 $v"; tail -1 "$OUT/gpt2_$v.json" | cut -c1-160
done
