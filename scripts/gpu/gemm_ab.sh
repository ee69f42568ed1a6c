#!/bin/bash
# GEMM change check: tests/test_gemm_gpu.py, then weight-gradient timings at gpt2-xl / GPT-2 shapes
# and the two benches, each with ENV_A and ENV_B (e.g. MINGPT_GEMM_STREAMK=0 / =1).
#   scripts/gpu/gemm_ab.sh TAG "ENV_A" "ENV_B"
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-gab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for v in A B; do
  E=$([ $v = A ] && echo "$2" || echo "$3")
  for d in 1600 768; do
    tok=$([ $d = 1600 ] && echo 16384 || echo 131072)
    echo "== $v ($E) D=$d"
    env $E timeout -k 10 200 python bench/bench_wgrad.py --D $d --tokens $tok --variants 0,1,5 > "$OUT/wgrad_${v}_$d.txt" 2>&1 || { tail -20 "$OUT/wgrad_${v}_$d.txt"; exit 1; }
    grep wgrad "$OUT/wgrad_${v}_$d.txt"
  done
done
for v in A B; do
  E=$([ $v = A ] && echo "$2" || echo "$3")
  env $E timeout -k 10 500 python bench.py --model gpt2-xl --batch 16 --also-batch 32 --steps 6 --warmup 2 > "$OUT/xl_$v.json" 2> "$OUT/xl_$v.err" || { tail -20 "$OUT/xl_$v.err"; exit 1; }
  echo "xl $v"; tail -1 "$OUT/xl_$v.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('extra',{}).get('batch32'))"
  env $E timeout -k 10 300 python bench.py --also-batch 0 --steps 10 --warmup 3 > "$OUT/gpt2_$v.json" 2> "$OUT/gpt2_$v.err" || { tail -20 "$OUT/gpt2_$v.err"; exit 1; }
  echo "gpt2 $v"; tail -1 "$OUT/gpt2_$v.json" | cut -c1-160
done
if [ "${EPIV:-0}" = 1 ]; then
  timeout -k 10 300 python bench/dev/gemm_epi_variants.py > "$OUT/epi_variants.txt" 2>&1 || { tail -20 "$OUT/epi_variants.txt"; exit 1; }
  cat "$OUT/epi_variants.txt"
fi
