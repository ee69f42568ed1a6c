#!/bin/bash
# Weight-gradient side stream everywhere (MINGPT_WGRAD_STREAM=1, compute stream then at high
# priority) vs the default auto policy: gpt2-xl B = 32 and GPT-2 B = 128, interleaved on one box.
#   scripts/gpu/stream_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-sab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for cfg in X=0 MINGPT_WGRAD_STREAM=1; do
    env $cfg timeout -k 10 300 python bench.py --model gpt2-xl --batch 32 --also-batch 0 --steps 5 --warmup 2 \
      > "$OUT/xl32_${cfg}_$r.json" 2> "$OUT/xl32_${cfg}_$r.err" || { tail -20 "$OUT/xl32_${cfg}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('xl32', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
      "$OUT/xl32_${cfg}_$r.json" "$cfg" "$r"
    env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/gpt2_${cfg}_$r.json" 2> "$OUT/gpt2_${cfg}_$r.err" \
      || { tail -20 "$OUT/gpt2_${cfg}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gpt2', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['extra'].get('batch64', {}).get('value'))" \
      "$OUT/gpt2_${cfg}_$r.json" "$cfg" "$r"
  done
done
