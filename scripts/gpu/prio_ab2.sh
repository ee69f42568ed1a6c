#!/bin/bash
# Compute stream at high HIP priority (MINGPT_COMPUTE_PRIORITY=-1) vs the default: GPT-2 B = 128
# (no side stream at 131k tokens), gpt2-xl B = 32, and the comm proxy beside each.
#   scripts/gpu/prio_ab2.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-prio2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  for cfg in X=0 MINGPT_COMPUTE_PRIORITY=-1; do
    env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 3 > "$OUT/gpt2_${cfg}_$r.json" 2> "$OUT/gpt2_${cfg}_$r.err" \
      || { tail -20 "$OUT/gpt2_${cfg}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gpt2', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['extra'].get('batch64', {}).get('value'))" \
      "$OUT/gpt2_${cfg}_$r.json" "$cfg" "$r"
    env $cfg timeout -k 10 300 python bench.py --model gpt2-xl --batch 32 --also-batch 0 --steps 5 --warmup 2 \
      > "$OUT/xl32_${cfg}_$r.json" 2> "$OUT/xl32_${cfg}_$r.err" || { tail -20 "$OUT/xl32_${cfg}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('xl32', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
      "$OUT/xl32_${cfg}_$r.json" "$cfg" "$r"
  done
done
for cfg in X=0 MINGPT_COMPUTE_PRIORITY=-1; do
  env $cfg timeout -k 10 300 python -u bench/comm_proxy.py --model gpt2-xl --batch 16 --steps 5 --configs 300:32:128 \
    > "$OUT/proxy_xl_$cfg.jsonl" 2> "$OUT/proxy_xl_$cfg.err" || { tail -20 "$OUT/proxy_xl_$cfg.err"; exit 1; }
  echo "$cfg"; grep '^{' "$OUT/proxy_xl_$cfg.jsonl" | cut -c1-330
done
