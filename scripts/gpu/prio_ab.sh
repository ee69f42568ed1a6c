#!/bin/bash
# gpt2-xl B = 16: weight-gradient side stream vs HIP stream priorities, interleaved on one box.
#   scripts/gpu/prio_ab.sh TAG [rounds]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-prio}; R=${2:-2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for cfg in X=0 MINGPT_WGRAD_PRIORITY=1 MINGPT_COMPUTE_PRIORITY=-1 MINGPT_WGRAD_STREAM=0; do
    env $cfg timeout -k 10 300 python bench.py --model gpt2-xl --batch 16 --also-batch 0 --steps 6 --warmup 2 \
      > "$OUT/${cfg}_$r.json" 2> "$OUT/${cfg}_$r.err" || { tail -20 "$OUT/${cfg}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
      "$OUT/${cfg}_$r.json" "$cfg" "$r"
  done
done
