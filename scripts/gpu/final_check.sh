#!/bin/bash
# End-of-session checkpoint: round_check (GPU suite, bench, kernel stats, LM-head-on-hipBLASLt bench,
# decode), then gpt2-xl at B = 16 and 32 and the gpt-mini hipGraph step.   scripts/gpu/final_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-final}; OUT=gpurun_out/$TAG
bash scripts/gpu/round_check.sh "$TAG" || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
for B in 16 32; do
  timeout -k 10 400 python bench.py --model gpt2-xl --batch $B --steps 6 --warmup 2 > "$OUT/xl_b$B.json" 2> "$OUT/xl_b$B.err" || { tail -20 "$OUT/xl_b$B.err"; exit 1; }
  tail -1 "$OUT/xl_b$B.json"
done
timeout -k 10 300 python bench.py --model gpt-mini --seq 128 --vocab 65 --batch 64 --steps 100 --warmup 20 --graph \
  > "$OUT/mini_graph.json" 2> "$OUT/mini_graph.err" || { tail -20 "$OUT/mini_graph.err"; exit 1; }
tail -1 "$OUT/mini_graph.json"
