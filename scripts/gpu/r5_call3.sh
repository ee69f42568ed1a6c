#!/bin/bash
# Round 5, call 3: kernel table of the current tree (B = 128), decode policy A/B, gpt2-xl points.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r5c3; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --also-batch 0 > "$OUT/prof_bench.log" 2>&1 || { tail -20 "$OUT/prof_bench.log"; exit 1; }
python scripts/kernel_stats.py "$OUT/prof" --steps 7 > "$OUT/kernel_stats.txt" && head -40 "$OUT/kernel_stats.txt"
bash scripts/gpu/decode_ab.sh r5c3dec || exit $?
for B in 16 32; do
  timeout -k 10 400 python bench.py --model gpt2-xl --batch $B --steps 6 --warmup 2 --also-batch 0 > "$OUT/xl_b$B.json" 2> "$OUT/xl_b$B.err" || { tail -20 "$OUT/xl_b$B.err"; exit 1; }
  grep '^{' "$OUT/xl_b$B.json" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('xl B=$B', j['value'], j['ms_per_step'])"
done
