#!/bin/bash
# The other BASELINE training configs on one GPU (gpt2-xl B=16, chargpt gpt-mini B=64) + a
# rocprofv3 step breakdown of gpt2-xl.   scripts/gpu/configs.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-cfgs}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model gpt2-xl --batch 16 --steps 6 --warmup 2 > "$OUT/xl.json" 2> "$OUT/xl.err" || { tail -20 "$OUT/xl.err"; exit 1; }
tail -1 "$OUT/xl.json"
timeout -k 10 300 python bench.py --model gpt-mini --seq 128 --vocab 65 --batch 64 --steps 100 --warmup 20 > "$OUT/mini.json" 2> "$OUT/mini.err" || { tail -20 "$OUT/mini.err"; exit 1; }
tail -1 "$OUT/mini.json"
bash scripts/gpu/prof.sh "$TAG/xlprof" X=1 "--model gpt2-xl --batch 16 --steps 3 --warmup 2"
