#!/bin/bash
# Comm/compute CU sharing on one GPU (parallel/comm_proxy.py): the proxy's GPU test, then
# bench/comm_proxy.py on GPT-2 B = 128 and gpt2-xl B = 16.   scripts/gpu/comm_proxy.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-proxy}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_dp_gpu.py -k comm_proxy -x -q --timeout 150 --timeout-method thread \
  > "$OUT/test.log" 2>&1 || { tail -30 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
timeout -k 10 400 python -u bench/comm_proxy.py --model gpt2 --batch 128 \
  --configs ${GPT2_CONFIGS:-300:32:32,0:32:32,300:32:8,300:64:32,600:32:32} > "$OUT/gpt2.jsonl" 2> "$OUT/gpt2.err" \
  || { tail -20 "$OUT/gpt2.err"; exit 1; }
cut -c1-400 "$OUT/gpt2.jsonl"
timeout -k 10 400 python -u bench/comm_proxy.py --model gpt2-xl --batch 16 --steps 5 \
  --configs ${XL_CONFIGS:-300:32:32,300:32:128} > "$OUT/xl.jsonl" 2> "$OUT/xl.err" || { tail -20 "$OUT/xl.err"; exit 1; }
cut -c1-400 "$OUT/xl.jsonl"
