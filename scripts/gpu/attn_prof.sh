#!/bin/bash
# attention kernels under rocprofv3 --kernel-trace --stats (B=32 GPT-2 shape)
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attnprof}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/bench_attention.py --B 32 > "$OUT/log" 2>&1 || { tail -20 "$OUT/log"; exit 1; }
grep -v amdgpu.ids "$OUT/log"
python scripts/kernel_stats.py "$OUT/prof" --top 12
