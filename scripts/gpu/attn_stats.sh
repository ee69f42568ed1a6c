#!/bin/bash
# Attention kernel stats at the GPT-2 bench shape (B = 128 by default): rocprofv3 kernel trace of
# bench/dev/attn_prof.py, summarised per kernel.   scripts/gpu/attn_stats.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-attn}; OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench/dev/attn_prof.py > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us  total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
